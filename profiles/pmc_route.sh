#!/bin/bash
# PMC passes on the default route kernel (run on the GPU box from the repo root):
#   $1 = output tag under gpurun_out/, $2 = kernel regex (default: route kernels).
# One pass per counter group (SQ issue/wait, FETCH_SIZE, WRITE_SIZE), each its own run.
set -euo pipefail
TAG=${1:-pmc}
RX=${2:-k_route}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu"
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_FLAT \
  --kernel-include-regex "$RX" -d "$OUT/sq" -o run --output-format csv -- $B > "$OUT/sq.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/fetch" -o run --output-format csv -- $B > "$OUT/fetch.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/write" -o run --output-format csv -- $B > "$OUT/write.log" 2>&1
