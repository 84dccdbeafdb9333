#!/bin/bash
# Profiling recipe for the route kernels (run on the GPU box from the repo root):
#   1. kernel trace + --stats of the default bench (all kernels),
#   2. separate PMC passes: FETCH_SIZE, WRITE_SIZE (TCC slots do not fit both in one
#      pass) and the SQ issue/wait group, each its own run.
# Output goes under gpurun_out/<tag>/; summaries are copied into profiles/.
set -euo pipefail
TAG=${1:-r01}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
RX="k_route|k_successor|k_fingers|k_nsucc|k_cz_build|k_tree_build"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu > "$OUT/bench_trace.log" 2>&1
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_fetch" -o run --output-format csv -- $B > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_write" -o run --output-format csv -- $B > "$OUT/bench_write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_FLAT \
  --kernel-include-regex "k_route" -d "$OUT/pmc_sq" -o run --output-format csv -- $B \
  > "$OUT/bench_sq.log" 2>&1
