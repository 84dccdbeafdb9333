#!/bin/bash
# PMC passes (SQ issue/wait group, FETCH_SIZE, WRITE_SIZE -- one run each) for the
# kernels matching $2 while running the python command in $3...
#   bash tools/pmc_kernel.sh <tag> <kernel-regex> <script> [args...]
set -eo pipefail
TAG=$1; RX=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU \
  --kernel-include-regex "$RX" -d "$OUT/pmc_sq" -o run --output-format csv -- python3 "$@" > "$OUT/sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_fetch" -o run --output-format csv -- python3 "$@" > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_write" -o run --output-format csv -- python3 "$@" > "$OUT/write.log" 2>&1
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.json"
cat "$OUT/pmc_summary.json"
