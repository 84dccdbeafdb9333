#!/bin/bash
# Profiling recipe for the per-row kernels (benches/bench_rows.py), run on the GPU
# box from the repo root: kernel trace + --stats, then separate PMC passes (SQ issue
# group, FETCH_SIZE, WRITE_SIZE).  Output under gpurun_out/<tag>/.
set -euo pipefail
TAG=${1:-rows}
RX=${2:-"k_misplaced|k_nsucc|k_ida|k_churn"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
B="python3 $GRAFT_REPO_ROOT/benches/bench_rows.py"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- $B > "$OUT/rows.json" 2> "$OUT/rows.err"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_FLAT \
  --kernel-include-regex "$RX" -d "$OUT/sq" -o run --output-format csv -- $B > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/fetch" -o run --output-format csv -- $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/write" -o run --output-format csv -- $B > "$OUT/write.log" 2>&1
