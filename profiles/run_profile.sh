#!/bin/bash
# Profiling recipe for the route kernel (run on the GPU box from the repo root):
#   kernel trace + stats of the default bench, then separate PMC passes for
#   FETCH_SIZE and WRITE_SIZE (TCC slots do not fit both in one pass).
# Output goes under gpurun_out/<tag>/; summaries are copied into profiles/.
set -euo pipefail
TAG=${1:-r01}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu > "$OUT/bench_trace.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "k_route|k_successor|k_fingers|k_nsucc" \
  -d "$OUT/pmc_fetch" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "k_route|k_successor|k_fingers|k_nsucc" \
  -d "$OUT/pmc_write" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu > "$OUT/bench_write.log" 2>&1
