#!/bin/bash
# Kernel trace (+ --stats) of the per-row bench: per-kernel durations for
# every config row (C2 successor variants, C3, C5, IDA).
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-rows_trace}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CX_ROWS_NO_CPU=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run \
  --output-format csv -- python3 $GRAFT_REPO_ROOT/benches/bench_rows.py > "$OUT/rows.json" 2> "$OUT/rows.err"
head -30 "$OUT/trace/run_kernel_stats.csv" | cut -c1-180
