#!/bin/bash
# Kernel trace of the G = 8 arc simulation (SoA protocol, C4 per-rank batch).
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-arc_trace}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/benches/bench_arc_sim.py --groups 8 --modes soa --keys-log2 28 --reps 1 \
  > "$OUT/sim.json" 2> "$OUT/sim.err"
grep -E "k_arc|k_route_tree" "$OUT/trace/run_kernel_stats.csv" | cut -c1-220
