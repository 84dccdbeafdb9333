#!/bin/bash
# Arc exchange: GPU arc tests (incl. the region partition) and the G = 8
# one-GPU projection of the two-pass vs single-pass partition.
set -eo pipefail
TAG=${1:-r03_arc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_arc.py tests/test_gpu_ida.py tests/test_gpu_liveness.py \
  -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_arc.log" 2>&1
tail -2 "$OUT/pytest_arc.log"
timeout -k 10 500 python3 -u benches/bench_arc_sim.py --keys-log2 28 --groups 8 --modes soa,soa_regions,soa_hints \
  --reps 3 > "$OUT/arc_sim_g8.json" 2> "$OUT/arc_sim_g8.err"
tail -1 "$OUT/arc_sim_g8.err" | cut -c1-600
echo done
