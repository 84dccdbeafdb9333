#!/bin/bash
# Arc SoA round 2: arc GPU tests, C4-size simulation, 1-rank arc bench, and a
# 2-rank gloo rehearsal of the pipelined ArcRouter on one GPU.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-arc_soa2}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_arc.py -x -q --timeout 300 \
  --timeout-method thread > "$OUT/pytest_arc.log" 2>&1
tail -2 "$OUT/pytest_arc.log"
timeout -k 10 500 python -u benches/bench_arc_sim.py --groups 8 --modes soa \
  --keys-log2 28 --reps 2 > "$OUT/arc_sim_q28.json" 2> "$OUT/arc_sim_q28.err"
python3 -c "
import json
a=json.load(open('$OUT/arc_sim_q28.json'))['arc'][0]
print({k: a[k] for k in a if k != 'route_ms'})"
timeout -k 10 300 python -u bench.py --mode arc --steps 5 --warmup 2 > "$OUT/bench_arc_n1.log" 2>&1
tail -1 "$OUT/bench_arc_n1.log" | cut -c1-400
bash tools/rehearse_arc_n2.sh
cp gpurun_out/arc_n2/bench_arc_n2.log "$OUT/"
