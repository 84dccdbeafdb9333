#!/bin/bash
# Arc-layout projection curve at C4's per-rank batch (2^25 lookups per rank):
# G = 1, 2, 4, 8 simulated ranks on one GPU, key-first SoA protocol.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-arc_curve}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
for g in 1 2 4 8; do
  lg=$((25 + $(python3 -c "import math;print(int(math.log2($g)))")))
  timeout -k 10 500 python -u benches/bench_arc_sim.py --groups $g --modes soa --keys-log2 $lg \
    --reps 2 > "$OUT/arc_g$g.json" 2> "$OUT/arc_g$g.err"
  python3 -c "
import json
d=json.load(open('$OUT/arc_g$g.json')); a=d['arc'][0]
print($g, 'replicated_ms_per_2^25', round(d['replicated_route_ms']/$g,3), 'compute', round(a['per_gpu_compute_ms'],3), 'xgmi', round(a['per_gpu_xgmi_ms_model'],3), 'proj %.3g'%a['projected_lookups_per_s_per_gpu'], 'overlap %.3g'%a['projected_lookups_per_s_per_gpu_overlapped'], a.get('equals_replicated'))"
done
