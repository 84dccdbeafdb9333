#!/bin/bash
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-arc}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u benches/bench_arc_sim.py --groups ${2:-8} > "$OUT/arc_sim.json" 2> "$OUT/arc_sim.err"
python3 -c "
import json
d=json.load(open('$OUT/arc_sim.json'))
print('replicated_ms', d['replicated_route_ms'])
for a in d['arc']: print(a['G'], round(a['per_gpu_compute_ms'],3), round(a['per_gpu_xgmi_ms_model'],3), '%.3g'%a['projected_lookups_per_s_per_gpu'], a['round_max_step_ms'], a['round_max_bucket_ms'])
"
