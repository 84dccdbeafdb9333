#!/bin/bash
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-arc}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_arc.py -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -3 "$OUT/pytest.log"
timeout -k 10 600 python -u benches/bench_arc_sim.py --groups 1,2,4,8 > "$OUT/arc_sim.json" 2> "$OUT/arc_sim.err"
python3 -c "
import json,sys
d=json.load(open('$OUT/arc_sim.json'))
print('replicated_ms', d['replicated_route_ms'])
for a in d['arc']: print(a['G'], a.get('mode'), a['rounds'], round(a['per_gpu_compute_ms'],3), round(a['per_gpu_xgmi_ms_model'],3), '%.3g'%a['projected_lookups_per_s_per_gpu'], a['records_in_per_round'], a['route_plane_bytes_per_gpu_max']>>30, 'GiB')
"
