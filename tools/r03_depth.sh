#!/bin/bash
# Route-table depth A/B (CX_ROUTE_R): headline kernel (bench_route: time, hop
# sum, requests per lookup) and churn -> route-ready (bench_ready) at
# R = 32 (default) / 28 / 26 / 24, alternating passes.
set -eo pipefail
TAG=${1:-r03_depth}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
for pass in a b; do
  for r in 32 28 26 24; do
    CX_ROUTE_R=$r timeout -k 10 200 python3 benches/bench_route.py 10 5 > "$OUT/route_R${r}_$pass.json" 2> "$OUT/route_R${r}_$pass.err"
    CX_ROUTE_R=$r timeout -k 10 200 python3 benches/bench_ready.py 24 4 > "$OUT/ready_R${r}_$pass.json" 2> "$OUT/ready_R${r}_$pass.err"
    python3 -c "
import json
a=json.loads(open('$OUT/route_R${r}_$pass.json').read().strip().splitlines()[-1])
b=json.loads(open('$OUT/ready_R${r}_$pass.json').read().strip().splitlines()[-1])
print('R', $r, '$pass', 'route ms', round(a['ms_min'],4), round(a['ms_median'],4), 'lk/s %.3e' % a['lookups_per_s'], 'hops_sum', a['hops_sum'], 'ok', a['owner_ok'], 'per_lookup', {k: round(v,4) for k,v in a['per_lookup'].items()}, 'ready', [round(x['route_ready_ms'],2) for x in b['reps'][1:]])"
  done
done
echo done
