#!/bin/bash
# In-process route-table depth A/B (benches/bench_depth.py), interleaved rounds.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03_depth_ab}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
for spec in 32,28 28,32 32,26; do
  timeout -k 10 300 python3 benches/bench_depth.py $spec 10 10 > "$OUT/depth_$spec.json" 2> "$OUT/depth_$spec.err"
  python3 -c "
import json
d=json.loads(open('$OUT/depth_$spec.json').read().strip().splitlines()[-1])
print('$spec', 'same', d['identical_results'], d['owner_equals_successor'])
for R,v in d['route'].items(): print('  R', R, 'ms min/med', round(v['ms_min'],4), round(v['ms_median'],4), 'GiB', v['table_bytes']>>30, 'exact', round(v['exact_hops'],4), 'ready', [round(x,2) for x in v['route_ready_ms']])"
done
echo done
