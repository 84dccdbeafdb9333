#!/bin/bash
# Route-table depth: per-launch cost of R = 28 / 30 vs 32 at 2^24, interleaved in one
# process (benches/bench_depth.py, 16 rounds x 10 launches), two processes for 28.
set -eo pipefail
TAG=${1:-r03_depth_pin}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
summ() {
  python3 -c "
import json
d=json.loads(open('$1').read().strip().splitlines()[-1])
print('$1'.split('/')[-1], 'same', d['identical_results'], d['owner_equals_successor'],
  {R: (round(v['ms_median'],4), round(v['ms_min'],4), round(v['exact_hops'],4), [round(x,2) for x in v['route_ready_ms']]) for R, v in d['route'].items()})"
}
timeout -k 10 300 python3 benches/bench_depth.py 32,28 16 10 > "$OUT/d28_a.json" 2> "$OUT/d28_a.err"
summ "$OUT/d28_a.json"
timeout -k 10 300 python3 benches/bench_depth.py 28,32 16 10 > "$OUT/d28_b.json" 2> "$OUT/d28_b.err"
summ "$OUT/d28_b.json"
timeout -k 10 300 python3 benches/bench_depth.py 32,30 16 10 > "$OUT/d30.json" 2> "$OUT/d30.err"
summ "$OUT/d30.json"
echo done
