#!/bin/bash
# Same-box A/B: exact hops below the route table inline (a_inline: the hop's
# finger and next-peer loads inside the compute phase) vs one memory round
# (b_round: A_EXACT fetches id(cur), id(cur + 1)), at table depth R = 32 / 28
# / 26 (CX_ROUTE_R), alternating passes; bench_route's hop sums must agree.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03_exact_ab}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
for pass in 1 2; do
  for r in 32 28 26; do
    for lib in a_inline b_round; do
      CX_ROUTE_R=$r CHORDX_LIB=$GRAFT_REPO_ROOT/ab_libs/$lib.so timeout -k 10 240 \
        python3 benches/bench_route.py 10 5 > "$OUT/${lib}_R${r}_$pass.json" 2> "$OUT/${lib}_R${r}_$pass.err"
      python3 -c "
import json
a=json.loads(open('$OUT/${lib}_R${r}_$pass.json').read().strip().splitlines()[-1])
print('$lib', 'R', $r, 'pass', $pass, 'ms', round(a['ms_min'],4), round(a['ms_median'],4), 'hops', a['hops_sum'], a['owner_ok'], 'probe %.3e' % a['probe'])"
    done
  done
done
echo done
