#!/bin/bash
# Round-3 A/Bs: route-table build variants (CX_CZ_PAIR 0/1 = default / two lanes
# per entry; 2/3 = stores-only / compute-only probes) under a kernel trace;
# route kernel on key-sorted vs input order (+ TCC hit/miss PMC passes);
# request ceiling vs table footprint; C5 key-sharded bench at N = 1 and the
# two-rank gloo rehearsal.  Every GPU step has its own limit; chained by &&.
set -eo pipefail
TAG=${1:-r03_ab1}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 1 2 3; do
  CX_CZ_PAIR=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/cz_$v" -o run \
    --output-format csv -- python3 "$R/benches/bench_czbuild.py" 24 > "$OUT/cz_$v.json" 2> "$OUT/cz_$v.err"
  tail -1 "$OUT/cz_$v.json" | cut -c1-300
done
for o in input keysorted; do
  CX_ORDER=$o timeout -k 10 200 python3 "$R/benches/bench_route.py" 10 3 --footprint > "$OUT/route_$o.json" 2> "$OUT/route_$o.err"
  tail -1 "$OUT/route_$o.json" | cut -c1-400
  CX_ORDER=$o timeout -k 10 200 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum \
    --kernel-include-regex "k_route_tree" -d "$OUT/pmc_tcc_$o" -o run --output-format csv \
    -- python3 "$R/benches/bench_route.py" 2 1 > "$OUT/pmc_tcc_$o.log" 2>&1
done
cd "$R"
timeout -k 10 300 python3 -u benches/bench_c5.py --steps 5 --warmup 2 > "$OUT/c5_n1.json" 2> "$OUT/c5_n1.err"
tail -1 "$OUT/c5_n1.json" | cut -c1-400
CX_DIST_BACKEND=gloo timeout -k 10 400 python3 -u benches/bench_c5.py --gpus 2 --peers-log2 22 \
  --keys-log2 24 --steps 3 --warmup 1 > "$OUT/c5_n2.json" 2> "$OUT/c5_n2.err"
tail -1 "$OUT/c5_n2.json" | cut -c1-400
timeout -k 10 400 python3 -u benches/bench_arc_sim.py --keys-log2 28 --groups 8 --modes soa,soa_regions \
  --reps 2 > "$OUT/arc_sim_g8.json" 2> "$OUT/arc_sim_g8.err"
tail -1 "$OUT/arc_sim_g8.json" | cut -c1-400
echo done
