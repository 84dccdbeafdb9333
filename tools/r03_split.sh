#!/bin/bash
# Root-centric build: LDS split (21 KB/block) at 4 / 5 / 6 waves per SIMD vs
# the default (37 KB/block, 4 blocks per CU), alternating passes; table hash
# must not change.
set -eo pipefail
TAG=${1:-r03_split}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
    --output-format csv -- python3 "$R/benches/bench_czbuild.py" 24 0 > "$OUT/$name.json" 2> "$OUT/$name.err"
  python3 -c "
import csv,json
d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
k=[round(float(r['AverageNs'])/1e6,2) for r in csv.DictReader(open('$OUT/$name/run_kernel_stats.csv')) if 'cz_build' in r['Name']]
print('$name', 'kernel_ms', k, 'hash', d['route_table_hash'], 'route_ok', d.get('route_ok'))"
}
for pass in a b; do
  run base_$pass X=0
  run split4_$pass CX_CZ_ROOTS_SPLIT=1 CX_CZ_ROOTS_WPE=4
  run split5_$pass CX_CZ_ROOTS_SPLIT=1 CX_CZ_ROOTS_WPE=5
  run split6_$pass CX_CZ_ROOTS_SPLIT=1 CX_CZ_ROOTS_WPE=6
done
run m1_split5 CX_CZ_ROOTS_MODE=1 CX_CZ_ROOTS_SPLIT=1 CX_CZ_ROOTS_WPE=5
run m1_split6 CX_CZ_ROOTS_MODE=1 CX_CZ_ROOTS_SPLIT=1 CX_CZ_ROOTS_WPE=6
echo done
