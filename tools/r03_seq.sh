#!/bin/bash
# Root-centric build: W1 after plane 0 (one window per lane at a time, LDS
# split) at 5 / 6 waves per SIMD vs the default, alternating; same hash.
set -eo pipefail
TAG=${1:-r03_seq}
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
  run seq5_$pass CX_CZ_ROOTS_SPLIT=2 CX_CZ_ROOTS_WPE=5
  run seq6_$pass CX_CZ_ROOTS_SPLIT=2 CX_CZ_ROOTS_WPE=6
  run chunk8_$pass CX_CZ_CHUNK=8
  run chunk32_$pass CX_CZ_CHUNK=32
done
echo done
