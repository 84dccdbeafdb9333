#!/bin/bash
# Route-table build with 32-bit slice gap codes vs 64-bit high words, and the
# slice codes with the LDS split at 4 / 5 waves and the sequential W1 at 5
# (fewer VGPRs now), alternating; every table hash must agree.  Route-table
# identity tests first.
set -eo pipefail
TAG=${1:-r03_codes}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_repair.py -m gpu -x -q -k "route_table or repair" \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
    --output-format csv -- python3 "$R/benches/bench_czbuild.py" 24 0 > "$OUT/$name.json" 2> "$OUT/$name.err"
  python3 -c "
import csv,json
d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
k=[round(float(r['AverageNs'])/1e6,2) for r in csv.DictReader(open('$OUT/$name/run_kernel_stats.csv')) if 'cz_build' in r['Name']]
print('$name', 'kernel_ms', k, 'hash', d['route_table_hash'], 'route_ok', d.get('route_ok'), 'wall', [round(x*1e3,1) for x in d['fingers_and_table_s']])"
}
for pass in a b; do
  run hi_$pass CX_CZ_CODES=hi
  run slice_$pass X=0
  run slice_seq5_$pass CX_CZ_ROOTS_SPLIT=2
  run slice_split5_$pass CX_CZ_ROOTS_SPLIT=3
  run slice_split4_$pass CX_CZ_ROOTS_SPLIT=1
done
echo done
