#!/bin/bash
# Slice-code build: dispatch chunk (row-blocks x all levels) 16 (default) vs 8 / 32 / 64,
# alternating; plus route-ready (planes-only tile from the first plane level).
set -eo pipefail
TAG=${1:-r03_chunk}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deferred_rows.py tests/test_gpu_repair.py -m gpu -x -q \
  -k "route_table or deferred or repair or finger" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
    --output-format csv -- python3 "$R/benches/bench_czbuild.py" 24 0 > "$OUT/$name.json" 2> "$OUT/$name.err"
  python3 -c "
import csv,json
d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
k={r['Name'][:20]: round(float(r['AverageNs'])/1e6,3) for r in csv.DictReader(open('$OUT/$name/run_kernel_stats.csv')) if 'cz_build' in r['Name'] or 'fingers_tile' in r['Name']}
print('$name', k, 'hash', d['route_table_hash'], 'route_ok', d.get('route_ok'), 'wall', [round(x*1e3,1) for x in d['fingers_and_table_s']])"
}
for pass in a b; do
  run default_$pass X=0
  run k16_$pass CX_CZ_CHUNK=16
  run hi_$pass CX_CZ_CODES=hi
done
cd "$R"
timeout -k 10 200 python3 benches/bench_ready.py 24 6 > "$OUT/ready.json" 2> "$OUT/ready.err"
python3 -c "
import json
d=json.loads(open('$OUT/ready.json').read())
print('ready', [round(x['route_ready_ms'],2) for x in d['reps']], d['hashes_equal'], d['hash'])"
echo done
