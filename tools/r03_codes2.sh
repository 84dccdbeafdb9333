#!/bin/bash
# Slice-code build defaults: sequential W1 at 5 waves (default now) vs 6 waves
# (8 spilled VGPRs), with the row word encoded late, and the high-word build;
# then churn -> route-ready with the new default.
set -eo pipefail
TAG=${1:-r03_codes2}
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
print('$name', 'kernel_ms', k, 'hash', d['route_table_hash'], 'route_ok', d.get('route_ok'), 'wall', [round(x*1e3,1) for x in d['fingers_and_table_s']])"
}
for pass in a b; do
  run default_$pass X=0
  run seq6_$pass CX_CZ_ROOTS_SPLIT=5
  run late_$pass CX_CZ_ROOTS_LATE=1
  run hi_$pass CX_CZ_CODES=hi
done
cd "$R"
timeout -k 10 200 python3 benches/bench_ready.py 24 6 > "$OUT/ready.json" 2> "$OUT/ready.err"
python3 -c "
import json
d=json.loads(open('$OUT/ready.json').read())
print('ready', [round(x['route_ready_ms'],2) for x in d['reps']], d['hashes_equal'])"
echo done
