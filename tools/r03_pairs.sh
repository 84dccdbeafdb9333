#!/bin/bash
# Two-hop planes kernel rewrite: identity tests, kernel trace of the build, route-ready.
set -eo pipefail
TAG=${1:-r03_pairs}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_repair.py tests/test_gpu_deferred_rows.py -m gpu -x -q \
  -k "route_table or repair or deferred or finger" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/benches/bench_ready.py" 24 4 > "$OUT/ready.json" 2> "$OUT/ready.err"
python3 -c "
import csv,json
for r in csv.DictReader(open('$OUT/trace/run_kernel_stats.csv')):
    if float(r['AverageNs'])>60000: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e6,3))
d=json.loads(open('$OUT/ready.json').read())
print('ready(traced)', [round(x['route_ready_ms'],2) for x in d['reps']], d['hashes_equal'])"
cd "$R"
timeout -k 10 200 python3 benches/bench_ready.py 24 6 > "$OUT/ready_plain.json" 2> "$OUT/ready_plain.err"
python3 -c "
import json
d=json.loads(open('$OUT/ready_plain.json').read())
print('ready', [round(x['route_ready_ms'],2) for x in d['reps']], d['hashes_equal'], d['hash'])"
echo done
