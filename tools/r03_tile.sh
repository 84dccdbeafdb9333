#!/bin/bash
# Planes-only finger tile (no row tile in LDS): parity tests, route-ready, tile kernel time.
set -eo pipefail
TAG=${1:-r03_tile}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deferred_rows.py tests/test_gpu_repair.py -m gpu -x -q \
  -k "route_table or deferred or repair or finger or churn" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 "$R/benches/bench_ready.py" 24 6 > "$OUT/plain.json" 2> "$OUT/plain.err"
python3 -c "
import json
d=json.loads(open('$OUT/plain.json').read())
print('ready', [round(x['route_ready_ms'],2) for x in d['reps']], d['hashes_equal'], d['hash'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run \
  --output-format csv -- python3 "$R/benches/bench_ready.py" 24 3 > "$OUT/traced.json" 2> "$OUT/traced.err"
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/trace/run_kernel_stats.csv')):
    if float(r['TotalDurationNs']) > 2e6: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e6,3))"
echo done
