#!/bin/bash
# f2 finger repair: its GPU tests, then route-ready with the repair
# (CX_READY_REPAIR=1, the A/B) and without (the streaming build, default);
# the traced run is the repair's.
set -eo pipefail
TAG=${1:-r03_repair}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_repair.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest_repair.log" 2>&1 || { tail -40 "$OUT/pytest_repair.log"; exit 1; }
tail -1 "$OUT/pytest_repair.log"
CX_READY_REPAIR=1 timeout -k 10 200 python3 benches/bench_ready.py 24 6 > "$OUT/ready_repair_on.json" 2> "$OUT/ready_repair_on.err"
cat "$OUT/ready_repair_on.json"
timeout -k 10 200 python3 benches/bench_ready.py 24 6 > "$OUT/ready_repair_off.json" 2> "$OUT/ready_repair_off.err"
cat "$OUT/ready_repair_off.json"
cd /tmp && export TMPDIR=/tmp
CX_READY_REPAIR=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run \
  --output-format csv -- python3 "$R/benches/bench_ready.py" 24 3 > "$OUT/traced.json" 2> "$OUT/traced.err"
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/trace/run_kernel_stats.csv')):
    if float(r['AverageNs'])>50000: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3))"
echo done
