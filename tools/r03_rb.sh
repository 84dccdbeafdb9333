#!/bin/bash
# Root-centric build A/B at 2^24, alternating on one box: CX_CZ_ROOTS_RB = 1
# (one lane computes both windows of its root, 256 rows a block) vs 256 / 192
# (one lane per window), then the route-table identity tests.
set -eo pipefail
TAG=${1:-r03_rb}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k route_table \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
for pass in a b; do
  for rb in 1 256 192; do
    CX_CZ_ROOTS_RB=$rb timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/rb${rb}_$pass" -o run \
      --output-format csv -- python3 "$R/benches/bench_czbuild.py" 24 0 > "$OUT/rb${rb}_$pass.json" 2> "$OUT/rb${rb}_$pass.err"
    python3 -c "
import csv,json,sys
d=json.loads(open('$OUT/rb${rb}_$pass.json').read().strip().splitlines()[-1])
k=[float(r['AverageNs'])/1e6 for r in csv.DictReader(open('$OUT/rb${rb}_$pass/run_kernel_stats.csv')) if 'cz_build' in r['Name']]
print('rb', $rb, '$pass', 'kernel_ms', k, 'hash', d['route_table_hash'])"
  done
done
# overlap probe (192 rows a block): compute only, stores only, and half the
# blocks each (different waves on one CU running the two halves)
for mode in 1 2 3; do
  CX_CZ_ROOTS_MODE=$mode timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/mode$mode" -o run \
    --output-format csv -- python3 "$R/benches/bench_czbuild.py" 24 0 > "$OUT/mode$mode.json" 2> "$OUT/mode$mode.err"
  python3 -c "
import csv
k=[float(r['AverageNs'])/1e6 for r in csv.DictReader(open('$OUT/mode$mode/run_kernel_stats.csv')) if 'cz_build' in r['Name']]
print('mode', $mode, 'kernel_ms', k)"
done
bash "$R/tools/r03_c5.sh" "${TAG}_c5"
echo done
