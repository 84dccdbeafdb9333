#!/bin/bash
# Root-centric build: A' from the row's two-hop plane (CX_CZ_ROOTS_A1=1, one
# dependent gather less on the b = 1 window) vs from the root (=0), alternating
# at 2^24 under a kernel trace, after the route-table identity tests.
set -eo pipefail
TAG=${1:-r03_a1}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k route_table \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
    --output-format csv -- python3 "$R/benches/bench_czbuild.py" 24 0 > "$OUT/$name.json" 2> "$OUT/$name.err"
  python3 -c "
import csv,json
d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
k=[float(r['AverageNs'])/1e6 for r in csv.DictReader(open('$OUT/$name/run_kernel_stats.csv')) if 'cz_build' in r['Name']]
print('$name', 'kernel_ms', k, 'hash', d['route_table_hash'])"
}
for pass in a b; do
  run a1_$pass CX_CZ_ROOTS_A1=1
  run a0_$pass CX_CZ_ROOTS_A1=0
done
run mode1 CX_CZ_ROOTS_MODE=1
run mode2 CX_CZ_ROOTS_MODE=2
run mode3 CX_CZ_ROOTS_MODE=3
echo done
