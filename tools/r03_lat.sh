#!/bin/bash
# Root-centric build: is it bound by rows in flight?  Alternating passes of
# the default, CX_CZ_ROOTS_LATE=1 (rh[A] per distinct root in the window
# phase: one dependent gather less per block), and CX_CZ_LDS_PAD (extra LDS
# per block: 3 / 2 resident blocks per CU instead of 4); compute-only probes.
set -eo pipefail
TAG=${1:-r03_lat}
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
  run late_$pass CX_CZ_ROOTS_LATE=1
  run pad3_$pass CX_CZ_LDS_PAD=4096
  run pad2_$pass CX_CZ_LDS_PAD=20480
done
run m1_base CX_CZ_ROOTS_MODE=1
run m1_late CX_CZ_ROOTS_MODE=1 CX_CZ_ROOTS_LATE=1
run m1_pad3 CX_CZ_ROOTS_MODE=1 CX_CZ_LDS_PAD=4096
run m2_base CX_CZ_ROOTS_MODE=2
run m2_pad3 CX_CZ_ROOTS_MODE=2 CX_CZ_LDS_PAD=4096
echo done
