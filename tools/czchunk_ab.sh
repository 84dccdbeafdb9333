#!/bin/bash
# cz build dispatch-order A/B: CX_CZ_CHUNK = 0 (plane order) and chunked orders,
# kernel times of k_cz_build under rocprofv3 (bench_churn.py 24).
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-czchunk}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for k in ${CHUNKS:-0 16 32 64}; do
  CX_CZ_CHUNK=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/k$k" -o run \
    --output-format csv -- python3 "$GRAFT_REPO_ROOT/benches/bench_churn.py" 24 > "$OUT/k$k.log" 2>&1
  python3 -c "import csv,sys; [print('K=' + sys.argv[2], r['Name'][:26], r['Calls'], round(float(r['AverageNs'])/1e6, 2), round(float(r['MinNs'])/1e6, 2)) for r in csv.DictReader(open(sys.argv[1])) if 'cz_build' in r['Name']]" "$OUT/k$k/run_kernel_stats.csv" "$k"
  grep -o '"identical": [a-z]*' "$OUT/k$k.log" || true
done
