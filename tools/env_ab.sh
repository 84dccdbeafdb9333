#!/bin/bash
# Env-switch A/B under rocprofv3 kernel stats (same box, one process per value):
#   VAR=CX_CZ_STORE VALS="0 1 2 3" RX=k_cz_build bash tools/env_ab.sh <tag> <script> [args]
set -eo pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in $VALS; do
  env "$VAR=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/v$v" -o run \
    --output-format csv -- python3 "$@" > "$OUT/v$v.log" 2>&1
  python3 -c "import csv,sys; [print(sys.argv[2], r['Name'][:32], r['Calls'], round(float(r['AverageNs'])/1e6, 3), round(float(r['MinNs'])/1e6, 3)) for r in csv.DictReader(open(sys.argv[1])) if sys.argv[3] in r['Name']]" "$OUT/v$v/run_kernel_stats.csv" "$VAR=$v" "$RX"
  grep -o '"identical": [a-z]*' "$OUT/v$v.log" || true
done
