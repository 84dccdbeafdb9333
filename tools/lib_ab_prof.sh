#!/bin/bash
# Same-box library A/B under rocprofv3 kernel stats: every ab_libs/*.so (CHORDX_LIB)
# runs <script> [args]; prints the stats rows whose name contains RX.
#   RX=k_fingers bash tools/lib_ab_prof.sh <tag> <script> [args]
set -eo pipefail
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lib in "$GRAFT_REPO_ROOT"/ab_libs/*.so; do
  name=$(basename "$lib" .so)
  CHORDX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
    --output-format csv -- python3 "$@" > "$OUT/$name.log" 2>&1
  python3 -c "import csv,sys; [print(sys.argv[2], r['Name'][:32], r['Calls'], round(float(r['AverageNs'])/1e6, 3)) for r in csv.DictReader(open(sys.argv[1])) if any(x in r['Name'] for x in sys.argv[3].split(','))]" "$OUT/$name/run_kernel_stats.csv" "$name" "$RX"
done
