#!/bin/bash
# Kernel-time A/B of library builds: for each ab_libs/*.so, run a python script
# under rocprofv3 --kernel-trace --stats with CHORDX_LIB pointing at it and
# print the stats rows matching a kernel regex.
#   bash tools/lib_ab.sh <tag> <kernel-grep> <script> [args...]
set -eo pipefail
TAG=$1; RX=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for lib in "$GRAFT_REPO_ROOT"/ab_libs/*.so; do
  name=$(basename "$lib" .so)
  CHORDX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$name" -o run \
    --output-format csv -- python3 "$@" > "$OUT/$name.log" 2>&1
  echo "== $name"
  python3 -c "import csv,sys; [print(r[\"Name\"][:60], r[\"Calls\"], float(r[\"AverageNs\"])/1e6, \"ms\") for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r[\"Name\"]]" "$OUT/$name/run_kernel_stats.csv" "$RX"
done
