#!/bin/bash
# Arc leg timeline (round 5): kernel + memory-copy trace of bench.py's arc
# sub-record at N = 1 (the other legs off), for the per-step breakdown.
#   bash tools/r05_arc_trace.sh <tag>
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/${1:-r05_arc_trace}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace -o arc \
  --output-format csv -- python3 $R/bench.py --steps 3 --warmup 2 --no-c2 --no-c3 --no-c5 \
  --no-churn --no-cpu > $O/bench.json 2> $O/bench.err
tail -1 $O/bench.json | head -c 300
find $O -name "*stats.csv" | sort
