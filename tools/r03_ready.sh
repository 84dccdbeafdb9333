#!/bin/bash
# churn -> route-ready breakdown: wall per stage, kernel and HIP API traces.
set -eo pipefail
TAG=${1:-r03_ready}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 "$R/benches/bench_ready.py" 24 5 > "$OUT/plain.json" 2> "$OUT/plain.err"
cat "$OUT/plain.json"
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --stats -d "$OUT/trace" -o run \
  --output-format csv -- python3 "$R/benches/bench_ready.py" 24 3 > "$OUT/traced.json" 2> "$OUT/traced.err"
cat "$OUT/traced.json"
ls "$OUT/trace"
echo done
