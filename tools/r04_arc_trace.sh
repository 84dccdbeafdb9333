#!/bin/bash
# Arc leg timeline (round 4): kernel trace of bench.py's arc sub-record at
# N = 1 (one-rank RCCL group), kernels of the arc path only.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/${1:-r04_arc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv \
  --kernel-include-regex "arc|route_tree<true|rccl|copyBuffer|fillBuffer" \
  -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-churn --no-c5 > $O/bench.log 2>&1
