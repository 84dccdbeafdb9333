#!/bin/bash
# Route-table build halves (round 4): kernel trace of k_cz_build_roots2 on quad
# planes (table_build 0) and 4-B planes (5) as the build, compute only
# (CX_CZ2_MODE=1) and stores only (2), then SQ / TA PMC of the two layouts.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/r04_modes
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for M in 3 7 11 15 0 8; do
  CX_CZ2_MODE=$M timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/mode$M -o run --output-format csv \
    --kernel-include-regex "cz_build|fingers" -- python3 $R/benches/bench_czbuild.py 24 0 2 > $O/mode$M.json 2> $O/mode$M.err
done
