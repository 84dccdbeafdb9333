#!/bin/bash
# Route-table build A/B: k_cz_build_roots2 (table_build 0) against
# k_cz_build_roots3 (8: both windows of a root at once, stores last).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/r04_modes5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ab -o run --output-format csv \
  --kernel-include-regex "cz_build" -- python3 $R/benches/bench_czbuild.py 24 0,8 3 > $O/ab.json 2> $O/ab.err
