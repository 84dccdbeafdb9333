#!/bin/bash
# Route-table build A/B: k_cz_build_roots2 (table_build 0) against
# k_cz_build_roots2<7, 0, true> (9: plane 0 stored after the W1 gathers).
# Round 4's first A/B (0 against 8, k_cz_build_roots3) is in
# profiles/r04/build_modes/roots3_ab.json.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/r04_modes6
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/ab -o run --output-format csv \
  --kernel-include-regex "cz_build" -- python3 $R/benches/bench_czbuild.py 24 0,9 4 > $O/ab.json 2> $O/ab.err
