#!/bin/bash
# Route-table build halves (round 4): kernel trace of k_cz_build_roots2
# (table_build 0) and the round-3 kernel (4) as the build, compute only
# (CX_CZ2_MODE=1 / CX_CZ_ROOTS_MODE=1) and stores only without gathers (3 / 2).
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/r04_modes3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # tag, table_builds, VAR=value...
  tag=$1; tb=$2; shift 2
  (export "$@"; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv \
    --kernel-include-regex "cz_build|fingers" -- python3 $R/benches/bench_czbuild.py 24 $tb 2 > $O/$tag.json 2> $O/$tag.err)
}
run build 0,4,6,7 CX_CZ2_MODE=0
run compute 0 CX_CZ2_MODE=1
run stores 0 CX_CZ2_MODE=3
run compute_old 4 CX_CZ_ROOTS_MODE=1
run stores_old 4 CX_CZ_ROOTS_MODE=2
