#!/bin/bash
# Store-path probes (round 4): pure stores (CX_CZ2_MODE=3) of k_cz_build_roots2
# at its per-level block sizes and at 256 / 320 rows for every level
# (CX_CZ2_NB=16 / 13), the same with the build, and the round-3 kernel's
# stores-only probe (table_build 4, CX_CZ_ROOTS_MODE=2) beside them.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/r04_modes2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # tag, table_builds, VAR=value...
  tag=$1; tb=$2; shift 2
  (export "$@"; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv \
    --kernel-include-regex "cz_build" -- python3 $R/benches/bench_czbuild.py 24 $tb 2 > $O/$tag.json 2> $O/$tag.err)
}
run s_auto 0 CX_CZ2_MODE=3
run s_nb16 0 CX_CZ2_MODE=3 CX_CZ2_NB=16
run s_nb13 0 CX_CZ2_MODE=3 CX_CZ2_NB=13
run s_old 4 CX_CZ_ROOTS_MODE=2
run b_nb16 0 CX_CZ2_NB=16
run b_auto 0 CX_CZ2_MODE=0
