#!/bin/bash
# Route-table build: does the 64 GiB write stream slow the window gathers?
# The build with every store folded into the table's first 128 MiB
# (CX_CZ2_MODE=16), beside the build and compute only, kernel trace; then
# FETCH_SIZE of the build and of compute only.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
O=$R/gpurun_out/r04_modes4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # tag, VAR=value...
  tag=$1; shift 1
  (export "$@"; timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/$tag -o run --output-format csv \
    --kernel-include-regex "cz_build" -- python3 $R/benches/bench_czbuild.py 24 0 2 > $O/$tag.json 2> $O/$tag.err)
}
run build CX_CZ2_MODE=0
run onchip CX_CZ2_MODE=16
run compute CX_CZ2_MODE=1
pmc() {  # tag, counter, VAR=value...
  tag=$1; c=$2; shift 2
  (export "$@"; timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "cz_build" \
    -d $O/$tag -o run --output-format csv -- python3 $R/benches/bench_czbuild.py 24 0 1 > $O/$tag.json 2> $O/$tag.err)
}
pmc fetch_build FETCH_SIZE CX_CZ2_MODE=0
pmc fetch_compute FETCH_SIZE CX_CZ2_MODE=1
pmc fetch_onchip FETCH_SIZE CX_CZ2_MODE=16
