#!/bin/bash
# Round 6 batch 8: GPU suite, sort trace, ABBA of the shift helpers (ab/
# libchordx_preshift.so = a3111de) on walk / C2 / route-ready, bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b8; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step sort_trace 120 rocprofv3 --kernel-trace --stats -d $O/sort_trace -o sort --output-format csv -- python3 tools/prof_sort.py 24
step ab_walk 900 bash tools/ab_lib.sh ab/libchordx_preshift.so r06/b8/walk_ab 3 benches/bench_walk.py 10 4
step ab_c2 300 bash tools/ab_lib.sh ab/libchordx_preshift.so r06/b8/c2_ab 2 benches/bench_c2.py
step ab_ready 600 bash tools/ab_lib.sh ab/libchordx_preshift.so r06/b8/ready_ab 2 benches/bench_ready.py 24 4
step bench 900 python -u bench.py
