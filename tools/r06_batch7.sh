#!/bin/bash
# Round 6 batch 7: prefix-ranked bucket sort (tests, trace); ABBA of the
# explicit-half shifts (ab/libchordx_preshift.so = a3111de) on the walk, C2
# and churn -> route-ready.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b7; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step pytest_sort 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k "ring_build or sort or churn or successor"
step sort_trace 120 rocprofv3 --kernel-trace --stats -d $O/sort_trace -o sort --output-format csv -- python3 tools/prof_sort.py 24
step ab_walk 900 bash tools/ab_lib.sh ab/libchordx_preshift.so r06/b7/walk_ab 2 benches/bench_walk.py 10 4
step ab_c2 300 bash tools/ab_lib.sh ab/libchordx_preshift.so r06/b7/c2_ab 2 benches/bench_c2.py
step ab_ready 600 bash tools/ab_lib.sh ab/libchordx_preshift.so r06/b7/ready_ab 2 benches/bench_ready.py 24 4
