#!/bin/bash
# Round 6 batch 14: the headline walk, this tree against round 5's HEAD
# (ab/libchordx_r5.so, built from 872c601), alternating on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b14; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step ab_walk 900 bash tools/ab_lib.sh ab/libchordx_r5.so r06/b14/walk_r5 3 benches/bench_route.py 10 5
