#!/bin/bash
# Round 6 batch 15: is the 2 % headline gap to round 5's library (b14) the
# ring sort's allocation pattern?  Three builds alternating on one box:
# A = this tree, L = this tree with the LSD ring sort (EXTRA=-DCX_RING_SORT_LSD),
# R = round 5's HEAD; benches/bench_route.py 10 5 each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b15; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python3 benches/bench_route.py 10 5 > $O/A_$i.json 2> $O/A_$i.err || exit 1
  CHORDX_LIB=$PWD/ab/libchordx_lsd.so timeout -k 10 300 python3 benches/bench_route.py 10 5 > $O/L_$i.json 2> $O/L_$i.err || exit 1
  CHORDX_LIB=$PWD/ab/libchordx_r5.so timeout -k 10 300 python3 benches/bench_route.py 10 5 > $O/R_$i.json 2> $O/R_$i.err || exit 1
  echo round $i done
done
