#!/bin/bash
# Round 6 batch 6: GPU suite + bench after the explicit-half shifts and the MSD
# ring sort; sort trace / PMC; C5 ABBA (round-4 HEAD 326314b vs round-5 HEAD
# 6d3632b, directory load factor 1/2 and 1/4 on each; HEAD first and last).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b6; mkdir -p $O $O/c5_abba
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
step bench 900 python -u bench.py
step sort_trace 120 rocprofv3 --kernel-trace --stats -d $O/sort_trace -o sort --output-format csv -- python3 tools/prof_sort.py 24
step sort_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $O/sort_fetch -o sort --output-format csv -- python3 tools/prof_sort.py 24
step sort_write 120 rocprofv3 --pmc WRITE_SIZE -d $O/sort_write -o sort --output-format csv -- python3 tools/prof_sort.py 24
i=0
for v in head r4 r5 r5 r4 r4q r5h r5h r4q head; do
  i=$((i+1))
  if [ $v = head ]; then S=benches/bench_c5.py; else S=ab/c5_$v/benches/bench_c5.py; fi
  step c5_abba/${i}_$v 300 python -u $S
done
