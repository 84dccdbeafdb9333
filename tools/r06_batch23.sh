#!/bin/bash
# Round 6 batch 23: PMC FETCH_SIZE / WRITE_SIZE of the exact successor kernel
# after the streaming key loads (benches/bench_succ.py 3), and its timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD; O=$R/gpurun_out/r06/b23; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step succ 300 python -u benches/bench_succ.py 20
grep '"peers"' $O/succ.log
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  step pmc_$c 180 rocprofv3 --kernel-trace --pmc $c --kernel-include-regex "k_successor" -d $O/pmc_$c -o run --output-format csv -- python3 $R/benches/bench_succ.py 3
done
python3 $R/tools/pmc_summary.py $O/pmc_FETCH_SIZE > $O/pmc_fetch_summary.json
python3 $R/tools/pmc_summary.py $O/pmc_WRITE_SIZE > $O/pmc_write_summary.json
