#!/bin/bash
# Round 6 batch 16: own lookups compacted by the count pass (keys, sources,
# indices) and walked from contiguous arrays (cx_arc_route_own) -- arc tests,
# then the G = 8 / 4 / 2 projections, compacted (A) against in place (B:
# CX_SIM_OWN=inplace, same library), alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b16; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_gpu_arc.py tests/test_multiproc.py -q --timeout 300 --timeout-method thread
tail -1 $O/pytest.log
for G in 8 4 2; do
  for i in 1 2; do
    timeout -k 10 300 python3 benches/bench_arc_exact_sim.py $G > $O/A_g${G}_$i.json 2> $O/A_g${G}_$i.err || exit 1
    CX_SIM_OWN=inplace timeout -k 10 300 python3 benches/bench_arc_exact_sim.py $G > $O/B_g${G}_$i.json 2> $O/B_g${G}_$i.err || exit 1
  done
  echo G=$G done
done
step sim_trace 300 rocprofv3 --kernel-trace --stats -d $O/sim_trace -o sim --output-format csv -- python3 benches/bench_arc_exact_sim.py 8
