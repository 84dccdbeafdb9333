#!/bin/bash
# Round 6 batch 13: count pass with key prefetch, GPU-only stage timing -- arc tests, G = 8 projection
# A/B against the previous build (ab/libchordx_h0.so), kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b13; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_gpu_arc.py -q -k "count or exact or rccl" --timeout 300 --timeout-method thread
tail -1 $O/pytest.log
step ab_sim 900 bash tools/ab_lib.sh ab/libchordx_h0.so r06/b13/sim_ab 2 benches/bench_arc_exact_sim.py 8
step sim_trace 300 rocprofv3 --kernel-trace --stats -d $O/sim_trace -o sim --output-format csv -- python3 benches/bench_arc_exact_sim.py 8
