#!/bin/bash
# Round 6 batch 11: interleaved directory successor (4 keys per lane) --
# successor / predecessor parity, C2 A/B against e256489, C2 kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b11; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step pytest 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -q --timeout 300 --timeout-method thread -k "successor or predecessor or c2 or get_pred"
step ab_c2 300 bash tools/ab_lib.sh ab/libchordx_e256.so r06/b11/c2_ab 3 benches/bench_c2.py
step c2_trace 120 rocprofv3 --kernel-trace --stats -d $O/c2_trace -o c2 --output-format csv -- python3 benches/bench_c2.py
step pytest_sort 600 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -k "ring_build or sort or churn"
step sort_trace 120 rocprofv3 --kernel-trace --stats -d $O/sort_trace -o sort --output-format csv -- python3 tools/prof_sort.py 24
