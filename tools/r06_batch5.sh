#!/bin/bash
# Round 6 batch 5: hazard discrimination (nop / waitcnt-zero builds), sort tests,
# sort kernel trace + PMC.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b5; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step czb_nop 300 python -u tools/diag_cz_build_r5.py libcxtest_nop.so
step czb_wz 300 python -u tools/diag_cz_build_r5.py libcxtest_wz.so
step czb 300 python -u tools/diag_cz_build_r5.py libcxtest.so
step pytest_sort 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -q --timeout 300 --timeout-method thread -k "ring_build or sort or churn"
step sort_trace 120 rocprofv3 --kernel-trace --stats -d $O/sort_trace -o sort --output-format csv -- python3 tools/prof_sort.py 24
step sort_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $O/sort_fetch -o sort --output-format csv -- python3 tools/prof_sort.py 24
step sort_write 120 rocprofv3 --pmc WRITE_SIZE -d $O/sort_write -o sort --output-format csv -- python3 tools/prof_sort.py 24
