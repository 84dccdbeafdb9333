#!/bin/bash
# Round 6 diagnostics 3: standalone k_cz_build variants; bench with the
# overlapped churn leg (no arc / cpu / c5 / c2 / c3).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/diag3; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step czb 300 python -u tools/diag_cz_build_r5.py
step bench_ovl 600 python -u bench.py --steps 5 --warmup 2 --no-arc --no-cpu --no-c5 --no-c2 --no-c3
