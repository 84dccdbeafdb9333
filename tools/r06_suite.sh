#!/bin/bash
# GPU suite + C++ driver + smoke + default bench (N = 1) into gpurun_out/$1.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=$PWD/gpurun_out/${1:-r06/suite}; mkdir -p "$OUT"
step() { local name=$1; shift; timeout -k 10 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
tail -1 "$OUT/pytest_gpu.log"
step cpp_driver 120 ./tests/cpp/test_chordx_api
tail -1 "$OUT/cpp_driver.log"
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py
grep '"metric"' "$OUT/bench.log" > "$OUT/bench.json"
