#!/bin/bash
# Fused DHash placement + maintenance scan (cx_dhash_maintenance): parity tests
# (churn-directory cases, device/foreign-parent, C5 at full size), then
# bench_c5 at N = 1 under a kernel trace.
set -eo pipefail
TAG=${1:-r03_c5}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v \
  -k "misplaced or c5 or nsucc or dhash" --timeout 400 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c5" -o run --output-format csv \
  -- python3 "$R/benches/bench_c5.py" > "$OUT/c5_n1.json" 2> "$OUT/c5_n1.err"
tail -1 "$OUT/c5_n1.json" | cut -c1-400
echo done
