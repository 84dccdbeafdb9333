#!/bin/bash
# Churn -> route-ready: identity test, stage times and kernel stats at 2^24.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-churn}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "level_planes" -x -v --timeout 200 \
  --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u benches/bench_churn.py 24 > "$OUT/bench_churn.json" 2> "$OUT/bench_churn.err"
cat "$OUT/bench_churn.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/benches/bench_churn.py" 24 > "$OUT/prof.log" 2>&1
head -14 "$OUT"/prof/run_kernel_stats.csv | cut -c1-160
