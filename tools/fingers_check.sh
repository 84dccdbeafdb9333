#!/bin/bash
# Finger build: parity tests + kernel stats of both builds at 2^20 and 2^24.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-fingers}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py \
  -k "finger or c4 or c3" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u benches/bench_fingers.py 20 24 > "$OUT/bench_fingers.json" 2> "$OUT/bench_fingers.err"
cat "$OUT/bench_fingers.json"
cd /tmp && export TMPDIR=/tmp
CX_BENCH_FINGERS_CHILD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tile" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/benches/bench_fingers.py" 24 > "$OUT/prof_tile.log" 2>&1
CX_BENCH_FINGERS_CHILD=1 CX_FINGERS_SEARCH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/search" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/benches/bench_fingers.py" 24 > "$OUT/prof_search.log" 2>&1
grep -h "k_fingers" "$OUT"/tile/run_kernel_stats.csv "$OUT"/search/run_kernel_stats.csv | cut -c1-200
