#!/bin/bash
# Search variants: parity tests, then bench_search under a kernel trace.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-search}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "successor or predecessor" -x -q \
  --timeout 250 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -1 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 $GRAFT_REPO_ROOT/benches/bench_search.py > "$OUT/bench_search.json" 2> "$OUT/bench_search.err"
cat "$OUT/bench_search.json"
grep -E "k_successor" "$OUT/trace/run_kernel_stats.csv" | cut -c1-60,100-200
