#!/bin/bash
# Round-3 check on the GPU box: GPU suite, smoke, default bench (N = 1, with the
# arc / churn / CPU legs), the two-rank gloo rehearsal of `bench.py --gpus 2`
# (ranks share cuda:0, 2^22 ring so both replicas fit), kernel trace of the bench.
# Each GPU step has its own limit; chained by &&.
set -eo pipefail
TAG=${1:-r03}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 120 ./tests/cpp/test_chordx_api > "$OUT/cpp_driver.log" 2>&1
tail -1 "$OUT/cpp_driver.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 500 python -u bench.py > "$OUT/bench_default.log" 2>&1
grep '"metric"' "$OUT/bench_default.log" > "$OUT/bench.json"
cut -c1-400 "$OUT/bench.json"
CX_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --peers-log2 22 --keys-log2 23 \
  --steps 5 --warmup 2 --cpu-seconds 6 > "$OUT/bench_n2.log" 2>&1
grep '"metric"' "$OUT/bench_n2.log" > "$OUT/bench_n2.json"
cut -c1-300 "$OUT/bench_n2.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu > "$OUT/bench_trace.log" 2>&1
echo done
