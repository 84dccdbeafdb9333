#!/bin/bash
# Round 3 (session 2): churn -> route-ready overheads (ring stream/scratch reuse,
# pooled churn temporaries, bucket sort of the joins, deferred finger rows):
# GPU suite, C++ driver, smoke, route-ready breakdown, default bench line.
set -eo pipefail
TAG=${1:-r03_ovh}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 ./tests/cpp/test_chordx_api > "$OUT/cpp_driver.log" 2>&1
tail -1 "$OUT/cpp_driver.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 200 python3 benches/bench_ready.py 24 6 > "$OUT/ready.json" 2> "$OUT/ready.err"
cat "$OUT/ready.json"
CX_JOIN_SORT=radix CX_FINGERS_ROWS=1 timeout -k 10 200 python3 benches/bench_ready.py 24 6 > "$OUT/ready_old.json" 2> "$OUT/ready_old.err"
cat "$OUT/ready_old.json"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cut -c1-400 "$OUT/bench.json"
echo done
