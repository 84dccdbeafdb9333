#!/bin/bash
# Round-5 evidence in one call (repo root on the GPU box), each GPU step with
# its own limit, chained by &&:
#   GPU suite, C++ driver, smoke, default bench (N = 1) under a kernel trace
#   (+ trace agreement), walk PMC groups (tools/r05_walk_pmc.sh), PMC FETCH /
#   WRITE passes of the route-table build and the C5 kernel, two-rank gloo
#   rehearsal of bench.py.
set -eo pipefail
TAG=${1:-r05_final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest_gpu.log" 2>&1
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 120 ./tests/cpp/test_chordx_api > "$OUT/cpp_driver.log" 2>&1
tail -1 "$OUT/cpp_driver.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$OUT/bench_traced.log" 2>&1
grep '"metric"' "$OUT/bench_traced.log" > "$OUT/bench.json"
cut -c1-300 "$OUT/bench.json"
python3 "$R/tools/trace_agreement.py" "$OUT/trace" "$OUT/bench.json" 3 10 > "$OUT/trace_agreement.txt"
tail -2 "$OUT/trace_agreement.txt"
# keep the merge-back small: only the stats and the hot kernels' launches
find "$OUT/trace" -name "*kernel_trace.csv" -exec sh -c 'grep -E "Kernel_Name|k_walk|k_cz_build|k_misplaced|k_fingers|k_arc" "$1" > "$1.route" && mv "$1.route" "$1"' _ {} \;
cd "$R"
timeout -k 10 900 bash tools/r05_walk_pmc.sh "$TAG/walk_pmc" > "$OUT/walk_pmc.log" 2>&1
tail -1 "$OUT/walk_pmc.log"
cd /tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-arc --no-churn --no-c2 --no-c3"
RX="k_cz_build|k_fingers_tile|k_misplaced"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_fetch" -o run --output-format csv -- $B > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_write" -o run --output-format csv -- $B > "$OUT/pmc_write.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$OUT/pmc_fetch" > "$OUT/pmc_fetch_summary.json"
python3 "$R/tools/pmc_summary.py" "$OUT/pmc_write" > "$OUT/pmc_write_summary.json"
cd "$R"
CX_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --peers-log2 22 --keys-log2 23 \
  --c5-keys-log2 24 --steps 5 --warmup 2 --cpu-seconds 6 > "$OUT/bench_n2.log" 2>&1
grep '"metric"' "$OUT/bench_n2.log" > "$OUT/bench_n2.json"
cut -c1-200 "$OUT/bench_n2.json"
echo done
