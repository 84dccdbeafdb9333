#!/bin/bash
# Round-3 evidence in one call (repo root on the GPU box), each GPU step with
# its own limit, chained by &&:
#   GPU suite, C++ driver, smoke, default bench (N = 1) under a kernel trace
#   (+ trace agreement), PMC FETCH / WRITE passes of the route kernel and the
#   route-table build, C5 bench, two-rank gloo rehearsals of bench.py and
#   bench_c5.py on one GPU.
set -eo pipefail
TAG=${1:-r03_final}
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
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 10 --warmup 3 > "$OUT/bench_traced.log" 2>&1
grep '"metric"' "$OUT/bench_traced.log" > "$OUT/bench.json"
cut -c1-300 "$OUT/bench.json"
python3 "$R/tools/trace_agreement.py" "$OUT/trace" "$OUT/bench.json" 3 10 > "$OUT/trace_agreement.txt"
cat "$OUT/trace_agreement.txt" | tail -2
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-arc --no-churn"
RX="k_route_tree|k_cz_build|k_fingers_tile"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_fetch" -o run --output-format csv -- $B > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_write" -o run --output-format csv -- $B > "$OUT/pmc_write.log" 2>&1
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/pmc_summary.json"
cd "$R"
timeout -k 10 300 python3 -u benches/bench_c5.py > "$OUT/c5_n1.json" 2> "$OUT/c5_n1.err"
tail -1 "$OUT/c5_n1.json" | cut -c1-200
CX_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --peers-log2 22 --keys-log2 23 \
  --steps 5 --warmup 2 --cpu-seconds 6 > "$OUT/bench_n2.log" 2>&1
grep '"metric"' "$OUT/bench_n2.log" > "$OUT/bench_n2.json"
cut -c1-200 "$OUT/bench_n2.json"
CX_DIST_BACKEND=gloo timeout -k 10 400 python3 -u benches/bench_c5.py --gpus 2 --peers-log2 22 \
  --keys-log2 24 --steps 3 --warmup 1 > "$OUT/c5_n2.json" 2> "$OUT/c5_n2.err"
tail -1 "$OUT/c5_n2.json" | cut -c1-200
# root-centric build and its probes at 2^24: 0 = the build, 1 compute only,
# 2 stores only, 3 half the blocks each
cd /tmp
for mode in 0 1 2 3; do
  CX_CZ_ROOTS_MODE=$mode timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/mode$mode" -o run \
    --output-format csv -- python3 "$R/benches/bench_czbuild.py" 24 0 > "$OUT/mode$mode.json" 2> "$OUT/mode$mode.err"
  python3 -c "
import csv
k=[float(r['AverageNs'])/1e6 for r in csv.DictReader(open('$OUT/mode$mode/run_kernel_stats.csv')) if 'cz_build' in r['Name']]
print('mode', $mode, 'kernel_ms', k)"
done
echo done
