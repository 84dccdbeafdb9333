#!/bin/bash
# Round-6 evidence in one call (repo root on the GPU box), each GPU step with
# its own limit; a step that aborts, faults or times out ends the call:
#   GPU suite, C++ driver, smoke, default bench (N = 1, untraced), the same
#   under a kernel trace (+ trace agreement), walk PMC groups, PMC FETCH /
#   WRITE of the route-table build and the C5 kernel, C2 LDS-search PMC.
TAG=${1:-r06/final3}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
step() { local name=$1; shift; timeout -k 10 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
tail -1 "$OUT/pytest_gpu.log"
step cpp_driver 120 ./tests/cpp/test_chordx_api
tail -1 "$OUT/cpp_driver.log"
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python -u bench.py
grep '"metric"' "$OUT/bench.log" > "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
step bench_traced 900 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 10 --warmup 3
grep '"metric"' "$OUT/bench_traced.log" > "$OUT/bench_traced.json"
python3 "$R/tools/trace_agreement.py" "$OUT/trace" "$OUT/bench_traced.json" 3 10 > "$OUT/trace_agreement.txt"
tail -2 "$OUT/trace_agreement.txt"
find "$OUT/trace" -name "*kernel_trace.csv" -exec sh -c 'grep -E "Kernel_Name|k_walk|k_cz_build|k_misplaced|k_fingers|k_arc|k_ms_|k_rs_" "$1" > "$1.route" && mv "$1.route" "$1"' _ {} \;
cd "$R"
step walk_pmc 1200 bash tools/r05_walk_pmc.sh "$TAG/walk_pmc"
cd /tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-arc --no-churn --no-c2 --no-c3"
RX="k_cz_build|k_fingers_tile|k_misplaced"
step pmc_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_fetch" -o run --output-format csv -- $B
step pmc_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "$RX" \
  -d "$OUT/pmc_write" -o run --output-format csv -- $B
python3 "$R/tools/pmc_summary.py" "$OUT/pmc_fetch" > "$OUT/pmc_fetch_summary.json"
python3 "$R/tools/pmc_summary.py" "$OUT/pmc_write" > "$OUT/pmc_write_summary.json"
cd "$R"
for g in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU" "FETCH_SIZE" "WRITE_SIZE"; do
  k=$((k+1)); cd /tmp
  step c2_pmc$k 120 rocprofv3 --kernel-trace --pmc $g --kernel-include-regex "k_successor_lds" -d "$OUT/c2_pmc$k" -o run --output-format csv -- python3 "$R/benches/bench_c2.py" 1
done
echo done
