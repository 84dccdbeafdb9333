#!/bin/bash
# Arc tests (regions + source hints), route-table identity tests incl. the
# root-centric build, then kernel traces of the default and root-centric builds
# at 2^24 and the G = 8 arc projection (two-pass / regions / hints).
set -eo pipefail
TAG=${1:-r03_roots}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1 || rc=$?
# test failures (rc 1) are read from the log; a crash, abort or time limit ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"; exit $rc; fi
tail -2 "$OUT/pytest.log"
cd /tmp && export TMPDIR=/tmp
for tb in 0 3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/cz_tb$tb" -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT/benches/bench_czbuild.py" 24 $tb > "$OUT/cz_tb$tb.json" 2> "$OUT/cz_tb$tb.err"
  tail -1 "$OUT/cz_tb$tb.json" | cut -c1-300
done
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "k_cz_build" \
  -d "$OUT/pmc_fetch_tb3" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/benches/bench_czbuild.py" 24 3 \
  > "$OUT/pmc_fetch_tb3.log" 2>&1
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python3 -u benches/bench_arc_sim.py --keys-log2 28 --groups 8 --modes soa,soa_regions,soa_hints \
  --reps 3 > "$OUT/arc_sim_g8.json" 2> "$OUT/arc_sim_g8.err"
grep '"G"' "$OUT/arc_sim_g8.err" | cut -c1-300
echo done
