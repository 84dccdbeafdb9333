#!/bin/bash
# Extra round-end evidence: streaming ceilings, the replicated and arc bench
# flows with two ranks on one GPU (gloo), the table-build edge-ring tests.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-extra}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u benches/bench_stream.py > "$OUT/stream.json" 2> "$OUT/stream.err"
cat "$OUT/stream.json"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "table_builds_edge or route_table" -x -q \
  --timeout 200 --timeout-method thread > "$OUT/pytest_tables.log" 2>&1
tail -1 "$OUT/pytest_tables.log"
bash tools/rehearse_n2.sh
cp gpurun_out/n2/bench_n2.log "$OUT/"
bash tools/rehearse_arc_n2.sh
cp gpurun_out/arc_n2/bench_arc_n2.log "$OUT/"
