#!/bin/bash
# Replicated vs key-first arc walk on one rank: timings, then PMC passes.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-arc_kernel}
mkdir -p "$OUT"
B="python3 $GRAFT_REPO_ROOT/benches/bench_arc_kernel.py"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- $B > "$OUT/ab.json" 2> "$OUT/ab.err"
cat "$OUT/ab.json"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_FLAT \
  --kernel-include-regex "k_route_tree" -d "$OUT/sq" -o run --output-format csv -- $B > "$OUT/sq.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "k_route_tree" \
  -d "$OUT/fetch" -o run --output-format csv -- $B > "$OUT/fetch.log" 2>&1
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.json"
python3 -c "
import json
d=json.load(open('$OUT/pmc_summary.json'))
for k,v in d.items(): print(k, {c: '%.4g'%x for c,x in v.items()})"
