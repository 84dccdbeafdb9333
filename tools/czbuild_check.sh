#!/bin/bash
# Route-table build change check: identity / parity tests, churn bench, kernel stats + VALU count.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-czbuild}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_arc.py -k "route or table or finger or arc" -x -q \
  --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -u benches/bench_churn.py > "$OUT/churn.json" 2> "$OUT/churn.err"
python3 -c "
import json; d=json.load(open('$OUT/churn.json')); print({k:(round(x*1e3,2) if isinstance(x,float) else x) for k,x in d.items() if 'hash' not in k})"
cd /tmp && export TMPDIR=/tmp
B="python3 $GRAFT_REPO_ROOT/benches/bench_churn.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $B > "$OUT/trace.log" 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
  --kernel-include-regex "k_cz_build" -d "$OUT/sq" -o run --output-format csv -- $B > "$OUT/sq.log" 2>&1
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.json"
python3 -c "
import json
d=json.load(open('$OUT/pmc_summary.json'))
for k,v in d.items(): print(k, {c: '%.4g'%x for c,x in v.items()})"
grep -E "k_cz_build<2, 3>" "$OUT/trace/run_kernel_stats.csv" | cut -d, -f1-6 | cut -c1-40,140-
