#!/bin/bash
# Churn directory for the misplaced scan: parity tests, C5 bench (both
# variants), kernel trace + FETCH/WRITE passes of the bench.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-misplaced_cd}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py \
  -k "misplaced or churn or c5" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u benches/bench_misplaced.py > "$OUT/bench.json"
cat "$OUT/bench.json"
B="python3 $GRAFT_REPO_ROOT/benches/bench_misplaced.py"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- $B > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --kernel-include-regex "k_misplaced|k_cd_" \
  -d "$OUT/fetch" -o run --output-format csv -- $B > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --kernel-include-regex "k_misplaced|k_cd_" \
  -d "$OUT/write" -o run --output-format csv -- $B > "$OUT/write.log" 2>&1
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.json"
python3 -c "
import json
d=json.load(open('$OUT/pmc_summary.json'))
for k,v in d.items(): print(k, {c: '%.4g'%x for c,x in v.items()})"
grep -E "k_misplaced|k_cd_" "$OUT/trace/run_kernel_stats.csv" | cut -c1-200
