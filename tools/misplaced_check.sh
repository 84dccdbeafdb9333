#!/bin/bash
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-misplaced}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py \
  -k "misplaced or churn or c5" -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
tail -3 "$OUT/pytest.log"
timeout -k 10 200 python -u benches/bench_misplaced.py > "$OUT/derived.json"
CX_MISPLACED_SEARCH=1 timeout -k 10 200 python -u benches/bench_misplaced.py > "$OUT/search.json"
cat "$OUT/derived.json" "$OUT/search.json"
bash tools/pmc_kernel.sh ${1:-misplaced}_pmc "k_misplaced" $GRAFT_REPO_ROOT/benches/bench_misplaced.py | grep -v "^ *\"SQ"
