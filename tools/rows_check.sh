# GPU suite + per-row bench (benches/bench_rows.py) in one call.
set -eo pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/rows_check
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u benches/bench_rows.py > $OUT/rows.json 2> $OUT/rows.err
python3 -c "import json; d=json.load(open('$OUT/rows.json')); c=d['C5']; print({k: c[k] for k in c if 's' in k})"
timeout -k 10 120 python -u benches/bench_ida.py > $OUT/ida.json 2> $OUT/ida.err
cat $OUT/ida.json
DIAG_RUNS=30 bash tools/cpp_fault_diag.sh
