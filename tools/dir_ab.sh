# Directory size A/B: parity tests with the largest setting, then per-row benches.
set -eo pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/dir_ab
mkdir -p $OUT
CX_DIR_EXTRA=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_x2.log 2>&1
tail -1 $OUT/pytest_x2.log
for x in 0 1 2; do
  CX_DIR_EXTRA=$x timeout -k 10 300 python -u benches/bench_rows.py > $OUT/rows_x$x.json 2> $OUT/rows_x$x.err
  echo "x=$x done"
done
