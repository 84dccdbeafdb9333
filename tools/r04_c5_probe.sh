#!/bin/bash
# C5 scan halves (round 4): bench_c5.py with CX_MISPLACED_PROBE = 0 (scan),
# 1 (no row flush), 2 (no search), alternating, timing from the bench line.
set -eo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=$PWD/gpurun_out/${1:-r04_c5probe}
mkdir -p $O
for r in 1 2; do
  for p in 0 1 2; do
    CX_MISPLACED_PROBE=$p timeout -k 10 300 python3 benches/bench_c5.py --steps 10 --warmup 2 \
      --oracle-sample 4096 > $O/p${p}_$r.json 2> $O/p${p}_$r.err
  done
done
