#!/bin/bash
# Same-box A/B of ab_libs/*.so on the route bench with random sources
# (CX_SRC=random), twice in alternating order.
set -eo pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-route_ab_src}
mkdir -p "$OUT"
cd "$GRAFT_REPO_ROOT"
for pass in 1 2; do
  for lib in ab_libs/*.so; do
    CX_SRC=random CHORDX_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 240 python -u benches/bench_route.py 10 5 \
      | tee -a "$OUT/route_ab.jsonl"
  done
done
