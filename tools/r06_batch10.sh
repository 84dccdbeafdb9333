#!/bin/bash
# Round 6 batch 10: GPU suite (compact own walk), arc projections G = 2/4/8,
# gloo rehearsals N = 2 / 8 with progress lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/b10; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step pytest 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
for G in 8 4 2; do
  step sim_g$G 600 python -u benches/bench_arc_exact_sim.py $G 25
done
step bench_n2 900 env CX_DIST_BACKEND=gloo python -u bench.py --gpus 2 --peers-log2 22 --keys-log2 23 --c5-keys-log2 24 --steps 5 --warmup 2 --cpu-seconds 4
step bench_n8 1200 env CX_DIST_BACKEND=gloo python -u bench.py --gpus 8 --peers-log2 20 --keys-log2 21 --c5-keys-log2 22 --steps 3 --warmup 1 --cpu-seconds 3
