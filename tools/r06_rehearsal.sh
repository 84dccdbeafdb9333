#!/bin/bash
# Round 6: gloo rehearsals of bench.py's multi-rank flow on one GPU (N = 2 and
# 8 ranks sharing the card, small ring), with every leg's checks.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06/rehearsal; mkdir -p $O
CX_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --peers-log2 22 --keys-log2 23 \
  --c5-keys-log2 24 --steps 5 --warmup 2 --cpu-seconds 4 > $O/bench_n2.log 2>&1 && \
CX_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 8 --peers-log2 20 --keys-log2 21 \
  --c5-keys-log2 22 --steps 3 --warmup 1 --cpu-seconds 3 > $O/bench_n8.log 2>&1
echo rc=$?
