#!/bin/bash
# Round 6 batch 18: bench.py with the per-leg watchdog -- default run, a run
# whose legs are given 2 s (the churn leg then aborts: the headline line must
# still print, exit 0), and the N = 2 gloo rehearsal on one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b18; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step bench 600 python -u bench.py
grep '"metric"' $O/bench.log > $O/bench.json
CX_BENCH_LEG_LIMIT_S=2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > $O/guard.log 2>&1; echo "guard rc=$?"
grep -c '"legs_aborted"' $O/guard.log
CX_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --peers-log2 22 --keys-log2 23 \
  --c5-keys-log2 24 --steps 5 --warmup 2 --cpu-seconds 4 > $O/n2.log 2>&1; echo "n2 rc=$?"
grep '"metric"' $O/n2.log > $O/n2.json
