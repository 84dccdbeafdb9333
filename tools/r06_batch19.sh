#!/bin/bash
# Round 6 batch 19: bench.py with failing legs reported (LegGuard.run): the
# default run, a run with an injected failure in the arc leg (the line must
# print with `legs_failed`, status 0), the slice-table GPU tests, and the
# N = 2 gloo rehearsal on one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06/b19; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -le 1 ] || exit $rc; }
step tests 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "slice_table"
tail -1 $O/tests.log
step bench 600 python -u bench.py
grep '"metric"' $O/bench.log > $O/bench.json
CX_BENCH_FAIL_LEG=arc timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-churn > $O/fail.log 2>&1; echo "fail rc=$?"
grep -c '"legs_failed"' $O/fail.log
CX_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --peers-log2 22 --keys-log2 23 \
  --c5-keys-log2 24 --steps 5 --warmup 2 --cpu-seconds 4 > $O/n2.log 2>&1; echo "n2 rc=$?"
grep '"metric"' $O/n2.log > $O/n2.json
