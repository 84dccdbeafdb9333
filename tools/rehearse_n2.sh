# Rehearsal of the multi-rank bench flow on a one-GPU box: 2 ranks share cuda:0
# over gloo (RCCL refuses two ranks on one device); smaller ring to fit twice.
set -eo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/n2
CX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --peers-log2 22 --keys-log2 23 \
  --steps 3 --warmup 1 > gpurun_out/n2/bench_n2.log 2>&1
grep '"metric"' gpurun_out/n2/bench_n2.log | cut -c1-600
