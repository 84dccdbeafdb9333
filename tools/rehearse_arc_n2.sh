# Rehearsal of the arc-mode bench (SoA protocol, pipelined pieces) with two
# ranks sharing cuda:0 over gloo (RCCL refuses two ranks on one device).
set -eo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/arc_n2
CX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --mode arc --peers-log2 22 \
  --keys-log2 23 --steps 3 --warmup 1 > gpurun_out/arc_n2/bench_arc_n2.log 2>&1
grep '"metric"' gpurun_out/arc_n2/bench_arc_n2.log | cut -c1-900
