"""World-size-2 rehearsal of bench.py's multi-GPU path on CPU (gloo).

Each rank routes its shard of the global key stream against its own replica of
the ring (here: the CPU oracle stands in for the per-rank engine, since this
runs without a GPU); the harness pieces bench.py uses (chordx.dist: shard,
barrier, max/sum over ranks) must give exactly the single-process answer.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, per_rank, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "p2p-dhts_amd"), os.path.join(root, "oracle")]
    import oracle as O
    import torch.distributed as tdist
    from chordx import dist
    w, r, _ = dist.init("gloo")
    assert (w, r) == (world, rank)
    ring = O.ring_build(O.splitmix_keys(0x5EED0005, 5000))  # replicated ring
    P = O.Peers(ring, O.fingers(ring, threads=2))
    q0, q1 = dist.shard(rank, per_rank)
    keys = O.splitmix_keys(0x5EED0006, q1 - q0, offset=q0)
    src = (np.arange(q0, q1) % len(ring)).astype(np.uint32)
    dist.barrier(world)
    owner, hops, status = O.route(P, src, keys, threads=2)
    t = dist.max_over_ranks(float(rank + 1), world)
    bad = dist.sum_over_ranks(int((status != 0).sum()), world)
    s_h = dist.sum_over_ranks(int(hops.sum()), world)
    out[rank] = (owner.tolist(), hops.tolist(), t, bad, s_h)
    tdist.destroy_process_group()


def test_world2_sharded_route_equals_single_process():
    import oracle as O
    world, per_rank = 2, 3000
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), per_rank, out), nprocs=world,
                       join=True, start_method="spawn")
    ring = O.ring_build(O.splitmix_keys(0x5EED0005, 5000))
    P = O.Peers(ring, O.fingers(ring))
    keys = O.splitmix_keys(0x5EED0006, world * per_rank)
    src = (np.arange(world * per_rank) % len(ring)).astype(np.uint32)
    owner, hops, _ = O.route(P, src, keys)
    got_owner = out[0][0] + out[1][0]
    got_hops = out[0][1] + out[1][1]
    assert got_owner == owner.tolist() and got_hops == hops.tolist()
    assert out[0][2] == out[1][2] == 2.0           # max over ranks
    assert out[0][3] == 0 and out[0][4] == out[1][4] == int(hops.sum())
