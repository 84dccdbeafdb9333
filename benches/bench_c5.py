#!/usr/bin/env python3
"""C5 on N GPUs: DHash n = 14 replica lists + the global-maintenance misplaced
scan for 2^26 keys after a batched 1 % join / 1 % leave churn of a 2^24-peer
ring (BASELINE.json configs[4]), key-sharded over ranks.

Every rank generates its share of the old ring's IDs, one all_gather
replicates them (RCCL over xGMI), and every rank applies the same churn
(cx_churn: joins splitmix 0x5EED0009, leaves = distinct peers by an odd
stride), so old ring, new ring and old_to_new are replicated.  Rank r then
scans keys [r Q / N, (r + 1) Q / N) of the 2^26-key stream (splitmix
0x5EED0008): one step = the keys' n-successor lists on the old ring
(DHashPeer::Create's placement, dhash_peer.cpp:103-129) + the misplaced scan
(RunGlobalMaintenance, dhash_peer.cpp:298-348), as one cx_dhash_maintenance
pass (the scan resolves each key's old successor anyway); the two separate
calls (cx_nsucc + cx_misplaced) are timed beside it as `unfused`.  Strong
scaling: the 2^26 keys are fixed, each rank scans 2^26 / N.  No collective in
the timed step; a 14-window never needs a halo because every rank holds both
rings.

Checks (reduced over ranks): the misplaced scan's new lists equal the new
ring's n-successor window of every key; counts = 14; and on rank 0 a sample
equals the oracle's RunGlobalMaintenance restatement (test infrastructure,
oracle/).  Prints one JSON line (rank 0).

    python benches/bench_c5.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "p2p-dhts_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import chordx  # noqa: E402
from chordx import dist  # noqa: E402

SEED_RING, SEED_KEYS, SEED_CHURN = 0x5EED0007, 0x5EED0008, 0x5EED0009
HBM_PEAK = 8.0e12
BYTES_MISPLACED = 139  # SURVEY 8(d) DHash model: 16 + 64 + 56 + 1 + 2 per key
BYTES_NSUCC = 137      # key 16 + one 64-B directory line + 14 x 4 list + 1 count per key
# one pass: key 16 + one 64-B line + old list 56 + count 1 + new list 56 +
# count 1 + mask 2 + targets 14 per key
BYTES_FUSED = 210


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--peers-log2", type=int, default=24)
    ap.add_argument("--keys-log2", type=int, default=26, help="total keys (all ranks)")
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--oracle-sample", type=int, default=1 << 16)
    return ap.parse_args()


def main():
    args = parse()
    rc = dist.launch_self(args.gpus, __file__, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    world, rank, local = dist.env_rank()
    local = local % max(1, torch.cuda.device_count())  # rehearsal: ranks share a GPU
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    backend = os.environ.get("CX_DIST_BACKEND", "nccl")
    dist.init(backend, dev)
    N, Q, n = 1 << args.peers_log2, 1 << args.keys_log2, args.n

    # ---- setup: replicated old ring, replicated churn ----
    share = torch.empty((N // world, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(share, SEED_RING, offset=rank * (N // world))
    ids = dist.gather_ids(share, world, backend)
    old = chordx.Ring(ids, device=local)
    del ids, share
    nj = N // 100
    joins = torch.empty((nj, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(joins, SEED_CHURN)
    pick = (torch.arange(nj, device=dev, dtype=torch.int64) * 0x9E3779B1) % old.n
    leaves = old.ids_device()[pick].contiguous()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    new, o2n = old.churn(joins, leaves)
    new.sync()
    t_churn = time.perf_counter() - t0

    # ---- this rank's key shard ----
    k0, k1 = dist.shard_range(rank, world, Q)
    q = k1 - k0
    keys = torch.empty((q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(keys, SEED_KEYS, offset=k0)

    def step():
        return old.dhash_maintenance(new, o2n, keys, n)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    # per-kernel times on this rank (HIP events on the launch stream), the
    # fused pass and the two separate calls
    s = torch.cuda.current_stream(dev)
    e0, e1, e2, e3 = (torch.cuda.Event(enable_timing=True) for _ in range(4))
    e0.record(s)
    old.nsucc(keys, n)
    e1.record(s)
    old.misplaced(new, o2n, keys, n)
    e2.record(s)
    step()
    e3.record(s)
    torch.cuda.synchronize(dev)
    nsucc_ms, misplaced_ms, fused_ms = (e0.elapsed_time(e1), e1.elapsed_time(e2),
                                        e2.elapsed_time(e3))

    dist.barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize(dev)
    dist.barrier(world)
    dt = time.perf_counter() - t0
    dt_max = dist.max_over_ranks(dt, world, dev)
    old_lists, old_count, lists, count, mask, target = out

    # ---- checks ----
    succ_new = new.successor(keys).to(torch.int64)
    want = (succ_new[:, None] + torch.arange(n, device=dev)) % new.n
    ok_lists = bool((lists.to(torch.int64) == want).all().item()) and \
        bool((count == n).all().item())
    ok_lists = dist.all_over_ranks(ok_lists, world, dev)
    succ_old = old.successor(keys).to(torch.int64)
    want = (succ_old[:, None] + torch.arange(n, device=dev)) % old.n
    ok_old = bool((old_lists.to(torch.int64) == want).all().item()) and \
        bool((old_count == n).all().item())
    ok_old = dist.all_over_ranks(ok_old, world, dev)
    del want, succ_old, succ_new
    misplaced_keys = dist.sum_over_ranks(int((mask != 0).sum().item()), world, dev)
    oracle_ok = None
    if rank == 0 and args.oracle_sample:
        import oracle as O
        m = min(args.oracle_sample, q)
        km = keys[:m].cpu().numpy().view(np.uint64)
        wl, wc, wm, wt = O.misplaced(old.ids(), new.ids(), o2n.cpu().numpy().view(np.uint32),
                                     km, n)
        so = O.successor(old.ids(), km).astype(np.int64)
        wol = ((so[:, None] + np.arange(n)) % old.n).astype(np.uint32)
        oracle_ok = bool((lists[:m].cpu().numpy().view(np.uint32) == wl).all()
                         and (count[:m].cpu().numpy() == wc).all()
                         and (mask[:m].cpu().numpy().view(np.uint16) == wm).all()
                         and (target[:m].cpu().numpy() == wt).all()
                         and (old_lists[:m].cpu().numpy().view(np.uint32) == wol).all())
    dist.barrier(world)
    if rank == 0:
        kps = Q * args.steps / dt_max
        print(json.dumps({
            "metric": "C5 keys/s (whole node): n = 14 replica lists + misplaced scan after "
                      "1 % / 1 % churn",
            "value": kps, "unit": "keys/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt_max * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "strong", "dtype": "u128", "data": "synthetic",
            "config": {"workload": f"C5: 2^{args.peers_log2}-peer ring (splitmix 0x5EED0007), "
                                   f"2^{args.keys_log2} keys (0x5EED0008) scanned by {world} "
                                   f"ranks, n = {n}, {nj} joins (0x5EED0009) + {nj} leaves",
                       "peers_old": old.n, "peers_new": new.n, "keys_total": Q,
                       "keys_per_gpu": q,
                       "parallelism": f"replicated old/new rings (IDs all-gathered), keys "
                                      f"sharded x{world}, no collective in the step"},
            "rank0_kernel_ms": {"fused": fused_ms, "nsucc": nsucc_ms,
                                "misplaced": misplaced_ms},
            "unfused": {"ms": nsucc_ms + misplaced_ms,
                        "keys_per_s_rank0": q / ((nsucc_ms + misplaced_ms) * 1e-3),
                        "note": "cx_nsucc + cx_misplaced as two calls (same outputs)"},
            "roofline": {"bound": "hbm", "unit": "GB/s",
                         "achieved": Q * BYTES_FUSED / (dt_max / args.steps) / 1e9,
                         "peak": HBM_PEAK * world / 1e9,
                         "frac": Q * BYTES_FUSED / (dt_max / args.steps) / (HBM_PEAK * world),
                         "model": f"{BYTES_FUSED} B per key (key, one 64-B search line, old "
                                  "and new 14-lists with counts, mask, targets) over the step "
                                  "time, whole node",
                         "per_kernel_rank0": {
                             "fused_frac": q * BYTES_FUSED / (fused_ms * 1e-3) / HBM_PEAK,
                             "nsucc_frac": q * BYTES_NSUCC / (nsucc_ms * 1e-3) / HBM_PEAK,
                             "misplaced_frac": q * BYTES_MISPLACED / (misplaced_ms * 1e-3)
                             / HBM_PEAK}},
            "churn_ms": t_churn * 1e3,
            "new_lists_equal_new_window": ok_lists,
            "old_lists_equal_old_window": ok_old,
            "keys_with_misplaced_holder": misplaced_keys,
            "oracle_sample_equal": oracle_ok,
            "oracle_sample_keys": min(args.oracle_sample, q) if args.oracle_sample else 0,
        }), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
