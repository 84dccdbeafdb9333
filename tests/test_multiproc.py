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


# ---------------------------------------------------------------------------
# Arc-sharded exchange protocol (chordx.arc.ArcRouter) over gloo, world 2 and 3.
# ---------------------------------------------------------------------------
class OracleArcEngine:
    """CPU stand-in for the per-rank arc engine (test infrastructure): a NEW
    lookup is resolved by the oracle, then travels as a WALK record to the
    rank whose arc holds the owner peer, which finishes it there -- locally or
    as a RESULT record back to the origin.  Exercises the protocol (buckets,
    count matrix, all_to_all, homecoming results, termination), not the walk,
    which tests/test_gpu_arc.py checks on the GPU."""

    def __init__(self, P, n):
        self.P, self.n = P, n
        self.region_cap = None  # force a region capacity (overflow fallback test)

    def arc_build(self, world, rank):
        from chordx.arc import arc_bounds
        self.lo, self.hi = arc_bounds(self.n, world, rank)

    def arc_seed(self, rank, src, keys):
        import torch
        q = keys.shape[0]
        r = torch.zeros((q, 4), dtype=torch.int64)
        r[:, :2] = keys.view(torch.int64).reshape(q, 2)
        r[:, 2] = (rank << 40) + torch.arange(q)
        r[:, 3] = src.to(torch.int64) & 0xFFFFFFFF
        return r

    def arc_step(self, rank, recs, owner, hops, status):
        import torch
        import oracle as O
        r = recs.numpy().copy()
        out = np.zeros_like(r)
        kind = (r[:, 3] >> 40) & 0xFF
        cur = r[:, 3] & 0xFFFFFFFF
        h = (r[:, 3] >> 32) & 0xFF
        new = np.nonzero(kind == 0)[0]
        res = {}
        if len(new):
            ow, hp, st = O.route(self.P, cur[new].astype(np.uint32),
                                 r[new, :2].view(np.uint64).reshape(-1, 2))
            for j, i in enumerate(new):
                o = int(ow[j])
                if st[j] != 0 or self.lo <= o < self.hi:
                    res[i] = (o, int(hp[j]), int(st[j]))
                else:
                    out[i] = r[i]
                    out[i, 3] = o | ((int(hp[j]) | (2 << 8)) << 32)
        for i in np.nonzero(kind == 2)[0]:
            res[i] = (int(cur[i]), int(h[i]), 0)
        for i in np.nonzero(kind == 1)[0]:
            res[i] = (int(r[i, 0]) & 0xFFFFFFFF, int(h[i]), (int(r[i, 0]) >> 32) & 0xFF)
        for i, (o, hh, st) in res.items():
            origin, idx = int(r[i, 2]) >> 40, int(r[i, 2]) & ((1 << 40) - 1)
            out[i, 2] = r[i, 2]
            if origin == rank:
                owner[idx] = o if o < (1 << 31) else o - (1 << 32)
                hops[idx] = hh
                status[idx] = st
                out[i, 3] = 3 << 40
            else:
                out[i, 0] = o | (st << 32)
                out[i, 3] = o | ((hh | (1 << 8)) << 32)
        return torch.from_numpy(out)

    # --- structure-of-arrays key-first protocol (ArcRouter.route_soa) ---
    def arc_partition(self, world, src, keys):
        import torch
        import oracle as O
        from chordx.arc import arc_of
        k = keys.numpy().view(np.uint64).reshape(-1, 2)
        own = O.successor(self.P.ring, k)
        dest = np.array([arc_of(int(o), self.n, world) for o in own], dtype=np.int64)
        order = np.argsort(dest, kind="stable")  # send slot -> lookup
        slot = np.empty_like(order)
        slot[order] = np.arange(len(order))       # lookup -> send slot
        counts = [int((dest == d).sum()) for d in range(world)]
        return (keys[torch.from_numpy(order)].contiguous(),
                src[torch.from_numpy(order)].contiguous(),
                torch.from_numpy(slot.astype(np.int32)), counts)

    arc_hints = True  # plumbing check: hint = 7 src + 1 must arrive next to its src

    def arc_partition_regions(self, world, src, keys, cap, hints=False):
        """Region layout of cx_arc_partition_regions: destination d's lookups
        at rows [d cap, d cap + count_d), perm = region slot; None past cap."""
        import torch
        sk, ss, slot, counts = self.arc_partition(world, src, keys)
        if self.region_cap is not None:
            cap = self.region_cap
        if any(c > cap for c in counts):
            return None
        start = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
        rk = torch.zeros((world * cap, 2), dtype=torch.int64)
        rs = torch.zeros(world * cap, dtype=torch.int32)
        dest = np.repeat(np.arange(world), counts)
        new_slot = dest * cap + (np.arange(len(dest)) - start[dest])
        rk[torch.from_numpy(new_slot)] = sk
        rs[torch.from_numpy(new_slot)] = ss
        perm = torch.from_numpy(new_slot[slot.numpy()].astype(np.int32))
        if hints:
            return rk, rs, perm, counts, rs.to(torch.int64) * 7 + 1
        return rk, rs, perm, counts

    def arc_route(self, src, keys, hint=None):
        import torch
        import oracle as O
        if hint is not None:  # the hints travelled with their lookups
            assert torch.equal(hint, src.to(torch.int64) * 7 + 1)
        k = keys.numpy().view(np.uint64).reshape(-1, 2)
        ow, hp, st = O.route(self.P, src.numpy().astype(np.uint32), k)
        own = np.asarray(ow, dtype=np.uint64)
        # every lookup sent here ends in this rank's arc (or fails at its source)
        assert all(st[j] != 0 or self.lo <= int(own[j]) < self.hi for j in range(len(own)))
        v = own | (np.asarray(hp, np.uint64) << 32) | (np.asarray(st, np.uint64) << 40)
        return torch.from_numpy((v | np.uint64(1 << 63)).view(np.int64))

    def arc_deliver(self, res, perm, owner, hops, status):
        v = res.numpy().view(np.uint64)
        slot = np.arange(len(v)) if perm is None else perm.numpy()
        for i, j in enumerate(slot):
            w = int(v[int(j)])
            o = w & 0xFFFFFFFF
            owner[i] = o if o < (1 << 31) else o - (1 << 32)
            hops[i] = (w >> 32) & 0xFF
            if status is not None:
                status[i] = (w >> 40) & 0xFF

    def arc_local_ring(self, lo, hi):
        """The arc's IDs as their own ring: successor() -> int32 indices in it."""
        import torch
        import oracle as O
        sub = np.ascontiguousarray(self.P.ring[lo:hi])

        class _Arc:
            def successor(self, keys):
                k = keys.numpy().view(np.uint64).reshape(-1, 2)
                return torch.from_numpy(O.successor(sub, k).astype(np.int32))
        return _Arc()

    def arc_bucket(self, world, recs):
        import torch
        import oracle as O
        from chordx.arc import arc_of
        r = recs.numpy()
        dest = []
        for row in r:
            kind = (int(row[3]) >> 40) & 0xFF
            if kind == 1:
                dest.append(int(row[2]) >> 40)
            elif kind == 2:
                dest.append(arc_of(int(row[3]) & 0xFFFFFFFF, self.n, world))
            elif kind == 0:  # a lookup sent ahead by key: the arc of its owner
                o = int(O.successor(self.P.ring, row[:2].view(np.uint64).reshape(1, 2))[0])
                dest.append(arc_of(o, self.n, world))
            else:
                dest.append(-1)
        dest = np.array(dest, dtype=np.int64)
        order = np.argsort(dest, kind="stable")
        order = order[dest[order] >= 0]
        counts = [int((dest == d).sum()) for d in range(world)]
        return torch.from_numpy(r[order].copy()), counts


def _arc_worker(rank, world, port, per_rank, out, key_first=True, protocol="records",
                chunks=None, sizes=None, regions=False, region_cap=None, exchange_always=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "p2p-dhts_amd"), os.path.join(root, "oracle"),
                    os.path.join(root, "tests")]
    import torch
    import torch.distributed as tdist
    import oracle as O
    from chordx import dist
    from chordx.arc import ArcRouter
    from test_multiproc import OracleArcEngine
    dist.init("gloo")
    if world == 1:
        assert dist.init_single("gloo")
    ring = O.ring_build(O.splitmix_keys(0x5EED0005, 3000))
    P = O.Peers(ring, O.fingers(ring, threads=2))
    if sizes is not None:  # uneven per-rank batches (one may be empty)
        per_rank = sizes[rank]
    keys = O.splitmix_keys(0x5EED0006, per_rank, offset=rank * 1000)
    src = torch.from_numpy(((np.arange(per_rank) * 7 + rank) % len(ring)).astype(np.int32))
    owner = torch.full((per_rank,), -9, dtype=torch.int32)
    hops = torch.zeros(per_rank, dtype=torch.uint8)
    status = torch.full((per_rank,), 7, dtype=torch.uint8)
    eng = OracleArcEngine(P, len(ring))
    eng.region_cap = region_cap
    router = ArcRouter(eng, len(ring), rank, world, exchange_always=exchange_always)
    router.regions = regions
    router.chunks = chunks
    rounds = router.route(src, torch.from_numpy(keys.view(np.int64).copy()), owner, hops, status,
                          key_first=key_first, protocol=protocol)
    out[rank] = (owner.numpy().view(np.uint32).tolist(), hops.tolist(), status.tolist(), rounds,
                 router.records_sent)
    tdist.destroy_process_group()


@pytest.mark.parametrize("key_first,protocol,chunks", [
    (True, "records", None), (False, "records", None), (True, "soa", None), (True, "soa", 3)])
@pytest.mark.parametrize("world", [2, 3])
def test_arc_router_protocol_gloo(world, key_first, protocol, chunks):
    import oracle as O
    per_rank = 700
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_arc_worker, args=(world, _free_port(), per_rank, out, key_first,
                                          protocol, chunks),
                       nprocs=world, join=True, start_method="spawn")
    ring = O.ring_build(O.splitmix_keys(0x5EED0005, 3000))
    P = O.Peers(ring, O.fingers(ring))
    for r in range(world):
        keys = O.splitmix_keys(0x5EED0006, per_rank, offset=r * 1000)
        src = ((np.arange(per_rank) * 7 + r) % len(ring)).astype(np.uint32)
        ow, hp, st = O.route(P, src, keys)
        assert out[r][0] == ow.tolist() and out[r][1] == hp.tolist()
        assert out[r][2] == st.tolist()
        # records: walk -> result -> home, then drained; soa: there and back
        assert out[r][3] == (3 if protocol == "records" else 2)
        assert out[r][4] > 0            # records crossed ranks


@pytest.mark.parametrize("region_cap", [None, 5])
@pytest.mark.parametrize("world", [2, 3])
def test_arc_router_soa_regions_gloo(world, region_cap):
    """Single-pass partition into destination regions (the layout of
    cx_arc_partition_regions): answers land in their region slots and every
    lookup equals the oracle walk; region_cap = 5 overflows every piece and
    exercises the two-pass fallback."""
    import oracle as O
    per_rank = 600
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_arc_worker, args=(world, _free_port(), per_rank, out, True, "soa", 2,
                                          None, True, region_cap),
                       nprocs=world, join=True, start_method="spawn")
    ring = O.ring_build(O.splitmix_keys(0x5EED0005, 3000))
    P = O.Peers(ring, O.fingers(ring))
    for r in range(world):
        keys = O.splitmix_keys(0x5EED0006, per_rank, offset=r * 1000)
        src = ((np.arange(per_rank) * 7 + r) % len(ring)).astype(np.uint32)
        ow, hp, st = O.route(P, src, keys)
        assert out[r][0] == ow.tolist() and out[r][1] == hp.tolist()
        assert out[r][2] == st.tolist()


@pytest.mark.parametrize("chunks", [None, 3])
def test_arc_router_soa_uneven_batches_gloo(chunks):
    """Ranks with different batch sizes, one of them empty, run the same
    collectives (the piece count is agreed in the count all_gather) and every
    lookup still equals the oracle walk (route_soa hung when the
    local batch size chose the piece count)."""
    import oracle as O
    world, sizes = 3, [700, 0, 350]
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_arc_worker, args=(world, _free_port(), 0, out, True, "soa", chunks,
                                          sizes),
                       nprocs=world, join=True, start_method="spawn")
    ring = O.ring_build(O.splitmix_keys(0x5EED0005, 3000))
    P = O.Peers(ring, O.fingers(ring))
    for r in range(world):
        keys = O.splitmix_keys(0x5EED0006, sizes[r], offset=r * 1000)
        src = ((np.arange(sizes[r]) * 7 + r) % len(ring)).astype(np.uint32)
        ow, hp, st = O.route(P, src, keys) if sizes[r] else ([], [], [])
        assert out[r][0] == list(map(int, ow)) and out[r][1] == list(map(int, hp))
        assert out[r][2] == list(map(int, st))
        assert out[r][3] == 2


@pytest.mark.parametrize("regions", [False, True])
def test_arc_router_soa_world1_exchanges_with_itself_gloo(regions):
    """A one-rank group with exchange_always (bench.py's N = 1 arc leg):
    route_soa takes the general path -- partition, count all_gather, the
    all_to_alls to and from itself, delivery through the permutation or the
    region slots -- instead of the in-place walk, and every lookup equals the
    oracle walk."""
    import oracle as O
    per_rank = 500
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_arc_worker, args=(1, _free_port(), per_rank, out, True, "soa", 2,
                                          None, regions, None, True),
                       nprocs=1, join=True, start_method="spawn")
    ring = O.ring_build(O.splitmix_keys(0x5EED0005, 3000))
    P = O.Peers(ring, O.fingers(ring))
    keys = O.splitmix_keys(0x5EED0006, per_rank)
    src = ((np.arange(per_rank) * 7) % len(ring)).astype(np.uint32)
    ow, hp, st = O.route(P, src, keys)
    assert out[0][0] == ow.tolist() and out[0][1] == hp.tolist() and out[0][2] == st.tolist()
    assert out[0][3] == 2 and out[0][4] == per_rank  # two rounds, every lookup exchanged


def _succ_worker(rank, world, port, per_rank, out, exchange_always):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "p2p-dhts_amd"), os.path.join(root, "oracle"),
                    os.path.join(root, "tests")]
    import torch
    import torch.distributed as tdist
    import oracle as O
    from chordx import dist
    from chordx.arc import ArcRouter
    from test_multiproc import OracleArcEngine
    dist.init("gloo")
    if world == 1:
        assert dist.init_single("gloo")
    ring = O.ring_build(O.splitmix_keys(0x5EED0005, 3000))
    P = O.Peers(ring, O.fingers(ring, threads=2))
    keys = O.splitmix_keys(0x5EED0016, per_rank, offset=rank * per_rank)
    # keys at and around peer IDs, and past the last peer (owner: peer 0)
    keys[:40] = ring[(np.arange(40) * 71) % len(ring)]
    keys[40] = np.array([2**64 - 1, 2**64 - 1], dtype=np.uint64)
    owner = torch.full((per_rank,), -9, dtype=torch.int32)
    router = ArcRouter(OracleArcEngine(P, len(ring)), len(ring), rank, world,
                       exchange_always=exchange_always)
    rounds = router.successor(torch.from_numpy(keys.view(np.int64).copy()), owner)
    out[rank] = (owner.numpy().view(np.uint32).tolist(), rounds, router.records_sent)
    tdist.destroy_process_group()


@pytest.mark.parametrize("world,exchange_always", [(1, True), (2, False), (3, False)])
def test_arc_exact_successor_gloo(world, exchange_always):
    """Exact-successor mode of the arc layout: keys bucketed by
    their owner's arc, all_to_all-v, searched against that rank's arc of the
    ring only, owners back -- equal to the oracle's StoredLocally answer."""
    import oracle as O
    per_rank = 400
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_succ_worker, args=(world, _free_port(), per_rank, out, exchange_always),
                       nprocs=world, join=True, start_method="spawn")
    ring = O.ring_build(O.splitmix_keys(0x5EED0005, 3000))
    for r in range(world):
        keys = O.splitmix_keys(0x5EED0016, per_rank, offset=r * per_rank)
        keys[:40] = ring[(np.arange(40) * 71) % len(ring)]
        keys[40] = np.array([2**64 - 1, 2**64 - 1], dtype=np.uint64)
        assert out[r][0] == O.successor(ring, keys).tolist()
        assert out[r][0][40] == 0
        assert out[r][1] == 2 and out[r][2] == per_rank


def test_bench_launches_n_ranks_itself():
    """`bench.py --gpus 2` without torchrun starts torch.distributed.run as a
    child and rank 0 of that job reports n_gpus = 2 (CX_BENCH_DRYRUN: the
    launch / rendezvous / barrier / max-over-ranks flow without a GPU)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(CX_BENCH_DRYRUN="1", CX_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1", "--cpu-seconds", "1"], env=env,
                       capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 3 and rec["warmup"] == 1
    # every world size carries the CPU baseline (rank 0) and the whole-node roofline
    assert rec["cpu_baseline"] is not None and rec["cpu_baseline"]["value"] > 0
    assert rec["cpu_baseline"]["n_gpus_beside"] == 2
    # the oracle sample's hop histogram: one bin per hop count
    hist = rec["cpu_baseline"]["hops_hist"]
    assert hist[0] >= 0 and sum(hist) > 0 and hist[-1] > 0
    assert rec["roofline"]["n_gpus"] == 2 and rec["roofline"]["peak"] == 2 * 8000.0


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0", CX_BENCH_DRYRUN="1")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


# ---------------------------------------------------------------------------
# C5 key-sharded over ranks (benches/bench_c5.py's layout): replicated old/new
# rings, each rank scans its dist.shard_range of the keys; the concatenation
# (dist.gather_rows) must equal the single-process RunGlobalMaintenance scan.
# ---------------------------------------------------------------------------
def _c5_worker(rank, world, port, total, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "p2p-dhts_amd"), os.path.join(root, "oracle")]
    import torch
    import torch.distributed as tdist
    import oracle as O
    from chordx import dist
    dist.init("gloo")
    old = O.ring_build(O.splitmix_keys(0x5EED0007, 4000))
    joins = O.splitmix_keys(0x5EED0009, 40)
    leaves = old[(np.arange(40) * 0x9E3779B1) % len(old)]
    new, o2n = O.churn(old, joins, leaves)
    k0, k1 = dist.shard_range(rank, world, total)
    keys = O.splitmix_keys(0x5EED0008, k1 - k0, offset=k0)
    lists, count, mask, target = O.misplaced(old, new, o2n, keys, 14, threads=2)
    got = [dist.gather_rows(torch.from_numpy(a.astype(np.int64)), world, "gloo").numpy()
           for a in (lists, count, mask, target)]
    out[rank] = [g.tolist() for g in got] + [(k0, k1)]
    tdist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 3001), (3, 2000)])
def test_c5_key_sharded_scan_equals_single_process(world, total):
    import oracle as O
    mgr = mp.Manager()
    out = mgr.dict()
    mp.start_processes(_c5_worker, args=(world, _free_port(), total, out), nprocs=world,
                       join=True, start_method="spawn")
    old = O.ring_build(O.splitmix_keys(0x5EED0007, 4000))
    joins = O.splitmix_keys(0x5EED0009, 40)
    leaves = old[(np.arange(40) * 0x9E3779B1) % len(old)]
    new, o2n = O.churn(old, joins, leaves)
    keys = O.splitmix_keys(0x5EED0008, total)
    want = O.misplaced(old, new, o2n, keys, 14)
    spans = [out[r][4] for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    assert all(spans[r][1] == spans[r + 1][0] for r in range(world - 1))
    for r in range(world):  # every rank holds the whole concatenation
        for g, w in zip(out[r][:4], want):
            assert np.array_equal(np.asarray(g).reshape(w.shape), w.astype(np.int64))
    assert 0 < int((want[2] != 0).sum()) < total
