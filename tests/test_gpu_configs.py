"""BASELINE configs C4 (per GPU) and C5 at their full sizes on the GPU.

C4 per GPU: the headline workload -- 2^24-peer ring (seed 0x5EED0005), 2^25
keys (seed 0x5EED0006), src = q mod N, the default route kernel.
  * every lookup: status OK and owner == exact successor (lower_bound with
    wrap, StoredLocally's converged answer, abstract_chord_peer.cpp:720-725);
  * owner and hops == the oracle's literal ForwardRequest walk
    (oracle/chord_oracle.c or_route, chord_peer.cpp:185-211) on a 2^20-key
    sample, over the engine's finger table;
  * that finger table == the oracle's PopulateFingerTable restatement
    (or_fingers_rows, abstract_chord_peer.cpp:564-613) on every row.
C5: 2^24-peer ring (seed 0x5EED0007), 2^26 keys (seed 0x5EED0008), n = 14,
1 % joins + 1 % leaves (seed 0x5EED0009, leaves chosen by index):
  * churned ring and old->new map == the oracle's;
  * new lists, counts, misplaced masks and transfer targets == the oracle's
    RunGlobalMaintenance restatement (dhash_peer.cpp:298-348) on ALL keys;
  * n-successor lists on the old ring == the successor window on all keys.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

N4, Q4 = 1 << 24, 1 << 25


@pytest.fixture(scope="module")
def c4(O):
    import torch

    import chordx
    ids = torch.empty((N4, 2), dtype=torch.int64, device="cuda:0")
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    del ids
    ring.build_fingers()
    ring.sync()
    keys = torch.empty((Q4, 2), dtype=torch.int64, device="cuda:0")
    chordx.fill_splitmix(keys, 0x5EED0006)
    src = (torch.arange(Q4, device="cuda:0", dtype=torch.int64) % ring.n).to(torch.int32)
    owner, hops, status = ring.route(src, keys)
    torch.cuda.synchronize()
    yield ring, keys, src, owner, hops, status
    del ring
    torch.cuda.empty_cache()


def test_c4_every_lookup_reaches_the_successor(c4):
    import torch
    ring, keys, src, owner, hops, status = c4
    assert ring.n == N4  # no duplicate IDs among 2^24 splitmix values
    assert ring.route_info()[0] == 5  # the default (benchmarked) kernel
    assert int((status != 0).sum()) == 0
    succ = ring.successor(keys)
    torch.cuda.synchronize()
    assert bool((owner == succ).all())
    mean = float(hops.double().mean())
    assert 11.5 < mean < 12.3  # ~ log2(N)/2 on a uniform ring


@pytest.fixture(scope="module")
def c4_host(O, c4):
    """The oracle's C4 ring and the engine's finger table on the host."""
    ring = c4[0]
    want_ring = O.ring_build(O.splitmix_keys(0x5EED0005, N4))
    F = ring.fingers_device().cpu().numpy().view(np.uint32)
    return want_ring, F


def test_c4_oracle_walk_and_fingers_on_samples(O, c4, c4_host):
    ring, keys, src, owner, hops, status = c4
    want_ring, F = c4_host
    ids = ring.ids()
    assert (ids == want_ring).all()
    # the whole 2^24 x 128 table, in 2^21-row pieces (bounded host memory)
    step = 1 << 21
    for p0 in range(0, N4, step):
        assert (F[p0:p0 + step] == O.fingers(want_ring, rows=(p0, p0 + step))).all(), p0
    sample = 1 << 20
    kh = keys[:sample].cpu().numpy().view(np.uint64)
    sh = src[:sample].cpu().numpy().view(np.uint32)
    wo, wh, ws = O.route(O.Peers(want_ring, F), sh, kh)
    assert (ws == 0).all()
    assert (owner[:sample].cpu().numpy().view(np.uint32) == wo).all()
    assert (hops[:sample].cpu().numpy() == wh).all()


@pytest.mark.parametrize("d", [0, 3, 7])
def test_c4_arc_layout_g8(O, c4, c4_host, d):
    """C4 as BASELINE.json states it, on one GPU: the 2^24 ring's arc layout for
    G = 8 ranks (top levels replicated, lower levels for the arc + its 2^122
    halo), rank d's received lookups -- the pieces that cx_arc_partition of
    each of the 8 origin ranks' 2^22 C4 keys sends to d -- walked by
    cx_arc_route and delivered by cx_arc_deliver: owner / hops / status equal
    the replicated cx_route's on every received lookup, and the oracle's
    literal walk (chord_peer.cpp:185-211) on a 2^18 sample.  Then the same for
    the default path: cx_arc_partition_regions with source hints, the hinted
    walk (cx_arc_route_hinted) and delivery through each origin's region slots."""
    import torch
    ring, keys, src, owner, hops, status = c4
    want_ring, F = c4_host
    G, per = 8, 1 << 22
    ring.arc_build(G, d)
    top, rows, plane_bytes = ring.arc_info()
    assert top == 6 and N4 // G < rows < N4 // G + N4 // 32  # the arc plus its halo
    rk, rs, total = [], [], 0
    for r in range(G):
        sl = slice(r * per, (r + 1) * per)
        sk, ss, perm, counts = ring.arc_partition(G, src[sl], keys[sl])
        assert sum(counts) == per
        assert torch.equal(torch.sort(perm.long()).values, torch.arange(per, device="cuda:0"))
        off = sum(counts[:d])
        rk.append(sk[off:off + counts[d]])
        rs.append(ss[off:off + counts[d]])
        total += counts[d]
    rk, rs = torch.cat(rk), torch.cat(rs)
    assert abs(total - per) < per // 50  # about an eighth of 2^25 lookups
    # every received key's owner lies in arc d
    lo, hi = d * N4 // G, (d + 1) * N4 // G
    succ = ring.successor(rk)
    assert bool(((succ >= lo) & (succ < hi)).all())
    res = ring.arc_route(rs, rk)
    ao = torch.full((total,), -7, dtype=torch.int32, device="cuda:0")
    ah = torch.full((total,), 77, dtype=torch.uint8, device="cuda:0")
    ast = torch.full((total,), 9, dtype=torch.uint8, device="cuda:0")
    ring.arc_deliver(res, None, ao, ah, ast)
    wo, wh, ws = ring.route(rs, rk)
    torch.cuda.synchronize()
    assert torch.equal(ao, wo) and torch.equal(ah, wh) and torch.equal(ast, ws)
    assert int((ast != 0).sum()) == 0 and torch.equal(ao, succ)
    sample = 1 << 18
    oo, oh, os_ = O.route(O.Peers(want_ring, F), rs[:sample].cpu().numpy().view(np.uint32),
                          rk[:sample].cpu().numpy().view(np.uint64))
    assert (os_ == 0).all()
    assert (ao[:sample].cpu().numpy().view(np.uint32) == oo).all()
    assert (ah[:sample].cpu().numpy() == oh).all()

    # ---- the default path (ArcRouter.route_soa, what bench.py and SCALE run):
    # single-pass region partition with origin-resolved source hints
    # (gs = 116 - ceil(log2 N) depends on the ring size), the hinted arc walk,
    # and delivery through the region slots back at each origin
    hk, hs, hh, slots = [], [], [], []
    for r in range(G):
        sl = slice(r * per, (r + 1) * per)
        cap = per // G + per // (4 * G) + 4096  # route_soa's region capacity
        part = ring.arc_partition_regions(G, src[sl], keys[sl], cap, hints=True)
        assert part is not None  # uniform keys never crowd one arc past cap
        sk, ss, perm, counts, sh = part
        assert sum(counts) == per and max(counts) <= cap
        r0 = d * cap
        hk.append(sk[r0:r0 + counts[d]])
        hs.append(ss[r0:r0 + counts[d]])
        hh.append(sh[r0:r0 + counts[d]])
        slots.append((perm, counts[d], cap))
    assert sum(x.shape[0] for x in hk) == total  # the same lookups reach rank d
    hk, hs, hh = torch.cat(hk), torch.cat(hs), torch.cat(hh)
    hres = ring.arc_route(hs, hk, hint=hh)
    wo, wh, ws = ring.route(hs, hk)
    ho = torch.full((total,), -7, dtype=torch.int32, device="cuda:0")
    hh8 = torch.full((total,), 77, dtype=torch.uint8, device="cuda:0")
    hst = torch.full((total,), 9, dtype=torch.uint8, device="cuda:0")
    ring.arc_deliver(hres, None, ho, hh8, hst)
    torch.cuda.synchronize()
    assert torch.equal(ho, wo) and torch.equal(hh8, wh) and torch.equal(hst, ws)
    assert int((hst != 0).sum()) == 0
    oo, oh, os_ = O.route(O.Peers(want_ring, F), hs[:sample].cpu().numpy().view(np.uint32),
                          hk[:sample].cpu().numpy().view(np.uint64))
    assert (os_ == 0).all()
    assert (ho[:sample].cpu().numpy().view(np.uint32) == oo).all()
    assert (hh8[:sample].cpu().numpy() == oh).all()
    # delivery at each origin r: the answers of region d land at the slots perm
    # names, and every lookup of origin r that went to d gets its own answer
    # (lookups sent elsewhere read other regions, filled with a sentinel here)
    off = 0
    for r, (perm, cnt, cap) in enumerate(slots):
        back = torch.zeros(G * cap, dtype=torch.int64, device="cuda:0")
        back[d * cap: d * cap + cnt] = hres[off:off + cnt]
        off += cnt
        o = torch.empty(per, dtype=torch.int32, device="cuda:0")
        h = torch.empty(per, dtype=torch.uint8, device="cuda:0")
        st = torch.empty(per, dtype=torch.uint8, device="cuda:0")
        ring.arc_deliver(back, perm, o, h, st)
        mine = (perm.long() >= d * cap) & (perm.long() < d * cap + cnt)
        assert int(mine.sum()) == cnt
        sl = slice(r * per, (r + 1) * per)
        assert torch.equal(o[mine], owner[sl][mine]) and torch.equal(h[mine], hops[sl][mine])
        assert int((st[mine] != 0).sum()) == 0


def test_c5_full_size_churn_and_misplaced_scan(O):
    import torch

    import chordx
    N5, q, n = 1 << 24, 1 << 26, 14
    ids = O.splitmix_keys(0x5EED0007, N5)
    want_old = O.ring_build(ids)
    old = chordx.Ring(ids)
    assert old.n == len(want_old)
    rng = np.random.default_rng(0x5EED0009)
    leaves = want_old[rng.choice(len(want_old), N5 // 100, replace=False)]
    joins = O.splitmix_keys(0x5EED0009, N5 // 100)
    new, o2n = old.churn(joins, leaves)
    want_new, want_o2n = O.churn(want_old, joins, leaves)
    assert (new.ids() == want_new).all() and (o2n == want_o2n).all()

    # n-successor windows on the old ring, every key (device-side property)
    keys_d = torch.empty((q, 2), dtype=torch.int64, device="cuda:0")
    chordx.fill_splitmix(keys_d, 0x5EED0008)
    lists_d, count_d = old.nsucc(keys_d, n)
    succ = old.successor(keys_d).to(torch.int64)
    want = (succ[:, None] + torch.arange(n, device="cuda:0")) % old.n
    torch.cuda.synchronize()
    assert bool((lists_d.to(torch.int64) == want).all()) and bool((count_d == n).all())
    del keys_d, lists_d, count_d, succ, want

    keys = O.splitmix_keys(0x5EED0008, q)
    lists, count, mask, target = old.misplaced(new, o2n, keys, n)
    wl, wc, wm, wt = O.misplaced(want_old, want_new, want_o2n, keys, n)
    assert (count == wc).all() and (mask == wm).all()
    assert (lists == wl).all() and (target == wt).all()
    assert 0 < int((mask != 0).sum()) < q
    del lists, count, mask, target
    # the fused step (bench_c5's): old lists = the old ring's window, the rest
    # = the scan's outputs (all 2^26 keys)
    keys_d = torch.from_numpy(keys.view(np.int64)).cuda()
    o2n_d = torch.from_numpy(o2n.view(np.int32)).cuda()
    ol, oc, nl, nc, nm, nt = old.dhash_maintenance(new, o2n_d, keys_d, n)
    succ = old.successor(keys_d).to(torch.int64)
    want = (succ[:, None] + torch.arange(n, device="cuda:0")) % old.n
    assert bool((ol.to(torch.int64) == want).all()) and bool((oc == n).all())
    del want, succ
    assert (nl.cpu().numpy().view(np.uint32) == wl).all()
    assert (nc.cpu().numpy() == wc).all() and (nm.cpu().numpy().view(np.uint16) == wm).all()
    assert (nt.cpu().numpy() == wt).all()
