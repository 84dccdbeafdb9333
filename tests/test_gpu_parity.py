"""Parity of the HIP engine (through the C ABI) against the CPU oracle.

Bit-exact integer comparisons throughout: owner indices, hop counts, finger
tables, replica lists, misplaced masks and transfer targets.  Sizes are chosen
so the oracle finishes in seconds; full BASELINE sizes are covered by
size-independent properties (test_gpu_fullsize.py).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

H = lambda s: int(s, 16)  # noqa: E731
MAX = (1 << 128) - 1


@pytest.fixture(scope="module")
def cx():
    import chordx
    if chordx.device_count() == 0:
        pytest.fail("gpu test without a HIP device")
    return chordx


def edge_ring(O, n, seed):
    """Random IDs plus the ring's edge values and adjacent pairs."""
    base = O.ints_from_keys(O.splitmix_keys(seed, n))
    if n <= 3:  # keep tiny rings tiny (N = 1, 2, 3 edge cases)
        return O.keys_from_ints(base)
    extra = [0, 1, MAX, MAX - 1, base[0] + 1, base[1] - 1, 1 << 127, (1 << 127) - 1]
    return O.keys_from_ints([v % (1 << 128) for v in base + extra])


def edge_keys(O, ring, seed, q):
    ids = O.ints_from_keys(ring)
    vals = O.ints_from_keys(O.splitmix_keys(seed, q))
    for v in ids[:64]:
        vals += [v, (v + 1) % (1 << 128), (v - 1) % (1 << 128)]
    vals += [0, 1, MAX, MAX - 1]
    return O.keys_from_ints(vals)


# ---------------------------------------------------------------- a13 ring build
@pytest.mark.parametrize("n", [1, 2, 3, 5, 1000, 4097, 70000])
def test_ring_build(cx, O, n):
    ids = O.splitmix_keys(1000 + n, n)
    if n > 3:  # duplicates must be dropped (remote_peer_list.cpp:56-58)
        ids = np.concatenate([ids, ids[: n // 3], O.keys_from_ints([0, MAX, 0])])
    ring = cx.Ring(ids)
    want = O.ring_build(ids)
    assert ring.n == len(want)
    assert (ring.ids() == want).all()


def test_ring_build_equal_high_bits(cx, O):
    """Keys that differ only in low bits / only in high bits (radix passes)."""
    v = [(7 << 100) + i for i in range(300)] + [(i << 120) for i in range(200)] + [5] * 10
    ids = O.keys_from_ints(v)
    assert (cx.Ring(ids).ids() == O.ring_build(ids)).all()


@pytest.mark.parametrize("kind", ["uniform", "cluster", "mixed", "dups"])
def test_ring_build_sort_paths(cx, O, kind):
    """Round 6 ring sort (cx_kernels.hip radix_sort): MSD buckets of ~256 keys
    sorted in LDS by (key, tag), and the LSD fallback (4 tag + 16 key passes)
    when a bucket passes 2048 keys.  uniform: the bucket path; cluster: one
    bucket holds everything (fallback); mixed: uniform keys plus a dense run
    in one bucket (fallback with most buckets already written); dups: many
    equal keys (the kept duplicate is the first by input order)."""
    rng = np.random.default_rng(0x50E7)
    if kind == "uniform":
        vals = O.ints_from_keys(O.splitmix_keys(0x50E8, 1 << 17))
    elif kind == "cluster":
        base = 0x3C3C_5A5A_0F0F_1234 << 64
        vals = [base + int(x) * 7919 for x in rng.permutation(6000)]
    elif kind == "mixed":
        vals = O.ints_from_keys(O.splitmix_keys(0x50E9, 1 << 16))
        vals += [(0x1234 << 112) + int(x) for x in rng.permutation(5000)]
    else:
        u = O.ints_from_keys(O.splitmix_keys(0x50EA, 3000))
        vals = [u[int(i)] for i in rng.integers(0, 3000, size=40000)]
    ids = O.keys_from_ints(vals)
    ring = cx.Ring(ids)
    assert (ring.ids() == O.ring_build(ids)).all()
    import torch
    from chordx.ring import sort_time
    d = torch.from_numpy(ids.view(np.int64).copy()).cuda()
    for variant in (0, 1):
        _, ok = sort_time(d, variant)
        assert ok, variant


# ---------------------------------------------------------------- a5/a7 successor
@pytest.mark.parametrize("search", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("n", [1, 2, 3, 8, 16, 17, 256, 257, 1000, 4095, 4096, 65537, 70000,
                               100000])
def test_successor(cx, O, n, search):
    ids = edge_ring(O, n, 77 + n)
    ring = cx.Ring(ids)
    ring.set_search_variant(search)
    want_ring = O.ring_build(ids)
    keys = edge_keys(O, want_ring, 5 + n, 20000)
    got = ring.successor(keys)
    assert (got == O.successor(want_ring, keys)).all()


@pytest.mark.parametrize("search", [0, 1, 2, 3, 4, 5])
def test_successor_c2(cx, O, search):
    """Config C2: 2^16-peer ring, 2^20 uniform keys (seeds of SURVEY 8d).
    Variant 1 takes the LDS slice table here (2^20 >= 4 n), 5 the directory."""
    ids = O.splitmix_keys(0x5EED0001, 1 << 16)
    keys = O.splitmix_keys(0x5EED0002, 1 << 20)
    ring = cx.Ring(ids)
    ring.set_search_variant(search)
    assert (ring.successor(keys) == O.successor(O.ring_build(ids), keys)).all()


@pytest.mark.parametrize("n", [75000, 79000, 81000])
def test_successor_lds_slice_table_fit_boundary(cx, O, n):
    """Rings at the LDS limit: 75 000 peers take b = 11, 79 000 b = 10 (the
    smallest allowed), 81 000 do not fit and search the directory; variant 1
    with >= 4 n keys and variant 4 give the oracle's answers either way."""
    ids = edge_ring(O, n, 0x51DA + n)
    want_ring = O.ring_build(ids)
    keys = edge_keys(O, want_ring, 0x51DB, 4 * n + 10)
    want = O.successor(want_ring, keys)
    for search in (4, 1):
        ring = cx.Ring(ids)
        ring.set_search_variant(search)
        assert (ring.successor(keys) == want).all(), search
        assert (ring.predecessor(keys[:5000]) == O.predecessor(want_ring, keys[:5000])).all()


def test_successor_lds_slice_table_concurrent_first_searches(cx, O):
    """Four host threads make the first slice-table searches of a ring at once
    (the table is built lazily by the first): every answer equals the oracle."""
    import threading
    ids = O.splitmix_keys(0x51D8, 50000)
    want_ring = O.ring_build(ids)
    keys = [O.splitmix_keys(0x51D9 + i, 1 << 16) for i in range(4)]
    for rep in range(3):
        ring = cx.Ring(ids)
        ring.set_search_variant(4)
        out, errs = [None] * 4, []

        def run(i):
            try:
                out[i] = ring.successor(keys[i])
            except Exception as e:  # pragma: no cover
                errs.append(e)

        th = [threading.Thread(target=run, args=(i,)) for i in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs
        for i in range(4):
            assert (out[i] == O.successor(want_ring, keys[i])).all(), (rep, i)


def test_successor_lds_slice_table_churned_ring(cx, O):
    """A ring from cx_churn builds its own slice table (lazily, from its own
    IDs): successor / predecessor through the table on the parent and on two
    chained churns equal the oracle on each ring, with the parent's table
    built first (stale tables must not travel with the search variant)."""
    ids = O.splitmix_keys(0x51D5, 30000)
    keys = O.splitmix_keys(0x51D6, 1 << 17)
    ring = cx.Ring(ids)
    ring.set_search_variant(4)
    want = O.ring_build(ids)
    assert (ring.successor(keys) == O.successor(want, keys)).all()
    for e in range(2):
        joins = O.splitmix_keys(0x51D7 + e, 3000)
        leaves = want[::7]
        new, _ = ring.churn(joins, leaves)
        want, _ = O.churn(want, joins, leaves)
        assert (new.ids() == want).all()
        new.set_search_variant(4)
        assert (new.successor(keys) == O.successor(want, keys)).all()
        assert (new.predecessor(keys) == O.predecessor(want, keys)).all()
        ring = new


@pytest.mark.parametrize("pred", [False, True])
@pytest.mark.parametrize("kind", ["cluster", "cluster_big", "runs", "tiny_gaps"])
def test_successor_lds_slice_table(cx, O, kind, pred):
    """The LDS slice table (search variants 4 and 1) where its slices cannot
    decide: a ring whose IDs share their top 40+ bits (one bucket, one run of
    equal slices: the full-ID binary search; with 40 000 such IDs the int16
    offset deviations overflow and the uint32 table is used), runs of IDs sharing the key's top
    b + 16 bits beside uniform ones, and IDs 1 apart; keys at, next to and
    between them.  Variant 1 at >= 4 n keys takes the same table."""
    rng = np.random.default_rng(0x51CE)
    if kind == "cluster":
        base = 0x0123_4567_89AB << 80
        vals = [base + (int(x) << 20) for x in rng.permutation(1 << 14)]
    elif kind == "cluster_big":  # offsets past int16 deviations: the uint32 table
        base = 0x0123_4567_89AB << 80
        vals = [base + (int(x) << 20) for x in rng.permutation(40000)]
    elif kind == "runs":
        vals = O.ints_from_keys(O.splitmix_keys(0x51CF, 20000))
        for j in range(40):
            top = O.ints_from_keys(O.splitmix_keys(0x51D0 + j, 1))[0] >> 100 << 100
            vals += [top + (int(x) << 40) for x in rng.permutation(300)]
    else:
        start = O.ints_from_keys(O.splitmix_keys(0x51D1, 1))[0]
        vals = [(start + i) % (1 << 128) for i in range(5000)]
        vals += O.ints_from_keys(O.splitmix_keys(0x51D2, 5000))
    ids = O.keys_from_ints(vals)
    want_ring = O.ring_build(ids)
    keys = edge_keys(O, want_ring, 0x51D3, 1 << 16)
    w = O.ints_from_keys(want_ring)
    near = [(w[int(i)] + int(d)) % (1 << 128) for i, d in
            zip(rng.integers(0, len(w), 4000), rng.integers(-3, 4, 4000))]
    keys = np.concatenate([keys, O.keys_from_ints(near)])
    want = (O.predecessor if pred else O.successor)(want_ring, keys)
    for search in (4, 1, 5):
        ring = cx.Ring(ids)
        ring.set_search_variant(search)
        got = ring.predecessor(keys) if pred else ring.successor(keys)
        assert (got == want).all(), search


# ---------------------------------------------------------------- a6 fingers
@pytest.mark.parametrize("search", [0, 1])
@pytest.mark.parametrize("n", [1, 2, 3, 17, 1000, 5000])
def test_fingers(cx, O, n, search):
    ids = edge_ring(O, n, 300 + n)
    ring = cx.Ring(ids)
    ring.set_search_variant(search)
    F = ring.build_fingers(copy_out=True)
    assert (F == O.fingers(O.ring_build(ids))).all()


def test_fingers_c2_ring(cx, O):
    ids = O.splitmix_keys(0x5EED0001, 1 << 16)
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    assert (F == O.fingers(O.ring_build(ids))).all()


# ---------------------------------------------------------------- a7-a9 route
@pytest.mark.parametrize("variant", [0, 4, 5])
def test_route_c1_golden(cx, O, c1truth, variant):
    """Config C1 ground truth (8 peers, key0..key999 from every peer)."""
    ids = O.keys_from_ints([O.uuid5_key(p) for p in c1truth["peers"]])
    ring = cx.Ring(ids)
    ring.set_route_variant(variant)
    assert [format(v, "x") for v in O.ints_from_keys(ring.ids())] == c1truth["ring"]
    ring.build_fingers()
    kv = O.keys_from_ints([O.uuid5_key(k) for k in c1truth["keys"]])
    src = np.repeat(np.arange(8, dtype=np.uint32), len(kv))
    owner, hops, status = ring.route(src, np.tile(kv, (8, 1)))
    assert owner.tolist() == c1truth["owner"]
    assert hops.tolist() == c1truth["hops"]
    assert (status == 0).all()


@pytest.mark.parametrize("variant", [0, 4, 5])
@pytest.mark.parametrize("n", [1, 2, 3, 9, 1000, 20000])
def test_route_converged(cx, O, n, variant):
    ids = edge_ring(O, n, 900 + n)
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    ring.set_route_variant(variant)
    want_ring = O.ring_build(ids)
    keys = edge_keys(O, want_ring, 31 + n, 30000)
    rng = np.random.default_rng(n)
    src = rng.integers(0, len(want_ring), len(keys)).astype(np.uint32)
    owner, hops, status = ring.route(src, keys)
    P = O.Peers(want_ring, F)
    wo, wh, ws = O.route(P, src, keys)
    assert (owner == wo).all() and (hops == wh).all() and (status == ws).all()
    assert (owner == O.successor(want_ring, keys)).all()


@pytest.mark.parametrize("q", [1, 2, 63, 64, 65, 1023, 1025, 4097, 70001, 458753, 917507])
def test_route_batch_sizes_write_exactly_q(cx, O, q):
    """The default walk stores each lookup's outputs as it finishes (no result
    ring): every batch size writes owner / hops / status of exactly its q
    lookups -- equal to the oracle -- and nothing past them.  Sizes cover one
    lookup per wave, partial waves, and the switch to one resident round of
    waves (>= 64 lookups per wave: 7 x 4 x 256 waves fill at 458752)."""
    import torch
    ids = O.splitmix_keys(0xBA7C, 20000)
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    assert ring.route_info()[0] == 5
    want_ring = O.ring_build(ids)
    keys = edge_keys(O, want_ring, 0xBA7D, q)[:q]
    src = (np.arange(q) * 7919 % len(want_ring)).astype(np.uint32)
    kd = torch.from_numpy(keys.view(np.int64).copy()).cuda()
    sd = torch.from_numpy(src.view(np.int32).copy()).cuda()
    pad = 300
    owner = torch.full((q + pad,), -9, dtype=torch.int32, device="cuda")
    hops = torch.full((q + pad,), 201, dtype=torch.uint8, device="cuda")
    status = torch.full((q + pad,), 77, dtype=torch.uint8, device="cuda")
    ring.route(sd, kd, out=(owner[:q], hops[:q], status[:q]))
    torch.cuda.synchronize()
    wo, wh, ws = O.route(O.Peers(want_ring, F), src, keys)
    assert (owner[:q].cpu().numpy().view(np.uint32) == wo).all()
    assert (hops[:q].cpu().numpy() == wh).all() and (status[:q].cpu().numpy() == ws).all()
    assert bool((owner[q:] == -9).all()) and bool((hops[q:] == 201).all())
    assert bool((status[q:] == 77).all())


def test_route_from_predecessor(cx, O, refvec):
    """ChordGetSucc.FromPredecessor: all fingers of the source point at itself."""
    g = refvec["get_succ"]["from_predecessor"]
    ids = O.keys_from_ints([H(x) for x in g["peers"]])
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    names = [format(v, "x") for v in O.ints_from_keys(ring.ids())]
    s = names.index(g["src"])
    F[s, :] = s
    ring.upload_fingers(F)
    owner, hops, status = ring.route(np.array([s], np.uint32), O.keys_from_ints([H(g["key"])]))
    assert owner[0] == (s - 1) % 2 and hops[0] == 1 and status[0] == 0


def test_route_local_key_custom_min_key(cx, O, refvec):
    g = refvec["get_succ"]["local_key"]
    ring = cx.Ring(O.keys_from_ints([H(g["peer"])]))
    ring.build_fingers()
    ring.upload_peer_state(min_keys=O.keys_from_ints([H(g["min_key"])]))
    owner, hops, status = ring.route(np.array([0], np.uint32), O.keys_from_ints([H(g["key"])]))
    assert owner[0] == 0 and hops[0] == 0 and status[0] == 0


def test_route_from_finger_table(cx, O, refvec):
    g = refvec["get_succ"]["from_finger_table"]
    ring = cx.Ring(O.keys_from_ints([H(x) for x in g["peers"]]))
    ring.build_fingers()
    names = [format(v, "x") for v in O.ints_from_keys(ring.ids())]
    owner, hops, _ = ring.route(np.array([names.index(g["src"])], np.uint32),
                                O.keys_from_ints([H(g["key"])]))
    assert names[owner[0]] == g["expected"] and hops[0] == 1


def clustered_ring(O, n, seed, spread_bits):
    """IDs packed within 2^spread_bits of a few centres: every packed-ID
    interval straddles decisions, forcing the exact-ID fallbacks of the table walks."""
    rng = np.random.default_rng(seed)
    centres = [int.from_bytes(rng.bytes(16), "big") for _ in range(4)] + [MAX - 5, 3]
    vals = []
    for j in range(n):
        c = centres[j % len(centres)]
        off = int.from_bytes(rng.bytes(16), "big") >> (128 - spread_bits)
        vals.append((c + off) % (1 << 128))
    return O.keys_from_ints(vals)


@pytest.mark.parametrize("search", [0, 1])
@pytest.mark.parametrize("spread", [8, 40, 100])
def test_successor_clustered_rings(cx, O, search, spread):
    """Skewed rings: whole clusters inside one directory bucket (binary-search path)."""
    ids = clustered_ring(O, 5000, spread, spread)
    ring = cx.Ring(ids)
    ring.set_search_variant(search)
    want_ring = O.ring_build(ids)
    keys = edge_keys(O, want_ring, spread, 20000)
    ints = O.ints_from_keys(want_ring)
    rng = np.random.default_rng(spread)
    near = O.keys_from_ints([(ints[j] + int(rng.integers(-2, 3))) % (1 << 128)
                             for j in rng.integers(0, len(ints), 20000)])
    keys = np.concatenate([keys, near])
    assert (ring.successor(keys) == O.successor(want_ring, keys)).all()
    lists, count = ring.nsucc(keys, 14)
    wl, wc = O.nsucc(O.Peers(want_ring, O.fingers(want_ring)), keys, 14)
    assert (lists == wl).all() and (count == wc).all()


@pytest.mark.parametrize("variant", [0, 4, 5])
@pytest.mark.parametrize("spread", [8, 40, 90, 100])
def test_route_clustered_rings(cx, O, variant, spread):
    ids = clustered_ring(O, 3000, spread, spread)
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    ring.set_route_variant(variant)
    want_ring = O.ring_build(ids)
    ints = O.ints_from_keys(want_ring)
    rng = np.random.default_rng(spread)
    # keys right next to peer IDs + random keys + keys inside the clusters
    kv = [(ints[j] + int(rng.integers(-3, 4))) % (1 << 128) for j in rng.integers(0, len(ints), 6000)]
    kv += O.ints_from_keys(O.splitmix_keys(spread, 6000))
    kv += [(ints[j] + (int.from_bytes(rng.bytes(16), "big") >> (128 - spread))) % (1 << 128)
           for j in rng.integers(0, len(ints), 6000)]
    keys = O.keys_from_ints(kv)
    src = rng.integers(0, len(ints), len(keys)).astype(np.uint32)
    owner, hops, status = ring.route(src, keys)
    wo, wh, ws = O.route(O.Peers(want_ring, F), src, keys)
    assert (owner == wo).all() and (hops == wh).all() and (status == ws).all()


def test_route_default_variant_and_escapes(cx, O):
    """Automatic variant: the pattern-keyed window table (5) up to 2^24 peers.
    A uniform ring encodes every node; a clustered one cannot (large index
    jumps, huge gaps) and still routes exactly through the fallbacks."""
    ring = cx.Ring(O.splitmix_keys(77, 20000))
    ring.build_fingers()
    v, esc, nbytes = ring.route_info()
    assert v == 5 and esc == 0 and nbytes == 20000 * 24 * 128  # R = 15 + 8 -> 24
    ids = clustered_ring(O, 3000, 5, 8)
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    v, esc, _ = ring.route_info()
    assert v == 5 and esc > 0
    want_ring = O.ring_build(ids)
    keys = O.splitmix_keys(78, 5000)
    src = np.random.default_rng(5).integers(0, len(want_ring), len(keys)).astype(np.uint32)
    owner, hops, status = ring.route(src, keys)
    wo, wh, ws = O.route(O.Peers(want_ring, F), src, keys)
    assert (owner == wo).all() and (hops == wh).all() and (status == ws).all()


def test_route_literal_random_edits(cx, O):
    """Hand-edited fingers + custom preds/min_keys: literal ForwardRequest walk,
    including hop-cap (self-loops with no live predecessor)."""
    rng = np.random.default_rng(42)
    ids = O.splitmix_keys(4242, 300)
    ring = cx.Ring(ids)
    want_ring = O.ring_build(ids)
    n = len(want_ring)
    F = ring.build_fingers(copy_out=True)
    rows = rng.integers(0, n, 60)
    F[rows, rng.integers(0, 128, 60)] = rng.integers(0, n, 60).astype(np.uint32)
    F[rows[:10], :] = rows[:10, None].astype(np.uint32)  # self-pointing rows
    preds = ((np.arange(n) - 1) % n).astype(np.uint32)
    preds[rows[:5]] = 0xFFFFFFFF  # dead predecessor -> livelock -> hop cap
    mk = O.keys_from_ints([(v + 1) % (1 << 128) for v in O.ints_from_keys(want_ring[preds % n])])
    ring.upload_fingers(F)
    ring.upload_peer_state(min_keys=mk, preds=preds)
    keys = O.splitmix_keys(4343, 40000)
    src = rng.integers(0, n, len(keys)).astype(np.uint32)
    src[:2000] = rows[rng.integers(0, 10, 2000)]
    owner, hops, status = ring.route(src, keys)
    wo, wh, ws = O.route(O.Peers(want_ring, F, min_keys=mk, preds=preds), src, keys)
    assert (owner == wo).all() and (hops == wh).all() and (status == ws).all()
    assert (status == 1).any()


@pytest.mark.parametrize("variant", [0, 4, 5])
def test_route_bad_src_is_flagged(cx, O, variant):
    ring = cx.Ring(O.splitmix_keys(3, 50))
    ring.build_fingers()
    ring.set_route_variant(variant)
    owner, hops, status = ring.route(np.array([0, 49, 50, 0xFFFFFFFF], np.uint32),
                                     O.splitmix_keys(4, 4))
    assert status.tolist()[2:] == [2, 2] and owner.tolist()[2:] == [0xFFFFFFFF] * 2


def test_fingers_upload_rejects_bad_index(cx, O):
    ring = cx.Ring(O.splitmix_keys(3, 50))
    F = ring.build_fingers(copy_out=True)
    F[3, 4] = 50
    with pytest.raises(cx.ChordError):
        ring.upload_fingers(F)


# ---------------------------------------------------------------- a10/a11 DHash
@pytest.mark.parametrize("search", [0, 1])
@pytest.mark.parametrize("n_ring", [1, 2, 13, 14, 15, 28, 3000])
def test_nsucc(cx, O, n_ring, search):
    ids = O.splitmix_keys(50 + n_ring, n_ring)
    ring = cx.Ring(ids)
    ring.set_search_variant(search)
    want_ring = O.ring_build(ids)
    keys = edge_keys(O, want_ring, 51, 5000)
    lists, count = ring.nsucc(keys, 14)
    P = O.Peers(want_ring, O.fingers(want_ring))
    wl, wc = O.nsucc(P, keys, 14)
    assert (lists == wl).all() and (count == wc).all()


def test_dhash_insufficient(cx, O):
    ring = cx.Ring(O.splitmix_keys(1, 9))
    with pytest.raises(cx.ChordError) as e:
        ring.dhash_check(14, 10)
    assert "Insufficient succs" in str(e.value)
    cx.Ring(O.splitmix_keys(1, 10)).dhash_check(14, 10)


# ---------------------------------------------------------------- a12 churn
@pytest.mark.parametrize("churn", [0, 1])
@pytest.mark.parametrize("search", [0, 1])
@pytest.mark.parametrize("n_old,nj,nl", [(1, 1, 0), (5, 0, 2), (60, 3, 4), (20000, 200, 200)])
def test_churn_and_misplaced(cx, O, n_old, nj, nl, search, churn):
    ids = O.splitmix_keys(7000 + n_old, n_old)
    old = cx.Ring(ids)
    old.set_search_variant(search)
    old.set_churn_variant(churn)
    want_old = O.ring_build(ids)
    rng = np.random.default_rng(n_old)
    joins = O.splitmix_keys(7100 + n_old, nj)
    if nj > 2:
        joins[1] = want_old[0]  # duplicate of a survivor: rejected
    leave_idx = rng.choice(len(want_old), nl, replace=False)
    leaves = np.concatenate([want_old[leave_idx], O.splitmix_keys(9, 1)])  # + unknown ID
    new, o2n = old.churn(joins, leaves)
    want_new, want_o2n = O.churn(want_old, joins, leaves)
    assert (new.ids() == want_new).all() and (o2n == want_o2n).all()
    keys = edge_keys(O, want_new, 77, 20000)
    for n in (2, 14):
        lists, count, mask, target = old.misplaced(new, o2n, keys, n)
        wl, wc, wm, wt = O.misplaced(want_old, want_new, want_o2n, keys, n)
        assert (lists == wl).all() and (count == wc).all()
        assert (mask == wm).all() and (target == wt).all()


def test_misplaced_caller_mapping(cx, O):
    """old_to_new is caller data: shifted, swapped, out-of-range or all-NONE
    mappings give exactly the oracle's answer.  A value other than CX_NONE that
    is not a new-ring index is a holder outside every list (oracle misplaced_one)."""
    ids = O.splitmix_keys(8080, 3000)
    old = cx.Ring(ids)
    want_old = O.ring_build(ids)
    joins = O.splitmix_keys(8081, 40)
    leaves = want_old[np.random.default_rng(3).choice(3000, 40, replace=False)]
    new, o2n = old.churn(joins, leaves)
    want_new, _ = O.churn(want_old, joins, leaves)
    keys = edge_keys(O, want_new, 78, 20000)
    rng = np.random.default_rng(4)
    shifted = np.where(o2n != 0xFFFFFFFF, (o2n + 1) % len(want_new), o2n).astype(np.uint32)
    swapped = o2n.copy()
    k = rng.choice(3000, 300, replace=False)
    swapped[k] = swapped[np.roll(k, 1)]
    wild = o2n.copy()
    sel = rng.random(3000) < 0.1
    wild[sel] = rng.integers(0, 2**32, sel.sum(), dtype=np.uint64).astype(np.uint32)
    wild[rng.random(3000) < 0.1] = 0x80000005  # out of range
    for m in (o2n, shifted, swapped, wild, np.full(3000, 0xFFFFFFFF, np.uint32)):
        m = np.ascontiguousarray(m, dtype=np.uint32)
        got = old.misplaced(new, m, keys, 14)
        exp = O.misplaced(want_old, want_new, m, keys, 14)
        for a, b in zip(got, exp):
            assert (a == b).all()


@pytest.mark.parametrize("churn", [0, 1])
def test_churn_edge_cases(cx, O, churn):
    """Joins repeating each other, a join taking a leaving peer's ID, joins
    below the smallest / above the largest ID, leaves of unknown IDs, and a
    churn that replaces every peer but one."""
    base = O.splitmix_keys(4242, 300)
    want_old = O.ring_build(base)
    v = O.ints_from_keys(want_old)
    cases = [
        (O.keys_from_ints([v[5] + 1, v[5] + 1, v[5] + 1, 0, MAX, v[0] - 1, v[-1] + 1]),
         O.keys_from_ints([v[7], v[8], 12345])),
        (O.keys_from_ints([v[7], v[9], (v[9] + v[10]) // 2]),    # join == leaver's ID
         O.keys_from_ints([v[7], v[9], v[10]])),
        (O.splitmix_keys(77, 50), want_old[1:]),                   # all but one leave
        (O.keys_from_ints([]), want_old[:0]),                      # no-op
        (O.keys_from_ints([v[3], v[4]]), want_old[:0]),            # joins = survivors only
        # 300 joins sharing their top bits, shuffled: the join bucket sort
        # overflows (one bucket) and the merge sorts them with the radix sort
        (O.keys_from_ints([v[5] + 1 + (k * 7919) % 300 for k in range(300)]),
         O.keys_from_ints([v[6]])),
    ]
    for joins, leaves in cases:
        old = cx.Ring(want_old)
        old.set_churn_variant(churn)
        new, o2n = old.churn(joins, leaves)
        want_new, want_o2n = O.churn(want_old, joins, leaves)
        assert (new.ids() == want_new).all() and (o2n == want_o2n).all()
    old = cx.Ring(want_old[:2])
    old.set_churn_variant(churn)
    with pytest.raises(cx.ChordError):
        old.churn(O.keys_from_ints([]), want_old[:2])               # empty ring


def test_global_maintenance_fixture(cx, O, refvec):
    g = refvec["global_maintenance"]
    ring = cx.Ring(O.keys_from_ints([H(x) for x in g["peers"]]))
    names = [format(v, "x") for v in O.ints_from_keys(ring.ids())]
    keys = O.keys_from_ints([H(k) for k in g["keys"]])
    holders = np.full((len(keys), 1), names.index(g["holder"]), np.uint32)
    lists, count, mask, target = ring.misplaced_holders(keys, holders, g["n"])
    assert (mask == 1).all()
    assert all(names[lists[q, target[q, 0]]] == g["expected_target"] for q in range(len(keys)))


def test_misplaced_holders_random(cx, O):
    ids = O.splitmix_keys(31337, 500)
    ring = cx.Ring(ids)
    want = O.ring_build(ids)
    rng = np.random.default_rng(5)
    keys = O.splitmix_keys(31338, 5000)
    holders = rng.integers(0, 500, (5000, 6)).astype(np.uint32)
    holders[rng.random((5000, 6)) < 0.2] = 0xFFFFFFFF
    holders[rng.random((5000, 6)) < 0.05] = 500 + 7  # not a ring index: never in a list
    s = O.successor(want, keys)
    holders[:, 0] = s  # make some holders correct
    got = ring.misplaced_holders(keys, holders, 4)
    exp = O.misplaced_holders(want, keys, holders, 4)
    for a, b in zip(got, exp):
        assert (a == b).all()


def test_misplaced_multi_holder_order(cx, O):
    """Several misplaced holders of one key (round-4 verdict item 7): holders
    are applied in list order, each handing the key to the first successor in
    list order that still lacks it (chord_oracle.c misplaced_from_list: the
    ordering assumption, parity-unpinned -- in the reference each holder's own
    maintenance thread runs RunGlobalMaintenance, dhash_peer.cpp:271-348, and
    thread timing decides).  Hand-derived on a 40-peer ring, n = 4; GPU equals
    the oracle and the hand derivation."""
    ids = O.splitmix_keys(0x0DE1, 40)
    want = O.ring_build(ids)
    ring = cx.Ring(ids)
    keys = O.splitmix_keys(0x0DE2, 64)
    s = O.successor(want, keys).astype(np.int64)
    n, N = 4, len(want)
    w = lambda k, j: (s[k] + j) % N  # noqa: E731  rank j of key k's new list
    holders = np.empty((64, 5), dtype=np.uint32)
    exp_mask = np.zeros(64, dtype=np.uint16)
    exp_tg = np.full((64, 5), 0xFF, dtype=np.uint8)
    for k in range(64):
        far = [(s[k] + 10 + 3 * j) % N for j in range(3)]  # never in the 4-window
        case = k % 4
        if case == 0:   # two misplaced holders, ranks 1 and 2 held: targets ranks 0, 3
            h = [far[0], w(k, 2), far[1], w(k, 1), 0xFFFFFFFF]
            exp_mask[k], exp_tg[k, 0], exp_tg[k, 2] = 0b101, 0, 3
        elif case == 1:  # three misplaced, nothing held: targets 0, 1, 2 in list order
            h = [far[2], far[0], 0xFFFFFFFF, far[1], w(k, 3)]
            exp_mask[k], exp_tg[k, 0], exp_tg[k, 1], exp_tg[k, 3] = 0b1011, 0, 1, 2
        elif case == 2:  # every rank held: misplaced holders keep the key (no target)
            h = [w(k, 0), far[0], w(k, 1), w(k, 2), w(k, 3)]
            exp_mask[k] = 0b10
        else:           # five misplaced, four ranks: the fifth finds none left
            h = [far[0], far[1], far[2], (s[k] + 20) % N, (s[k] + 25) % N]
            exp_mask[k] = 0b11111
            exp_tg[k, :4] = [0, 1, 2, 3]
        holders[k] = h
    got = ring.misplaced_holders(keys, holders, n)
    exp = O.misplaced_holders(want, keys, holders, n)
    for a, b in zip(got, exp):
        assert (a == b).all()
    assert (got[2].view(np.uint16) == exp_mask).all()
    assert (got[3] == exp_tg).all()


# ---------------------------------------------------------------- a2 InBetween
def test_in_between_gpu(cx, O, refvec):
    def u256(v):
        return [(v >> (64 * j)) & 0xFFFFFFFFFFFFFFFF for j in range(4)]

    cases = [(H(r["v"]), H(r["lb"]), H(r["ub"]), r["incl"], r["expect"])
             for r in refvec["in_between"]]
    rng = np.random.default_rng(9)
    special = [0, 1, MAX, 1 << 128, (1 << 128) + 1, (1 << 256) - 1, 1 << 127]
    vals = special + [int.from_bytes(rng.bytes(16), "big") for _ in range(8)]
    for v in vals:
        for lb in vals:
            for ub in vals:
                cases.append((v, lb, ub, True, None))
                cases.append((v, lb, ub, False, None))
    for inc in (True, False):
        sel = [c for c in cases if c[3] == inc]
        V = np.array([u256(c[0]) for c in sel], np.uint64)
        L = np.array([u256(c[1]) for c in sel], np.uint64)
        U = np.array([u256(c[2]) for c in sel], np.uint64)
        got = cx.in_between(V, L, U, inc)
        for c, g in zip(sel, got):
            want = O.in_between(c[0], c[1], c[2], inc)
            assert bool(g) == want
            if c[4] is not None:
                assert want == c[4]
    from chordx import ChordKey
    assert not ChordKey("f4ee136cb4059b2883450e7e93698be").in_between(
        H("633bd46b5c515992a5ce553d0680bec9"), H("f4ee136cb4059b2883450e7e93698bd"))


# ---------------------------------------------------------------- device buffers
def test_device_memkind_matches_host(cx, O):
    import torch
    ids = O.splitmix_keys(0x5EED0003, 1 << 14)
    ring = cx.Ring(ids)
    ring.build_fingers()
    q = 1 << 16
    keys_d = torch.empty((q, 2), dtype=torch.int64, device="cuda:0")
    cx.fill_splitmix(keys_d, 0x5EED0004)
    keys_h = O.splitmix_keys(0x5EED0004, q)
    assert (keys_d.cpu().numpy().view(np.uint64) == keys_h).all()
    src_d = (torch.arange(q, device="cuda:0", dtype=torch.int32) % ring.n)
    od, hd, sd = ring.route(src_d, keys_d)
    oh, hh, sh = ring.route(src_d.cpu().numpy().astype(np.uint32), keys_h)
    torch.cuda.synchronize()
    assert (od.cpu().numpy().view(np.uint32) == oh).all()
    assert (hd.cpu().numpy() == hh).all()
    ow = ring.successor(keys_d)
    torch.cuda.synchronize()
    assert (ow.cpu().numpy().view(np.uint32) == O.successor(O.ring_build(ids), keys_h)).all()


# ---------------------------------------------------------------- a1 IDs
def test_uuid5_fixture_ids(cx, O, refvec):
    """GPU SHA-1/UUIDv5 of the 103 fixture ip:port names and the Join key names."""
    names = [r["name"] for r in refvec["id_hash"]]
    got = cx.uuid5_dns(names)
    assert [format(v, "x") for v in O.ints_from_keys(got)] == [r["id"] for r in refvec["id_hash"]]
    jk = refvec["join_placement"]["keys"]
    got = cx.uuid5_dns([k["plain"] for k in jk])
    assert [format(v, "x") for v in O.ints_from_keys(got)] == [k["hash"] for k in jk]
    from chordx import ChordKey
    assert str(ChordKey("127.0.0.1:5012", hashed=False)) == "91186395ae2562aaa1ff7f3513747e9"


def test_uuid5_lengths_and_bytes(cx, O):
    """SHA-1 padding boundaries (1 vs 2 vs 3 blocks), empty names, arbitrary bytes."""
    rng = np.random.default_rng(11)
    names = [b""] + [bytes(rng.integers(0, 256, L, dtype=np.uint8)) for L in
                     list(range(0, 140)) + [183, 184, 247, 248, 1000]]
    names += [f"key{i}".encode() for i in range(2000)]
    got = cx.uuid5_dns(names)
    import uuid as U
    want = [int.from_bytes(U.uuid5(U.NAMESPACE_DNS, n.decode("latin-1")).bytes, "big")
            if all(c < 128 for c in n) else None for n in names]
    for g, w, n in zip(O.ints_from_keys(got), want, names):
        if w is not None:
            assert g == w
    # arbitrary (non-ASCII) bytes checked against the C oracle's SHA-1
    for g, n in zip(O.ints_from_keys(got), names):
        k = O.lib().or_uuid5_dns(n, len(n))
        assert g == (k.lo | (k.hi << 64))


@pytest.mark.parametrize("spread", [40, 100, 127])
def test_fingers_streaming_build_clustered(cx, O, spread):
    """The streaming finger build (ID-slice windows, k_fingers_tile; rings of
    2^18 peers or more) with IDs packed so tightly that slices tie, windows
    overflow and key ranges are exceeded: every entry bit-exact vs the
    oracle's PopulateFingerTable restatement."""
    ids = clustered_ring(O, (1 << 18) + 77, 0xF1 + spread, spread)
    want = O.ring_build(ids)
    assert len(want) >= 1 << 18
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    assert (ring.ids() == want).all()
    assert (F == O.fingers(want)).all()


def test_fingers_streaming_build_uniform_tail(cx, O):
    """Ring size not a multiple of the 128-peer block, wrap at the last peer."""
    ids = O.splitmix_keys(0xF2, (1 << 18) + 1234)
    want = O.ring_build(ids)
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    assert (F == O.fingers(want)).all()


def test_misplaced_with_foreign_map_and_chained_churn(cx, O):
    """cx_misplaced derives new successors from the churn's recorded old->new
    map; a caller map that differs from it (here: one survivor treated as
    departed) must take the two-search path, and a ring churned twice pairs
    each scan with its own map.  All keys vs the oracle."""
    n_old, q = 5000, 60000
    ids = O.splitmix_keys(0xC5, n_old)
    old = cx.Ring(ids)
    want_old = O.ring_build(ids)
    rng = np.random.default_rng(0xC6)
    leaves = want_old[rng.choice(len(want_old), 300, replace=False)]
    joins = O.splitmix_keys(0xC7, 300)
    new, o2n = old.churn(joins, leaves)
    want_new, want_o2n = O.churn(want_old, joins, leaves)
    keys = O.splitmix_keys(0xC8, q)
    for m in (o2n, o2n.copy()):  # the recorded map and an equal copy
        got = old.misplaced(new, m, keys, 14)
        want = O.misplaced(want_old, want_new, want_o2n, keys, 14)
        for g, w in zip(got, want):
            assert (g == w).all()
    foreign = o2n.copy()
    foreign[np.flatnonzero(foreign != O.NONE)[7]] = O.NONE
    got = old.misplaced(new, foreign, keys, 14)
    want = O.misplaced(want_old, want_new, foreign, keys, 14)
    for g, w in zip(got, want):
        assert (g == w).all()
    # second churn: new -> newer; and the stale pairing (old, newer) is rejected
    joins2 = O.splitmix_keys(0xC9, 200)
    newer, o2n2 = new.churn(joins2, want_new[:50])
    want_newer, want_o2n2 = O.churn(want_new, joins2, want_new[:50])
    got = new.misplaced(newer, o2n2, keys, 14)
    want = O.misplaced(want_new, want_newer, want_o2n2, keys, 14)
    for g, w in zip(got, want):
        assert (g == w).all()




@pytest.mark.parametrize("search", [1, 2, 3, 4, 5])
def test_predecessor(cx, O, refvec, search):
    """Batched GetPredecessor vs the oracle: reference fixtures, edge rings and
    keys (IDs, +-1, 0, 2^128 - 1), N = 1, 2, 3."""
    for case in ("in_succ_list", "from_finger_table"):
        g = refvec["get_pred"][case]
        ring = cx.Ring(O.keys_from_ints([H(x) for x in g["peers"]]))
        ring.set_search_variant(search)
        names = [format(v, "x") for v in O.ints_from_keys(ring.ids())]
        assert names[ring.predecessor(O.keys_from_ints([H(g["key"])]))[0]] == g["expected"]
    for n, seed in ((1, 1), (2, 2), (3, 3), (1000, 4), (70001, 5)):
        ids = edge_ring(O, n, seed)
        want_ring = O.ring_build(ids)
        ring = cx.Ring(ids)
        ring.set_search_variant(search)
        keys = edge_keys(O, want_ring, seed + 100, 20000)
        assert (ring.predecessor(keys) == O.predecessor(want_ring, keys)).all()


@pytest.mark.parametrize("lg", [12, 20])
def test_route_table_from_level_planes_identical(lg):
    """The pattern-keyed table built from finger level planes is bit-identical
    to the one built from the row-major finger table."""
    import torch

    import chordx
    ids = torch.empty((1 << lg, 2), dtype=torch.int64, device="cuda:0")
    chordx.fill_splitmix(ids, 0x5EED0003 + lg)
    ring = chordx.Ring(ids)
    ring.build_fingers()
    assert ring.route_info()[0] == 5
    h_planes = ring.route_table_hash()
    ring.set_table_build(1)
    ring.build_fingers()
    h_rows = ring.route_table_hash()
    ring.set_table_build(2)
    ring.build_fingers()
    h_planes_only = ring.route_table_hash()
    ring.set_table_build(3)  # one lane per entry (the default is root-centric)
    ring.build_fingers()
    h_entry = ring.route_table_hash()
    from chordx import _lib
    # the default with most rows deferred to overflow launches (48 roots per block)
    ring.set_table_build(0)
    _lib.set_fault(2)
    try:
        ring.build_fingers()
    finally:
        _lib.set_fault(0)
    h_ovf = ring.route_table_hash()
    assert h_planes == h_rows == h_planes_only == h_entry == h_ovf
    assert h_planes != 0


@pytest.mark.parametrize("lg", [12, 16])
def test_route_table_without_planes_memory(cx, O, lg):
    """The default build when HBM for the finger level planes runs out
    (fault-injected allocation failure): it falls back to the row-major finger
    table, whose build reads 64-bit ID high words -- the 32-bit slices it had
    prepared must be replaced, or the build reads past them.  The table must
    equal the forced row-major build's, and routes must equal the oracle's."""
    import torch
    ids = torch.empty((1 << lg, 2), dtype=torch.int64, device="cuda:0")
    cx.fill_splitmix(ids, 0x5EED0303 + lg)
    ring = cx.Ring(ids)
    ring.set_table_build(1)
    ring.build_fingers()
    h_rows = ring.route_table_hash()
    ring.set_table_build(0)
    from chordx import _lib
    _lib.set_fault(1)
    try:
        ring.build_fingers()
    finally:
        _lib.set_fault(0)
    assert ring.route_info()[0] == 5
    assert ring.route_table_hash() == h_rows != 0
    want = O.ring_build(ids.cpu().numpy().view(np.uint64))
    keys = O.splitmix_keys(0x5EED0304, 4096)
    src = (np.arange(4096) * 131 % len(want)).astype(np.uint32)
    o, h, s = ring.route(src, keys)
    wo, wh, ws = O.route(O.Peers(want, O.fingers(want)), src, keys)
    assert (o == wo).all() and (h == wh).all() and (s == ws).all()


@pytest.mark.parametrize("kind", ["small", "mixed", "clustered"])
def test_route_table_builds_edge_rings(cx, O, kind):
    """The default route-table build (level + two-hop planes) equals the
    level-planes-only build on small rings, rings mixing a dense cluster with
    uniform IDs, and a dense cluster alone (escapes equal too), and routes
    through it equal the oracle."""
    rng = np.random.default_rng(len(kind))
    if kind == "small":
        ids = O.splitmix_keys(0xB0, 200)
    else:
        base = 0x3C3C_5A5A_0F0F_1234 << 64
        m = 1500 if kind == "mixed" else 6000
        vals = [base + i * 7919 for i in range(m)]
        if kind == "mixed":
            vals += O.ints_from_keys(O.splitmix_keys(0xB1, 6000))
        ids = O.keys_from_ints(vals)
    ring = cx.Ring(ids)
    ring.build_fingers()
    assert ring.route_info()[0] == 5
    h0, e0 = ring.route_table_hash(), ring.route_info()[1]
    ring.set_table_build(1)  # row-major fingers
    ring.build_fingers()
    h1, e1 = ring.route_table_hash(), ring.route_info()[1]
    ring.set_table_build(2)
    ring.build_fingers()
    h2, e2 = ring.route_table_hash(), ring.route_info()[1]
    ring.set_table_build(3)  # one lane per entry (the default is root-centric)
    ring.build_fingers()
    h3, e3 = ring.route_table_hash(), ring.route_info()[1]
    from chordx import _lib
    ring.set_table_build(0)
    _lib.set_fault(2)  # the default with overflow launches (48 roots per block)
    try:
        ring.build_fingers()
    finally:
        _lib.set_fault(0)
    h5, e5 = ring.route_table_hash(), ring.route_info()[1]
    assert h0 == h1 == h2 == h3 == h5 and h0 != 0
    assert e0 == e1 == e2 == e3 == e5
    ring.set_table_build(0)
    ring.build_fingers()
    want = O.ring_build(ids)
    keys = edge_keys(O, want, 0xB2, 5000)
    src = rng.integers(0, len(want), len(keys)).astype(np.uint32)
    got = ring.route(src, keys)
    exp = O.route(O.Peers(want, O.fingers(want)), src, keys)
    for a, b in zip(got, exp):
        assert (a == b).all()


def test_route_table_builds_deterministic_all_escapes(cx, O):
    """A dense cluster alone: every finger at a table level wraps the ring, so
    every word of the table is an escape (n * R * 16) in every build, and
    repeated builds are bit-identical.  Round 5: the level-planes build (2)
    took the exact-ID branch of its gap code through a variable 128-bit shift
    whose result differed by lane and run (a few hundred slot-8 words came out
    representable); the branch is now 64-bit arithmetic on the IDs' halves."""
    base = 0x3C3C_5A5A_0F0F_1234 << 64
    ids = O.keys_from_ints([base + i * 7919 for i in range(6000)])
    ring = cx.Ring(ids)
    seen = set()
    for tb in (0, 1, 2, 3, 2, 1, 2):
        ring.set_table_build(tb)
        ring.build_fingers()
        v, esc, nbytes = ring.route_info()
        assert v == 5 and esc == nbytes // 4, (tb, esc, nbytes)
        seen.add(ring.route_table_hash())
    assert len(seen) == 1
    ring.set_table_build(0)


def test_route_table_escape_count_with_overflow(cx, O):
    """Escape accounting of the default build when rows are deferred to
    overflow launches: a ring of four dense clusters plus a few
    uniform IDs has many nodes the 4-B format cannot hold -- row words
    included (fingers that land in the empty space between clusters) -- and,
    with 48 roots per block (fault 2), most rows go to overflow launches.  The
    count must equal the one-lane-per-entry build's, which has no overflow."""
    vals = []
    for c in range(4):
        base = int(O.ints_from_keys(O.splitmix_keys(0xE5C0 + c, 1))[0])
        vals += [(base + i * 104729) % (1 << 128) for i in range(2500)]
    vals += O.ints_from_keys(O.splitmix_keys(0xE5C9, 700))
    ids = O.keys_from_ints(vals)
    from chordx import _lib
    ring = cx.Ring(ids)
    ring.set_table_build(3)  # one lane per entry: no overflow path
    ring.build_fingers()
    h3, e3 = ring.route_table_hash(), ring.route_info()[1]
    ring.set_table_build(0)
    ring.build_fingers()
    h0, e0 = ring.route_table_hash(), ring.route_info()[1]
    _lib.set_fault(2)
    try:
        ring.build_fingers()
    finally:
        _lib.set_fault(0)
    h5, e5 = ring.route_table_hash(), ring.route_info()[1]
    assert e3 > 0
    assert h0 == h3 == h5 and e0 == e3 == e5
    want = O.ring_build(ids)
    keys = edge_keys(O, want, 0xE5CA, 4000)
    src = (np.arange(len(keys)) * 7 % len(want)).astype(np.uint32)
    got = ring.route(src, keys)
    exp = O.route(O.Peers(want, O.fingers(want)), src, keys)
    for a, b in zip(got, exp):
        assert (a == b).all()


# ------------------------------------------------- a12 churn directory (fast path)
def _churn_cases(O):
    """(old IDs, joins, leaves) exercising the churn directory's corners."""
    rng = np.random.default_rng(99)
    out = []
    ids = O.splitmix_keys(5150, 20000)
    R = O.ring_build(ids)
    out.append(("uniform_1pct", ids, O.splitmix_keys(5151, 200),
                R[rng.choice(20000, 200, replace=False)]))
    # joiners packed right after old peers: windows with many joiners, buckets
    # holding 3+ merged entries, equal hints (IDs differing in the low bits)
    v = O.ints_from_keys(R)
    dense = [v[i] + 1 + j for i in range(0, 20000, 97) for j in range(20)]
    out.append(("dense_joins", ids, O.keys_from_ints(dense),
                R[rng.choice(20000, 3000, replace=False)]))
    # clustered ring: every ID in one narrow band (a handful of buckets)
    base = 0x0FED_CBA9_8765_4321 << 64
    cl = O.keys_from_ints([base + i * 131 for i in range(4000)] + [(1 << 127) + i for i in range(40)])
    out.append(("clustered", cl, O.keys_from_ints([base + i * 131 + 7 for i in range(0, 4000, 3)]),
                cl[rng.choice(4040, 500, replace=False)]))
    # heavy churn: half the ring leaves, as many join
    out.append(("half", ids, O.splitmix_keys(5152, 10000),
                R[rng.choice(20000, 10000, replace=False)]))
    # small rings straddling the 32-peer threshold of the directory path
    s = O.splitmix_keys(5153, 40)
    Rs = O.ring_build(s)
    out.append(("small", s, O.splitmix_keys(5154, 3), Rs[:9]))
    return out


@pytest.mark.parametrize("case", range(5))
def test_misplaced_churn_directory(cx, O, case):
    """cx_misplaced on a ring from cx_churn with cx_churn's mapping takes the
    churn directory (one gather per key); it must equal the two-search path
    and the oracle on keys at and next to every old, new, joining and
    departed ID, for both list lengths and a caller copy of the mapping."""
    name, ids, joins, leaves = _churn_cases(O)[case]
    old = cx.Ring(ids)
    want_old = O.ring_build(ids)
    new, o2n = old.churn(joins, leaves)
    want_new, want_o2n = O.churn(want_old, joins, leaves)
    assert (o2n == want_o2n).all()
    rng = np.random.default_rng(case)
    vals = O.ints_from_keys(O.splitmix_keys(600 + case, 30000))
    for arr in (want_old, want_new, joins, leaves):
        a = O.ints_from_keys(arr)
        for x in (a if len(a) <= 3000 else [a[i] for i in rng.choice(len(a), 3000, replace=False)]):
            vals += [x, (x + 1) % (1 << 128), (x - 1) % (1 << 128)]
    vals += [0, 1, MAX, MAX - 1]
    keys = O.keys_from_ints(vals)
    for n in (1, 5, 14, 16):
        got = old.misplaced(new, o2n.copy(), keys, n)
        new.set_misplaced_variant(0)
        two = old.misplaced(new, o2n, keys, n)
        new.set_misplaced_variant(1)
        exp = O.misplaced(want_old, want_new, want_o2n, keys, n)
        for a, b, c in zip(got, two, exp):
            assert (a == c).all(), (name, n)
            assert (b == c).all(), (name, n)
        # fused placement + scan (cx_dhash_maintenance), directory and two-search paths
        wl_old, wc_old = nsucc_window(O, want_old, keys, n)
        for variant in (1, 0):
            new.set_misplaced_variant(variant)
            fz = old.dhash_maintenance(new, o2n, keys, n)
            assert (fz[0] == wl_old).all() and (fz[1] == wc_old).all(), (name, n, variant)
            for a, c in zip(fz[2:], exp):
                assert (a == c).all(), (name, n, variant)
        new.set_misplaced_variant(1)
        ol, oc = old.nsucc(keys, n)
        assert (ol == wl_old).all() and (oc == wc_old).all()


def nsucc_window(O, ring, keys, n):
    """GetNSuccessors' converged result (abstract_chord_peer.cpp:345-373):
    ring[(succ(key) + j) mod N] for j < min(n, N), CX_NONE after."""
    N = len(ring)
    s = O.successor(ring, keys).astype(np.int64)
    j = np.arange(n, dtype=np.int64)
    w = ((s[:, None] + j) % N).astype(np.uint32)
    w[:, j >= min(n, N)] = 0xFFFFFFFF
    return w, np.full(len(keys), min(n, N), dtype=np.uint8)


def test_misplaced_churn_directory_device_and_foreign_parent(cx, O):
    """Device buffers through the directory path; a ring churned from a
    different parent (or a mapping that differs in one entry) takes the
    two-search path and still matches the oracle."""
    import torch
    ids = O.splitmix_keys(5160, 5000)
    want_old = O.ring_build(ids)
    old = cx.Ring(ids)
    joins = O.splitmix_keys(5161, 60)
    leaves = want_old[np.random.default_rng(5).choice(5000, 60, replace=False)]
    new, o2n = old.churn(joins, leaves)
    want_new, want_o2n = O.churn(want_old, joins, leaves)
    keys = edge_keys(O, want_new, 79, 20000)
    exp = O.misplaced(want_old, want_new, want_o2n, keys, 14)
    kd = torch.from_numpy(keys.view(np.int64).copy()).cuda()
    od = torch.from_numpy(o2n.view(np.int32).copy()).cuda()
    got = old.misplaced(new, od, kd, 14)
    for a, b in zip(got, exp):
        assert (a.cpu().numpy().view(b.dtype).reshape(b.shape) == b).all()
    fz = old.dhash_maintenance(new, od, kd, 14)
    for a, b in zip(fz, nsucc_window(O, want_old, keys, 14) + tuple(exp)):
        assert (a.cpu().numpy().view(b.dtype).reshape(b.shape) == b).all()
    other = cx.Ring(ids)   # same IDs, not new's parent
    got = other.misplaced(new, o2n, keys, 14)
    for a, b in zip(got, exp):
        assert (a == b).all()
    fz = other.dhash_maintenance(new, o2n, keys, 14)
    for a, b in zip(fz, nsucc_window(O, want_old, keys, 14) + tuple(exp)):
        assert (a == b).all()
    bent = o2n.copy()
    bent[17] = 0xFFFFFFFF
    got = old.misplaced(new, bent, keys, 14)
    for a, b in zip(got, O.misplaced(want_old, want_new, bent, keys, 14)):
        assert (a == b).all()
