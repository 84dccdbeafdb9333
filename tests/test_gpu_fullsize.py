"""BASELINE-size checks (config C3 and a C5-shaped churn) on the GPU.

Where the oracle cannot cover the full size in seconds, size-independent
properties are checked on every element and the oracle on a sample:
  * route owner == exact successor (lower_bound with wrap) for all 2^24 keys;
  * route hops/owner identical between the two route kernels (finger+ring
    gathers vs route table) for all keys, and equal to the oracle's literal
    ForwardRequest walk on a 2^17-key sample;
  * the full 2^20 x 128 finger table equals the oracle's, bit for bit.
"""
import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.fixture(scope="module")
def c3(O):
    import chordx
    ids = O.splitmix_keys(0x5EED0003, 1 << 20)
    ring = chordx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    return chordx, ring, F, O.ring_build(ids)


def test_c3_fingers_bit_exact(O, c3):
    _, ring, F, want_ring = c3
    assert ring.n == len(want_ring)
    assert (ring.ids() == want_ring).all()
    assert (F == O.fingers(want_ring)).all()


def test_c3_routed_lookups(O, c3):
    import torch
    cx, ring, F, want_ring = c3
    q = 1 << 24
    keys = torch.empty((q, 2), dtype=torch.int64, device="cuda:0")
    cx.fill_splitmix(keys, 0x5EED0004)
    src = (torch.arange(q, device="cuda:0", dtype=torch.int64) % ring.n).to(torch.int32)
    ring.set_route_variant(0)
    o0, h0, s0 = ring.route(src, keys)
    ring.set_route_variant(4)
    o4, h4, s4 = ring.route(src, keys)
    ring.set_route_variant(5)
    o5, h5, s5 = ring.route(src, keys)
    assert ring.route_info()[0] == 5
    succ = ring.successor(keys)
    torch.cuda.synchronize()
    o1, h1 = o0, h0  # the per-hop walk (no table) is the reference of the table walks
    assert int((s0 != 0).sum()) == 0 and bool((o0 == succ).all())
    assert bool((o4 == o1).all()) and bool((h4 == h1).all()) and int((s4 != 0).sum()) == 0
    assert bool((o5 == o1).all()) and bool((h5 == h1).all()) and int((s5 != 0).sum()) == 0
    mean = float(h1.double().mean())
    assert 9.0 < mean < 11.0  # ~log2(N)/2 for uniform rings
    # oracle literal walk on a sample, with the oracle's own finger table
    sample = 1 << 17
    kh = keys[:sample].cpu().numpy().view(np.uint64)
    sh = src[:sample].cpu().numpy().view(np.uint32)
    wo, wh, ws = O.route(O.Peers(want_ring, F), sh, kh)
    assert (o1[:sample].cpu().numpy().view(np.uint32) == wo).all()
    assert (h1[:sample].cpu().numpy() == wh).all()


@pytest.mark.parametrize("churn", [0, 1])
def test_c5_shaped_churn(O, churn):
    """1% joins + 1% leaves on a 2^20 ring; n=14 lists, misplaced mask and
    targets for 2^21 keys: all keys vs oracle."""
    import chordx
    n_old, q = 1 << 20, 1 << 21
    ids = O.splitmix_keys(0x5EED0007, n_old)
    old = chordx.Ring(ids)
    old.set_churn_variant(churn)
    want_old = O.ring_build(ids)
    rng = np.random.default_rng(0x5EED0009)
    leaves = want_old[rng.choice(n_old, n_old // 100, replace=False)]
    joins = O.splitmix_keys(0x5EED0009, n_old // 100)
    new, o2n = old.churn(joins, leaves)
    want_new, want_o2n = O.churn(want_old, joins, leaves)
    assert (new.ids() == want_new).all() and (o2n == want_o2n).all()
    keys = O.splitmix_keys(0x5EED0008, q)
    lists, count, mask, target = old.misplaced(new, o2n, keys, 14)
    wl, wc, wm, wt = O.misplaced(want_old, want_new, want_o2n, keys, 14)
    assert (lists == wl).all() and (count == wc).all()
    assert (mask == wm).all() and (target == wt).all()
    assert 0 < int((mask != 0).sum()) < q
