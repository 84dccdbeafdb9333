"""Route-table depth (a7-a9's converged table): the table covers
finger levels [128 - R, 128) and the walk takes exact hops below it
(ClosestPrecedingFinger over the finger table, chord_peer.cpp:157-176, one
level at a time).  The depth changes only where a hop's finger comes from, so
owners, hop counts and statuses must not depend on R.  Default R = log2 n + 8
rounded up to 4 (32 at 2^24); cxi_set_route_depth overrides it per ring before
its first finger build."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cx():
    import chordx
    if chordx.device_count() == 0:
        pytest.fail("gpu test without a HIP device")
    return chordx


def default_depth(n):
    lg = 0
    while (1 << lg) < n:
        lg += 1
    return max(16, (lg + 8 + 3) // 4 * 4)


@pytest.mark.parametrize("n", [20000, (1 << 18) + 3, 1 << 20])
def test_default_depth(cx, O, n):
    ring = cx.Ring(O.splitmix_keys(0x5EED0401 + n, n))
    ring.build_fingers()
    v, esc, nbytes = ring.route_info()
    # escapes: nodes past the 16-bit gap code (2^(gs + 16), gs = 116 - ceil(log2 n):
    # 8-16x the mean gap, so the largest gaps of a ring just above a power of two
    # overflow it); the walk takes them exactly
    assert v == 5 and esc < n * default_depth(n) * 32 // 1000
    assert nbytes == n * default_depth(n) * 128


@pytest.fixture(scope="module")
def depth_setup(cx, O):
    n = (1 << 18) + 3
    ids = O.splitmix_keys(0x5EED0410, n)
    want = O.ring_build(ids)
    q = 1 << 16
    keys = O.splitmix_keys(0x5EED0411, q)
    src = (np.arange(q) * 7919 % n).astype(np.uint32)
    base = cx.Ring(ids)
    base.build_fingers()
    ob, hb, sb = base.route(src, keys)
    assert (sb == 0).all() and (ob == O.successor(want, keys)).all()
    wo, wh, _ = O.route(O.Peers(want, O.fingers(want)), src[:4096], keys[:4096])
    assert (ob[:4096] == wo).all() and (hb[:4096] == wh).all()
    return ids, keys, src, ob, hb


# 16: the shallowest table (many exact hops); 20 / 32: either side of the
# default 28 at this size; 40: planes below the streaming tile's first level
# (the build reads them from the finger rows); 59: the deepest the pattern-keyed
# build takes (its lowest plane level 128 - R - 5 must be >= 64)
@pytest.mark.parametrize("R", [16, 20, 32, 40, 59])
def test_depth_override_same_routes(cx, depth_setup, R):
    ids, keys, src, ob, hb = depth_setup
    ring = cx.Ring(ids)
    ring.set_route_depth(R)
    ring.build_fingers()
    v, esc, nbytes = ring.route_info()
    assert v == 5 and nbytes == ring.n * R * 128
    # escapes (nodes the walk takes exactly) stay rare down to ~2^-16 of the
    # mean gap; levels far below it (R = 59 here: 2^-41) hold mostly escapes
    assert R > 40 or esc < ring.n * R * 32 // 1000
    o, h, s = ring.route(src, keys)
    assert (o == ob).all() and (h == hb).all() and (s == 0).all()


def test_depth_override_errors(cx, O):
    ring = cx.Ring(O.splitmix_keys(0x5EED0420, 5000))
    for bad in (15, 60, 64, 65, -1):
        with pytest.raises(cx.ChordError):
            ring.set_route_depth(bad)
    ring.set_route_depth(0)  # back to the default
    ring.build_fingers()
    assert ring.route_info()[2] == 5000 * default_depth(5000) * 128
    with pytest.raises(cx.ChordError):  # the table exists: its depth is fixed
        ring.set_route_depth(32)
