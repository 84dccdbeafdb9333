"""Row f2: finger repair after churn (finger_table.h:148-168 AdjustFingers /
ReplaceDeadPeer, abstract_chord_peer.cpp:615-645 FixOtherFingers, batched).

A churned ring remaps its parent's finger level planes through the churn's
old_to_new map and searches exactly only the fingers a churn event touched
(k_planes_repair; an A/B, off by default: bit-identical but slower than the
streaming build).  The repaired ring must route exactly like a
ring whose fingers were searched from scratch: identical route-table hash, the
oracle's finger table and walk.  The streaming finger build (and so the
repair) starts at 2^18 peers.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MAX = (1 << 128) - 1


@pytest.fixture(scope="module")
def cx():
    import chordx
    if chordx.device_count() == 0:
        pytest.fail("gpu test without a HIP device")
    return chordx


def churned_pair(cx, O, ids, joins, leaves):
    """(repaired child, child built from scratch, oracle ring of the child)."""
    old = cx.Ring(ids)
    old.set_fingers_repair(True)
    old.build_fingers()
    a, o2n = old.churn(joins, leaves)
    a.build_fingers()
    old.set_fingers_repair(False)
    b, o2n_b = old.churn(joins, leaves)
    b.build_fingers()
    assert (np.asarray(o2n) == np.asarray(o2n_b)).all()
    want, _ = O.churn(O.ring_build(ids), joins, leaves)
    return old, a, b, want


def check_same(cx, O, a, b, want, q=1 << 16, fingers=False):
    rep, searched = a.fingers_repair_info()
    assert rep and searched > 0
    assert b.fingers_repair_info()[0] is False
    assert a.route_table_hash() == b.route_table_hash()
    keys = O.splitmix_keys(0x5EED00F1, q)
    src = (np.arange(q) % a.n).astype(np.uint32)
    oa, ha, sa = a.route(src, keys)
    ob, hb, sb = b.route(src, keys)
    assert (oa == ob).all() and (ha == hb).all() and (sa == 0).all() and (sb == 0).all()
    assert (oa == O.successor(want, keys)).all()
    if fingers:  # rows materialised on demand equal the oracle's table
        F = a.fingers_device().cpu().numpy().view(np.uint32)
        assert (F == O.fingers(want)).all()
        wo, wh, _ = O.route(O.Peers(want, F), src[:4096], keys[:4096])
        assert (oa[:4096] == wo).all() and (ha[:4096] == wh).all()


def test_repair_uniform_churn(cx, O):
    """1 % joins + 1 % leaves of a 2^18-peer ring (C5's churn shape)."""
    n = 1 << 18
    ids = O.splitmix_keys(0x5EED0101, n)
    want_old = O.ring_build(ids)
    rng = np.random.default_rng(1)
    joins = O.splitmix_keys(0x5EED0102, n // 100)
    leaves = want_old[rng.choice(n, n // 100, replace=False)]
    _, a, b, want = churned_pair(cx, O, ids, joins, leaves)
    check_same(cx, O, a, b, want, fingers=True)


def test_repair_adversarial_events(cx, O):
    """Events placed where the remap rule must refuse: joins exactly at finger
    targets id_p + 2^l, joins packed into one gap, runs of adjacent leavers
    (a finger and its predecessor both gone), the ring's first and last peers
    leaving (cyclic x - 1), and joins below the smallest / above the largest ID."""
    n = (1 << 18) + 77
    ids = O.splitmix_keys(0x5EED0103, n)
    want_old = O.ring_build(ids)
    v = O.ints_from_keys(want_old)
    m = len(v)
    rng = np.random.default_rng(2)
    jv = []
    for p in rng.choice(m, 300, replace=False):
        lvl = int(rng.integers(93, 128))
        jv.append((v[p] + (1 << lvl)) % (1 << 128))       # t exactly
        jv.append((v[p] + (1 << lvl) - 1) % (1 << 128))   # just below t
    g = int(rng.integers(0, m - 1))
    jv += [v[g] + 1 + k for k in range(500)]               # 500 joins in one gap
    jv += [0, 1, MAX, v[0] - 1, v[-1] + 1]
    vs = set(v)
    joins = O.keys_from_ints(sorted(set(x for x in jv if x not in vs)))
    li = set()
    for s0 in rng.choice(m - 8, 200, replace=False):
        li.update(range(int(s0), int(s0) + 4))             # runs of adjacent leavers
    li.update([0, 1, m - 1, m - 2])
    leaves = want_old[sorted(li)]
    _, a, b, want = churned_pair(cx, O, ids, joins, leaves)
    check_same(cx, O, a, b, want)


def test_repair_chained_and_size_change(cx, O):
    """Three churn epochs in a row, each repairing from the previous repaired
    ring; the second one shrinks the ring (leaves only), the third grows it
    (every epoch stays at 2^18 peers or more, the streaming build's range)."""
    n = (1 << 18) + 20000
    ids = O.splitmix_keys(0x5EED0104, n)
    ring = cx.Ring(ids)
    ring.set_fingers_repair(True)
    ring.build_fingers()
    ref = cx.Ring(ids)
    ref.set_fingers_repair(False)
    ref.build_fingers()
    want = O.ring_build(ids)
    rng = np.random.default_rng(3)
    for epoch, (nj, nl) in enumerate([(2621, 2621), (0, 5000), (9000, 100)]):
        joins = O.splitmix_keys(0x5EED0200 + epoch, nj)
        leaves = want[rng.choice(len(want), nl, replace=False)]
        ring2, _ = ring.churn(joins, leaves)
        ring2.build_fingers()
        ref2, _ = ref.churn(joins, leaves)
        ref2.build_fingers()
        want, _ = O.churn(want, joins, leaves)
        assert (ring2.ids() == want).all()
        check_same(cx, O, ring2, ref2, want, q=1 << 14)
        ring.close()
        ref.close()
        ring, ref = ring2, ref2


def test_repair_parent_destroyed_first(cx, O):
    """The parent's planes outlive the parent (shared with the churned ring)."""
    n = 1 << 18
    ids = O.splitmix_keys(0x5EED0105, n)
    old = cx.Ring(ids)
    old.set_fingers_repair(True)
    old.build_fingers()
    want_old = O.ring_build(ids)
    joins = O.splitmix_keys(0x5EED0106, 1000)
    leaves = want_old[::300]
    new, _ = old.churn(joins, leaves)
    old.close()
    new.build_fingers()
    ref = cx.Ring(O.churn(want_old, joins, leaves)[0])
    ref.build_fingers()
    assert new.fingers_repair_info()[0]
    assert new.route_table_hash() == ref.route_table_hash()
