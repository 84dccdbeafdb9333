"""a9 on the GPU: ForwardRequest's dead-finger branch (chord_peer.cpp:193-208,
dhash_peer.cpp:505-526) in the literal walk, through the C ABI, against the
oracle's restatement.  The scenarios are the oracle tests' (which pin them by
hand-derived expectations and the reference's GET_SUCC_FAILING fixture) plus
random rings with dead peers, edited fingers, unset predecessors and ragged
successor lists, for both forwarding rules."""
import numpy as np
import pytest

from test_oracle_golden import failing_state

pytestmark = pytest.mark.gpu

H = lambda s: int(s, 16)  # noqa: E731


@pytest.fixture(scope="module")
def cx():
    import chordx
    if chordx.device_count() == 0:
        pytest.fail("gpu test without a HIP device")
    return chordx


def _upload(ring, st):
    ring.upload_fingers(st["F"])
    ring.upload_peer_state(min_keys=st.get("min_keys"), preds=st.get("preds"))
    ring.upload_liveness(alive=st.get("alive"), succs=st.get("succs"), ns=st.get("ns", 0),
                         rule=st.get("rule", 0))


@pytest.mark.parametrize("fill", [False, True])
@pytest.mark.parametrize("rule", [0, 1])
def test_get_succ_failing(cx, O, refvec, fill, rule):
    """ChordGetSucc.Failing: GetSuccessor must throw.  Literal state (empty
    finger table) -> CX_Q_NOT_FOUND; every finger = the dead succ ->
    CX_Q_FAILED ("Lookup failed"), for the Chord and the DHash rule."""
    g = refvec["get_succ"]["failing"]
    want_ring, p, st = failing_state(O, g, fill, rule)
    ring = cx.Ring(want_ring)
    assert (ring.ids() == want_ring).all()
    _upload(ring, st)
    owner, hops, status = ring.route(np.array([p], np.uint32), O.keys_from_ints([H(g["key"])]))
    assert status[0] == (cx.CX_Q_FAILED if fill else cx.CX_Q_NOT_FOUND)
    assert owner[0] == cx.CX_NONE and hops[0] == 0
    wo, wh, ws = O.route(O.Peers(want_ring, **st), [p], O.keys_from_ints([H(g["key"])]))
    assert (owner == wo).all() and (hops == wh).all() and (status == ws).all()


@pytest.mark.parametrize("dead", [(), (2,), (3,), (2, 3)])
@pytest.mark.parametrize("rule", [0, 1])
def test_five_peer_fallbacks(cx, O, dead, rule):
    ids = O.keys_from_ints([k << 124 for k in range(1, 6)])
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    alive = np.ones(5, np.uint8)
    alive[list(dead)] = 0
    ring.upload_liveness(alive=alive, ns=3, rule=rule)
    keys = O.keys_from_ints([0x38 << 120, 0, (1 << 128) - 1, 5 << 124, (5 << 124) + 1])
    src = np.zeros(len(keys), np.uint32)
    owner, hops, status = ring.route(src, keys)
    wo, wh, ws = O.route(O.Peers(ids, F, alive=alive, ns=3, rule=rule), src, keys)
    assert (owner == wo).all() and (hops == wh).all() and (status == ws).all()


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("rule", [0, 1])
def test_random_dead_peers(cx, O, seed, rule):
    rng = np.random.default_rng(seed)
    n, q, ns = 300, 20000, 4
    ids = O.ring_build(O.splitmix_keys(0xA9 + seed, n))
    n = len(ids)
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    # churned state: some fingers point at the wrong (possibly dead) peer,
    # a few ranges were never filled, some predecessors unset
    edit = rng.random(F.shape) < 0.05
    F[edit] = rng.integers(0, n, int(edit.sum()))
    F[rng.random(F.shape) < 0.002] = O.NONE
    preds = ((np.arange(n) - 1) % n).astype(np.uint32)
    preds[rng.random(n) < 0.1] = O.NONE
    alive = (rng.random(n) > 0.15).astype(np.uint8)
    succs = ((np.arange(n)[:, None] + 1 + np.arange(ns)[None, :]) % n).astype(np.uint32)
    ragged = rng.integers(0, ns + 1, n)
    for p in range(n):
        succs[p, ragged[p]:] = O.NONE
    st = dict(F=F, preds=preds, alive=alive, succs=succs, rule=rule)
    _upload(ring, st)
    keys = O.splitmix_keys(0xB9 + seed, q)
    src = rng.integers(0, n, q).astype(np.uint32)
    owner, hops, status = ring.route(src, keys)
    wo, wh, ws = O.route(O.Peers(ids, **st), src, keys)
    assert (status == ws).all() and (owner == wo).all() and (hops == wh).all()
    # every outcome kind occurs
    kinds = set(np.unique(ws).tolist())
    assert {0, 3}.issubset(kinds), kinds


def test_rejected_uploads_leave_state(cx, O):
    """A rejected upload (an entry that is neither a ring index nor CX_NONE)
    must leave the current fingers / peer state / liveness untouched."""
    ids = O.ring_build(O.splitmix_keys(77, 50))
    ring = cx.Ring(ids)
    F = ring.build_fingers(copy_out=True)
    keys = O.splitmix_keys(78, 2000)
    src = (np.arange(2000) % len(ids)).astype(np.uint32)
    F2 = F.copy()
    F2[3, :] = 3
    ring.upload_fingers(F2)
    before = ring.route(src, keys)
    bad = F.copy()
    bad[7, 9] = len(ids) + 5
    with pytest.raises(cx.ChordError):
        ring.upload_fingers(bad)
    with pytest.raises(cx.ChordError):
        ring.upload_peer_state(preds=np.full(len(ids), len(ids), np.uint32))
    with pytest.raises(cx.ChordError):
        ring.upload_liveness(succs=np.full((len(ids), 2), len(ids), np.uint32))
    after = ring.route(src, keys)
    for a, b in zip(before, after):
        assert (a == b).all()
    wo, wh, ws = O.route(O.Peers(ids, F2), src, keys)
    assert (after[0] == wo).all() and (after[1] == wh).all()


def test_liveness_reset_restores_converged_walk(cx, O):
    """cx_liveness_upload(NULL, NULL) resets the ring to "all alive, converged
    lists": route() leaves the literal walk (the route table applies again,
    same owners/hops as before any upload) and the arc calls accept the ring
    (the literal walk used to stay on for good)."""
    ids = O.ring_build(O.splitmix_keys(91, 3000))
    ring = cx.Ring(ids)
    ring.build_fingers()
    keys = O.splitmix_keys(92, 4000)
    src = (np.arange(4000) % len(ids)).astype(np.uint32)
    base = ring.route(src, keys)
    alive = np.ones(len(ids), np.uint8)
    alive[::7] = 0
    ring.upload_liveness(alive=alive, rule=cx.CX_FWD_DHASH)
    assert ring.route_info()[0] == -1          # literal walk
    with pytest.raises(cx.ChordError):
        ring.arc_build(2, 0)
    ring.upload_liveness()                     # reset
    assert ring.route_info()[0] == 5           # converged table walk again
    again = ring.route(src, keys)
    for a, b in zip(base, again):
        assert (a == b).all()
    ring.arc_build(2, 0)                       # accepted after the reset
