"""cx_fingers_build without fingers_out on a ring of 2^18 peers or more hands
the default route only the finger levels its table reads and writes the
row-major finger table (PopulateFingerTable, abstract_chord_peer.cpp:564-613)
when it is first read.  The deferred table must be the oracle's, every reader
must see it complete, and routes must not change when it appears."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cx():
    import chordx
    if chordx.device_count() == 0:
        pytest.fail("gpu test without a HIP device")
    return chordx


@pytest.fixture(scope="module")
def setup(cx, O):
    ids = O.splitmix_keys(0x5EED0301, (1 << 18) + 3)
    want = O.ring_build(ids)
    return ids, want, O.fingers(want)


def test_deferred_rows_route_then_read(cx, O, setup):
    ids, want, F = setup
    ring = cx.Ring(ids)
    ring.build_fingers()
    q = 1 << 15
    keys = O.splitmix_keys(0x5EED0302, q)
    src = (np.arange(q) % ring.n).astype(np.uint32)
    o1, h1, s1 = ring.route(src, keys)  # cz walk; exact hops from the directory
    wo, wh, _ = O.route(O.Peers(want, F), src[:4096], keys[:4096])
    assert (o1[:4096] == wo).all() and (h1[:4096] == wh).all() and (s1 == 0).all()
    got = ring.fingers_device().cpu().numpy().view(np.uint32)  # written now
    assert (got == F).all()
    o2, h2, s2 = ring.route(src, keys)  # the walk now reads the rows
    assert (o1 == o2).all() and (h1 == h2).all() and (s2 == 0).all()


def test_deferred_rows_other_readers(cx, O, setup):
    """A non-default walk, a rebuild with fingers_out, and the arc build each
    write the deferred rows before reading them."""
    ids, want, F = setup
    q = 1 << 14
    keys = O.splitmix_keys(0x5EED0303, q)
    src = (np.arange(q) % len(want)).astype(np.uint32)
    base = cx.Ring(ids)
    base.build_fingers()
    ob, hb, _ = base.route(src, keys)
    r4 = cx.Ring(ids)
    r4.build_fingers()
    r4.set_route_variant(4)  # lookahead-tree walk: reads rows
    o4, h4, s4 = r4.route(src, keys)
    assert (o4 == ob).all() and (h4 == hb).all() and (s4 == 0).all()
    rc = cx.Ring(ids)
    rc.build_fingers()
    assert (rc.build_fingers(copy_out=True) == F).all()
    ra = cx.Ring(ids)
    ra.build_fingers()
    ra.arc_build(1, 0)
    assert (ra.fingers_device().cpu().numpy().view(np.uint32) == F).all()


def test_deferred_rows_concurrent_first_readers(cx, O, setup):
    """Several host threads ask for the deferred table at once: each gets the
    complete table."""
    ids, want, F = setup
    ring = cx.Ring(ids)
    ring.build_fingers()
    out, errs = [None] * 4, []

    def read(i):
        try:
            out[i] = ring.fingers_device().cpu().numpy().view(np.uint32).copy()
        except Exception as e:  # pragma: no cover
            errs.append(e)

    th = [threading.Thread(target=read, args=(i,)) for i in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    for got in out:
        assert (got == F).all()
