"""Raw-value (>= 2^128) wire keys in the oracle: GenericKey keeps
uint256("0x" + s) (key.h:73-75); InBetween's point test (key.h:108-113) sees
the raw value, its ranged tests the value mod 2^128 (key.h:116-118).  These
pin the rule cx_wire.cpp's wide_keys applies on the GPU results."""
import numpy as np
import pytest

MASK = (1 << 128) - 1


def test_hex_value(O):
    assert O.hex_value("ff") == 255
    assert O.hex_value("1" + "0" * 32) == 1 << 128
    assert O.hex_value("f" * 64) == (1 << 256) - 1
    assert O.hex_value("1" + "0" * 64) == 0              # unchecked uint256 wraps
    for bad in ("", "0x1", "g", " 1"):
        with pytest.raises(ValueError):
            O.hex_value(bad)


def test_wide_keys_route_as_mod_except_point_tests(O):
    ring = O.ring_build(O.splitmix_keys(0x77, 200))
    P = O.Peers(ring, O.fingers(ring))
    ids = O.ints_from_keys(ring)
    n = len(ids)
    rnd = np.random.default_rng(3)
    vals = [int(rnd.integers(1, 1 << 62)) << 192 | (int(rnd.integers(0, 1 << 62)) << 64)
            | int(rnd.integers(0, 1 << 62)) for _ in range(300)]
    src = rnd.integers(0, n, len(vals))
    o, h, st = O.route_raw(P, src, vals)
    o2, h2, st2 = O.route(P, src, O.keys_from_ints([v & MASK for v in vals]))
    assert (st == 0).all() and (o == o2).all() and (h == h2).all()


def test_wide_key_next_to_an_id_fails_iff_the_walk_visits_it(O):
    """m = id(x) + 1 with a raw value >= 2^128 fails finger 0's point range
    [id+1, id+1] at x ("ChordKey not found", finger_table.h:129); the walk to
    m visits x iff hops(m) == hops(id(x)) + 1 (cx_wire.cpp wide_keys)."""
    for seed, n in ((1, 64), (2, 300), (3, 2), (4, 3)):
        ring = O.ring_build(O.splitmix_keys(seed, n))
        P = O.Peers(ring, O.fingers(ring))
        ids = O.ints_from_keys(ring)
        src = np.arange(n, dtype=np.uint32)
        for x in range(n):
            m = (ids[x] + 1) & MASK
            _, _, st = O.route_raw(P, src, [(1 << 128) | m] * n)
            _, h1, _ = O.route(P, src, O.keys_from_ints([m] * n))
            _, h0, _ = O.route(P, src, O.keys_from_ints([ids[x]] * n))
            assert ((st == 4) == (h1.astype(int) == h0.astype(int) + 1)).all()
            assert set(st.tolist()) <= {0, 4}


def test_wide_key_equal_to_an_adjacent_id_never_resolves(O):
    """Owner o with pred id = id(o) - 1: StoredLocally(o) is a point test
    (min_key == id), so key id(o) + 2^128 fails from every source."""
    base = O.ints_from_keys(O.splitmix_keys(5, 40))
    ring = O.ring_build(O.keys_from_ints(base + [(base[0] + 1) & MASK]))
    ids = O.ints_from_keys(ring)
    o = ids.index((base[0] + 1) & MASK)
    P = O.Peers(ring, O.fingers(ring))
    n = len(ids)
    src = np.arange(n, dtype=np.uint32)
    _, _, st = O.route_raw(P, src, [(1 << 128) | ids[o]] * n)
    assert (st == 4).all()
    _, _, st = O.route(P, src, O.keys_from_ints([ids[o]] * n))
    assert (st == 0).all()
