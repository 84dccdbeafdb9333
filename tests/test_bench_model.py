"""bench.py's request model of the exact successor search
(dir_search_requests): its host replay of the bucket-directory search
(cx_common.hpp dir_successor) must reach the oracle's successor on every key,
or the requests it counts are not the kernel's."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

MAX = (1 << 128) - 1


@pytest.mark.parametrize("kind", ["uniform", "small", "cluster", "edges"])
def test_dir_search_replay_reaches_the_successor(kind):
    import bench
    import oracle as O
    rng = np.random.default_rng(0xD1E)
    if kind == "uniform":
        ids, keys = O.splitmix_keys(11, 1 << 16), O.splitmix_keys(12, 1 << 18)
    elif kind == "small":
        ids, keys = O.splitmix_keys(13, 5), O.splitmix_keys(14, 4000)
    elif kind == "cluster":
        base = 0x0123_4567_89AB << 80
        ids = O.keys_from_ints([base + (int(x) << 30) for x in rng.permutation(5000)] +
                               O.ints_from_keys(O.splitmix_keys(15, 3000)))
        keys = O.keys_from_ints([base + int(x) for x in rng.integers(0, 1 << 44, 20000)] +
                                O.ints_from_keys(O.splitmix_keys(16, 20000)))
    else:
        v = O.ints_from_keys(O.splitmix_keys(17, 3000)) + [0, 1, MAX, MAX - 1]
        ids = O.keys_from_ints(v)
        keys = O.keys_from_ints([(x + d) % (1 << 128) for x in v for d in (-1, 0, 1)] +
                                [0, 1, MAX])
    ring = O.ring_build(ids)
    k = 1
    while (1 << k) < len(ring):
        k += 1
    d, r, ans = bench.dir_search_requests(ring, keys, k + 1, want_index=True)
    assert d == len(keys) and r >= 0
    assert (ans == O.successor(ring, keys)).all()
