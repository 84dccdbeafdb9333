"""Table pool (include/chordx.h cx_pool_trim / cx_pool_info): a destroyed
ring's tables wait in the pool for the next ring of the same size, the next
ring of that size takes them back (same route table, same answers), and
cx_pool_trim releases them."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cx():
    import chordx
    if chordx.device_count() == 0:
        pytest.fail("gpu test without a HIP device")
    return chordx


@pytest.mark.skipif(os.environ.get("CX_POOL_CAP_GIB", "").strip() == "0",
                    reason="the table pool is disabled (CX_POOL_CAP_GIB=0)")
def test_pool_keeps_and_trims_tables(cx, O):
    import torch
    n = 1 << 18
    ids = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    cx.fill_splitmix(ids, 0x9001)
    keys = O.splitmix_keys(0x9002, 4096)
    src = (np.arange(4096) % n).astype(np.uint32)
    cx.pool_trim()
    assert cx.pool_info() == (0, 0)
    r1 = cx.Ring(ids)
    r1.build_fingers()
    h1 = r1.route_table_hash()
    a1 = r1.route(src, keys)
    r1.close()
    blocks, nbytes = cx.pool_info()
    assert blocks >= 2 and nbytes >= n * 128 * 4  # the finger table at least
    r2 = cx.Ring(ids)
    r2.build_fingers()  # takes the pooled blocks back
    assert cx.pool_info()[1] < nbytes
    assert r2.route_table_hash() == h1
    for a, b in zip(a1, r2.route(src, keys)):
        assert (a == b).all()
    r2.close()
    cx.pool_trim()
    assert cx.pool_info() == (0, 0)
