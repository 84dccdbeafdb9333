"""Variable 128-bit shifts on gfx950 against host arithmetic (tests/hip/
u128_check.hip, libcxtest.so: test-only kernels, not the engine).

Round-5 VERDICT "What's weak" #2: a route-table word that differed by lane and
run was patched by replacing the exact-ID branch of the gap code (a variable
`u128 >> gs`) with 64-bit halves.  These tests settle whether the compiler's
shift lowering is involved: every amount 0..127 per lane (VGPR amounts), as a
kernel argument (SGPR amounts) and under lane-divergent branches, plus the
round-5 encode itself, standalone, on the operands of the failing ring (a
dense cluster whose fingers all wrap: the exact-ID branch on most words) and
on random operands.  Host results are Python integers (the reference's
uint128 arithmetic, key.h:236-270)."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
M128 = (1 << 128) - 1


@pytest.fixture(scope="module")
def T():
    path = os.path.join(HERE, "hip", "libcxtest.so")
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: make -C tests/hip")
    L = ctypes.CDLL(path)
    vp, u32, i = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
    L.cxt_shifts.argtypes = [vp, vp, i, vp, u32]
    L.cxt_encode_r5.argtypes = [u32, i, vp, vp, vp, vp, i, vp, u32]
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _ints(a):
    return [int(lo) | (int(hi) << 64) for lo, hi in a.reshape(-1, 2)]


def _cells(vals):
    return np.array([[v & (2**64 - 1), v >> 64] for v in vals], dtype=np.uint64)


def test_u128_shifts_all_amounts(T):
    rng = np.random.default_rng(0x5A1F7)
    q = 128 * 64  # every amount on every lane position of a wave, 64 values each
    vals = [int(x) for x in rng.integers(0, 2**63, size=q)]
    vals = [(v << 65) ^ (v * 0x9E3779B97F4A7C15) & M128 for v in vals]
    vals[:4] = [M128, 1, 1 << 127, 0]
    lane = np.arange(q)
    amt = ((lane * 37 + (lane >> 7)) % 128).astype(np.int32)  # lane-varying, all 128
    x = _cells(vals)
    for ua in (0, 1, 31, 63, 64, 65, 96, 103, 127):
        out = np.zeros((q * 6, 2), dtype=np.uint64)
        assert T.cxt_shifts(_p(x), _p(amt), ua, _p(out), q) == 0
        got = _ints(out)
        bad = []
        for j, v in enumerate(vals):
            a = int(amt[j])
            want = [(v << a) & M128, v >> a, (v << ua) & M128, v >> ua, (v << a) & M128, v >> a]
            if got[6 * j: 6 * j + 6] != want:
                bad.append((j, a, ua))
        assert not bad, bad[:8]


def _encode_r5_host(n, gs, ids, par, x, l):
    def expect(l_):
        sh = 128 - l_
        return 0 if sh > 40 else (n + (1 << (sh - 1))) >> sh
    d = x - par - expect(l)
    h = n // 2
    lo, hi = max(h + 1 - n, -32768), min(h, 32766)
    if not lo <= d <= hi:
        if d < 0:
            d += n
        if d < 0:
            d += n
        if d > h:
            d -= n
    code = ((ids[x] - ids[par] - (1 << l)) & M128) >> gs
    if code >= 1 << 64:
        code = 2**64 - 1
    if d < -32768 or d > 32766 or code >= 0xFFFF:
        return 0xFFFFFFFF
    return (code << 16) | (d + 32768)


@pytest.mark.parametrize("ring_kind", ["cluster", "uniform"])
def test_round5_encode_standalone(T, O, ring_kind):
    """The pre-0a5da05 encode outside the build kernel, per-lane and uniform
    levels: equal to host arithmetic on every operand set."""
    if ring_kind == "cluster":  # the ring of test_route_table_builds_deterministic_all_escapes
        base = 0x3C3C_5A5A_0F0F_1234 << 64
        ids = [base + i * 7919 for i in range(6000)]
    else:
        ids = sorted(set(O.ints_from_keys(O.splitmix_keys(0xE17C0, 6000))))
    n = len(ids)
    ib = max(1, (n - 1).bit_length())
    gs = 116 - ib
    R = ((ib + 8 + 3) // 4) * 4
    levels = list(range(128 - R - 5, 128))
    rng = np.random.default_rng(0xE5C)
    q = 1 << 16
    par = rng.integers(0, n, size=q).astype(np.uint32)
    x = rng.integers(0, n, size=q).astype(np.uint32)
    # half the operand sets as the build forms them: x = the finger of par at l
    lv = rng.choice(levels, size=q).astype(np.int32)
    import bisect
    for j in range(0, q, 2):
        t = (ids[par[j]] + (1 << int(lv[j]))) & M128
        k = bisect.bisect_left(ids, t)
        x[j] = k if k < n else 0
    ring = _cells(ids)
    want = [_encode_r5_host(n, gs, ids, int(par[j]), int(x[j]), int(lv[j])) for j in range(q)]
    out = np.zeros(q, dtype=np.uint32)
    assert T.cxt_encode_r5(n, gs, _p(ring), _p(par), _p(x), _p(lv), -1, _p(out), q) == 0
    assert [int(v) for v in out] == want
    for lvl in (levels[0], 103, 104, 108, 127):
        lu = np.full(q, lvl, dtype=np.int32)
        wu = [_encode_r5_host(n, gs, ids, int(par[j]), int(x[j]), lvl) for j in range(q)]
        assert T.cxt_encode_r5(n, gs, _p(ring), _p(par), _p(x), _p(lu), lvl, _p(out), q) == 0
        assert [int(v) for v in out] == wu, lvl
