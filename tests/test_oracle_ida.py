"""Pins the IDA oracle (oracle/ida_oracle.c) on CPU.

* The reference's own DHash test data (tests/golden/reference_vectors.json,
  "ida_values") must read back unchanged through encode -> any m of n
  fragments -> decode, with each test's (n, m, p).
* A second, independent restatement in pure Python (below, following
  ida.cpp:59-190 and matrix_math.cpp:21-168 line by line, C++ `int` modelled as
  wrapping int32) must agree with the C oracle value for value.
* The int32 corner: for (14, 10, 257) only fragment sets whose elementary
  symmetric sums e_1..e_9 leave int range (7 of the 1001 sets) decode to
  something else (the reference as compiled does the same; unpinned by any
  reference test, see ida_oracle.c).
"""
import itertools
import random

import numpy as np
import pytest

I32 = 1 << 32


def wrap(x):
    x %= I32
    return x - I32 if x >= 1 << 31 else x


def cmod(lhs, rhs):  # Modulo with C++ truncating %
    r = abs(lhs) % rhs
    r = -r if lhs < 0 else r
    return (r + rhs) % rhs


def py_encoding_matrix(m, n, p):
    rows = []
    for a in range(1, n + 1):
        row, elt = [], 1
        for _ in range(m):
            row.append(elt)
            elt = cmod(elt * a, p)
        rows.append(row)
    return rows


def py_mod_inverse(n, p):
    t, new_t, r, new_r = 0, 1, p, n
    while new_r:
        q = int(r / new_r)  # C++ truncation
        t, new_t = new_t, t - q * new_t
        r, new_r = new_r, r - q * new_r
    if r > 1:
        raise ZeroDivisionError("N is not invertible")
    return t + p if t < 0 else t


def py_vandermonde_inverse(basis, p):
    m = len(basis)
    el = [[0] * (m + 1) for _ in range(m + 1)]
    for i in range(1, m + 1):
        el[1][i] = wrap(el[1][i - 1] + basis[i - 1])
    for i in range(2, m + 1):
        for j in range(i, m + 1):
            el[i][j] = wrap(el[i - 1][j - 1] * basis[j - 1] + el[i][j - 1])
    sym = [el[i][m] for i in range(m + 1)]
    dens = []
    for i in range(m):
        prod = 1
        for j in range(m):
            if j != i:
                prod = cmod(prod * (basis[i] - basis[j]), p)
        dens.append(prod)
    res = []
    for i in range(m):
        row, sign = [1], -1
        for j in range(1, m):
            row.append(cmod(wrap(cmod(row[-1] * basis[i], p) + wrap(sign * sym[j])), p))
            sign = -sign
        row.reverse()
        inv = py_mod_inverse(dens[i], p)
        res.append([cmod(x * inv, p) for x in row])
    return [[res[j][i] for j in range(m)] for i in range(m)]


def py_encode(data, n, m, p):
    E = py_encoding_matrix(m, n, p)
    segs = [list(data[i:i + m]) + [0] * (m - len(data[i:i + m])) for i in range(0, len(data), m)]
    return [[cmod(sum(a * b for a, b in zip(E[i], s)), p) for s in segs] for i in range(n)]


def py_decode(frags, idx, m, p):
    inv = py_vandermonde_inverse(list(idx[:m]), p)
    S = len(frags[0])
    outm = [[0] * S for _ in range(m)]
    for i in range(m):
        for j in range(S):
            c = 0
            for k in range(m):
                c = cmod(wrap(c + inv[i][k] * frags[k][j]), p)
            outm[i][j] = c
    segs = [[outm[j][i] for j in range(m)] for i in range(S)]
    while segs and not any(segs[-1]):
        segs.pop()
    while segs and segs[-1][-1] == 0:
        segs[-1].pop()
    return [v for s in segs for v in s]


def int32_corner(idx):
    """True when an elementary symmetric sum e_1..e_(m-1) of the indices (the
    ones the numerators read, matrix_math.cpp:139) leaves int range."""
    m = len(idx)
    e = [1] + [0] * m
    for x in idx:
        for j in range(m, 0, -1):
            e[j] += e[j - 1] * x
    return any(e[j] >= 1 << 31 for j in range(1, m))


def test_golden_values_read_back(O, refvec):
    for case in refvec["ida_values"]:
        n, m, p = case["nmp"]
        data = [v.encode() for v in case["values"]]
        frags = O.ida_encode(data, n, m, p)
        for d, f in zip(data, frags):
            assert f.shape == (n, (len(d) + m - 1) // m)
            for sub in itertools.combinations(range(n), m):
                got = O.ida_decode([f[list(sub)]], [[s + 1 for s in sub]], m, p)[0]
                if int32_corner([s + 1 for s in sub]):
                    continue  # int32 corner, below
                assert bytes(got.astype(np.uint8)) == d and got.max() < 256


@pytest.mark.parametrize("nmp", [(14, 10, 257), (3, 2, 257), (2, 1, 257), (9, 4, 263),
                                 (20, 12, 40009)])
def test_c_oracle_equals_python_twin(O, nmp):
    n, m, p = nmp
    rng = random.Random(n * 1000 + m)
    for _ in range(3):
        data = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 3 * m + 7)))
        f = O.ida_encode([data], n, m, p)[0]
        assert f.tolist() == py_encode(data, n, m, p)
        subs = list(itertools.combinations(range(n), m))
        for sub in rng.sample(subs, min(40, len(subs))):
            sub = list(sub)
            rng.shuffle(sub)
            idx = [s + 1 for s in sub]
            got = O.ida_decode([f[sub]], [idx], m, p)[0].tolist()
            assert got == py_decode([f[s].tolist() for s in sub], idx, m, p)
            assert (O.ida_inverse(idx, p) == np.array(py_vandermonde_inverse(idx, p))).all()


def test_int32_corner_for_default_params(O):
    """Fragment sets of (14, 10) whose symmetric sums leave int range."""
    data = bytes(range(1, 200))
    f = O.ida_encode([data])[0]
    wrong = []
    for sub in itertools.combinations(range(14), 10):
        got = O.ida_decode([f[list(sub)]], [[s + 1 for s in sub]])[0]
        if len(got) != len(data) or got.max() > 255 or bytes(got.astype(np.uint8)) != data:
            wrong.append(tuple(s + 1 for s in sub))
    overflow = [tuple(s + 1 for s in sub) for sub in itertools.combinations(range(14), 10)
                if int32_corner([s + 1 for s in sub])]
    assert wrong and set(wrong) <= set(overflow)
    assert (1, 2, 3, 4, 5, 6, 7, 8, 9, 10) not in wrong  # what an all-alive Read uses
    assert (5, 6, 7, 8, 9, 10, 11, 12, 13, 14) in wrong


def test_decode_edge_cases(O):
    f = O.ida_encode([b"", b"\0\0\0", b"ab\0\0"])
    assert f[0].shape == (14, 0)
    idx = [list(range(1, 11))] * 2
    out = O.ida_decode([f[1][:10], f[2][:10]], idx)
    assert out[0].size == 0                     # all zero: nothing kept
    assert bytes(out[1].astype(np.uint8)) == b"ab"  # trailing zero bytes dropped
    with pytest.raises(RuntimeError):
        O.ida_decode([f[2][:10]], [[1, 1, 2, 3, 4, 5, 6, 7, 8, 9]])  # repeated index
