"""Python face of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It is the parity checker for the HIP engine, never the product.

Two parts:
  * ctypes bindings to liboracle.so (oracle/chord_oracle.c), the batch
    restatement of the reference's lookup path;
  * `GenericKey`, a pure-Python restatement of the reference's key template
    GenericKey<key_base, key_len> (src/data_structures/key.h:56-281) for the
    arithmetic known-answer tests, including the 8-bit ring of key_test.cc:5.

Keys are numpy uint64 arrays of shape (q, 2): column 0 = low 64 bits,
column 1 = high 64 bits (the cx_u128 / or_key layout).
"""
from __future__ import annotations

import ctypes
import os
import uuid

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
NONE = 0xFFFFFFFF
FINGERS = 128

# --------------------------------------------------------------------------
# Pure-Python restatement of GenericKey (small cases only).
# --------------------------------------------------------------------------


class GenericKey:
    """key.h:56-281 with its uint256_t/cpp_int semantics.

    value is the raw uint256 (may be non-canonical, e.g. 2**128 after 1-1).
    """

    U256 = 1 << 256

    def __init__(self, value: int, base: int = 16, length: int = 32):
        self.base, self.length = base, length
        self.ring = base ** length  # keys_in_ring_, key.h:279-280
        self.value = value % self.U256

    @classmethod
    def from_hex(cls, s: str) -> "GenericKey":  # key.h:73-75
        return cls(int(s, 16))

    @classmethod
    def from_plaintext(cls, s: str) -> "GenericKey":  # key.h:76-79
        return cls(int.from_bytes(uuid.uuid5(uuid.NAMESPACE_DNS, s).bytes, "big"))

    def hex(self) -> str:  # IntToHexStr, key.h:41-47: lowercase, no leading zeros
        return format(self.value, "x")

    def in_between(self, lb: int, ub: int, inclusive: bool = True) -> bool:
        """InBetween, key.h:103-131 (raw-bound compare, equal-bound point test)."""
        lb %= self.U256
        ub %= self.U256
        if lb == ub:
            return self.value == ub
        mlb, mub, mv = lb % self.ring, ub % self.ring, self.value % self.ring
        if lb < ub:
            return (mlb <= mv <= ub) if inclusive else (mlb < mv < ub)
        return not ((mub < mv < mlb) if inclusive else (mub <= mv <= mlb))

    def _new(self, v: int) -> "GenericKey":
        return GenericKey(v, self.base, self.length)

    def __add__(self, other):
        if isinstance(other, GenericKey):  # key.h:252-256
            return self._new((self.value + other.value) % self.ring)
        # key.h:236-240: uint256 add (wraps mod 2^256), then mod ring
        return self._new(((self.value + other) % self.U256) % self.ring)

    def __sub__(self, other):
        if isinstance(other, GenericKey):  # key.h:258-270: signed cpp_int
            diff = self.value - other.value
            return self._new(diff if diff > 0 else self.ring + diff)
        diff = (self.value - other) % self.U256  # key.h:245: uint256 wraps
        return self._new(diff if diff > 0 else self.ring + diff)

    def __eq__(self, other):
        return isinstance(other, GenericKey) and self.value == other.value

    def __hash__(self):
        return hash(self.value)


def nth_range(start: int, n: int):
    """FingerTable::GetNthRange, finger_table.h:177-188 (raw uint256 values)."""
    ring = 1 << 128
    lb = (start + (1 << n)) % ring
    ub = ((start + (1 << (n + 1))) % ring - 1) % GenericKey.U256
    return lb, ub


def uuid5_int(s: str) -> int:
    """Peer/key id from plaintext (abstract_chord_peer.cpp:21, key.h:29-33)."""
    return int.from_bytes(uuid.uuid5(uuid.NAMESPACE_DNS, s).bytes, "big")


# --------------------------------------------------------------------------
# numpy <-> 128-bit helpers
# --------------------------------------------------------------------------


def keys_from_ints(vals) -> np.ndarray:
    vals = list(vals)
    a = np.empty((len(vals), 2), dtype=np.uint64)
    for i, v in enumerate(vals):
        a[i, 0] = v & 0xFFFFFFFFFFFFFFFF
        a[i, 1] = (v >> 64) & 0xFFFFFFFFFFFFFFFF
    return a


def ints_from_keys(a: np.ndarray):
    a = np.asarray(a, dtype=np.uint64).reshape(-1, 2)
    return [int(lo) | (int(hi) << 64) for lo, hi in a]


# --------------------------------------------------------------------------
# ctypes bindings
# --------------------------------------------------------------------------


class _Key(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]


class _U256(ctypes.Structure):
    _fields_ = [("w", ctypes.c_uint64 * 4)]


class _Peers(ctypes.Structure):
    _fields_ = [
        ("ring", ctypes.c_void_p),
        ("n", ctypes.c_size_t),
        ("F", ctypes.c_void_p),
        ("min_keys", ctypes.c_void_p),
        ("preds", ctypes.c_void_p),
        ("alive", ctypes.c_void_p),
        ("succs", ctypes.c_void_p),
        ("ns", ctypes.c_int),
        ("rule", ctypes.c_int),
    ]


Q_OK, Q_HOPCAP, Q_BADPEER, Q_FAILED, Q_NOT_FOUND = 0, 1, 2, 3, 4
FWD_CHORD, FWD_DHASH = 0, 1


_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.or_uuid5_dns.restype = _Key
        L.or_uuid5_dns.argtypes = [ctypes.c_char_p, sz]
        L.or_in_between.restype = i
        L.or_in_between.argtypes = [_U256, _U256, _U256, i]
        L.or_ring_build.restype = sz
        L.or_ring_build.argtypes = [vp, sz, vp]
        L.or_successor_batch.argtypes = [vp, sz, vp, sz, vp, i]
        L.or_fingers_build.argtypes = [vp, sz, vp, i]
        L.or_predecessor_batch.argtypes = [vp, sz, vp, sz, vp, i]
        L.or_fingers_rows.argtypes = [vp, sz, sz, sz, vp, i]
        L.or_finger_index.restype = i
        L.or_finger_index.argtypes = [_Key, _Key]
        L.or_route_batch.argtypes = [ctypes.POINTER(_Peers), vp, vp, sz, vp, vp, vp, i]
        L.or_route_raw_batch.argtypes = [ctypes.POINTER(_Peers), vp, vp, vp, sz, vp, vp, vp]
        L.or_nsucc_batch.argtypes = [ctypes.POINTER(_Peers), vp, vp, sz, i, vp, vp, i]
        L.or_churn.restype = sz
        L.or_churn.argtypes = [vp, sz, vp, sz, vp, sz, vp, vp]
        L.or_misplaced.argtypes = [vp, sz, vp, sz, vp, vp, sz, i, vp, vp, vp, vp, i]
        L.or_misplaced_holders.argtypes = [vp, sz, vp, sz, vp, i, i, vp, vp, vp, vp, i]
        L.or_maintenance_routed.argtypes = [ctypes.POINTER(_Peers), ctypes.POINTER(_Peers), vp, vp,
                                            sz, i, vp, vp, vp, vp, vp, vp, i]
        L.or_splitmix_keys.argtypes = [ctypes.c_uint64, sz, sz, vp]
        L.or_ida_encoding_matrix.argtypes = [i, i, i, vp]
        L.or_ida_vandermonde_inverse.restype = i
        L.or_ida_vandermonde_inverse.argtypes = [vp, i, i, vp]
        L.or_ida_encode_batch.argtypes = [vp, vp, sz, i, i, i, vp]
        L.or_ida_decode_batch.restype = i
        L.or_ida_decode_batch.argtypes = [vp, vp, vp, sz, i, i, vp, vp]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _keys(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64).reshape(-1, 2))


def default_threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def uuid5_key(s: str) -> int:
    k = lib().or_uuid5_dns(s.encode(), len(s.encode()))
    return k.lo | (k.hi << 64)


def _u256(v: int) -> _U256:
    u = _U256()
    for j in range(4):
        u.w[j] = (v >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
    return u


def in_between(v: int, lb: int, ub: int, inclusive: bool = True) -> bool:
    return bool(lib().or_in_between(_u256(v), _u256(lb), _u256(ub), int(inclusive)))


def finger_index(peer_id: int, key: int) -> int:
    to = lambda v: _Key(v & 0xFFFFFFFFFFFFFFFF, v >> 64)  # noqa: E731
    return lib().or_finger_index(to(peer_id), to(key))


def ring_build(ids) -> np.ndarray:
    ids = _keys(ids).copy()
    m = lib().or_ring_build(_p(ids), len(ids), _p(ids))
    return ids[:m].copy()


def successor(ring, keys, threads=None) -> np.ndarray:
    ring, keys = _keys(ring), _keys(keys)
    out = np.empty(len(keys), dtype=np.uint32)
    lib().or_successor_batch(_p(ring), len(ring), _p(keys), len(keys), _p(out),
                             threads or default_threads())
    return out


def predecessor(ring, keys, threads=None) -> np.ndarray:
    ring, keys = _keys(ring), _keys(keys)
    out = np.empty(len(keys), dtype=np.uint32)
    lib().or_predecessor_batch(_p(ring), len(ring), _p(keys), len(keys), _p(out),
                               threads or default_threads())
    return out


def fingers(ring, threads=None, rows=None) -> np.ndarray:
    ring = _keys(ring)
    n = len(ring)
    if rows is None:
        F = np.empty((n, FINGERS), dtype=np.uint32)
        lib().or_fingers_build(_p(ring), n, _p(F), threads or default_threads())
    else:
        p0, p1 = rows
        F = np.empty((p1 - p0, FINGERS), dtype=np.uint32)
        lib().or_fingers_rows(_p(ring), n, p0, p1, _p(F), threads or default_threads())
    return F


class Peers:
    """Keeps the arrays alive for an or_peers struct.

    alive: per-peer 0/1 (None = every server answers); succs: (n, ns) successor
    lists (None = the converged next-ns window); rule: FWD_CHORD / FWD_DHASH."""

    def __init__(self, ring, F, min_keys=None, preds=None, alive=None, succs=None, ns=0,
                 rule=FWD_CHORD):
        self.ring = _keys(ring)
        self.F = np.ascontiguousarray(F, dtype=np.uint32)
        self.min_keys = None if min_keys is None else _keys(min_keys)
        self.preds = None if preds is None else np.ascontiguousarray(preds, dtype=np.uint32)
        self.alive = None if alive is None else np.ascontiguousarray(alive, dtype=np.uint8)
        self.succs = None
        if succs is not None:
            self.succs = np.ascontiguousarray(succs, dtype=np.uint32).reshape(len(self.ring), -1)
            ns = self.succs.shape[1]
        ptr = lambda a: None if a is None else a.ctypes.data  # noqa: E731
        self.s = _Peers(self.ring.ctypes.data, len(self.ring), self.F.ctypes.data,
                        ptr(self.min_keys), ptr(self.preds), ptr(self.alive), ptr(self.succs),
                        int(ns), int(rule))


def route(peers: Peers, src, keys, threads=None):
    keys = _keys(keys)
    src = np.ascontiguousarray(src, dtype=np.uint32)
    q = len(keys)
    owner = np.empty(q, dtype=np.uint32)
    hops = np.empty(q, dtype=np.uint8)
    status = np.empty(q, dtype=np.uint8)
    lib().or_route_batch(ctypes.byref(peers.s), _p(src), _p(keys), q, _p(owner), _p(hops),
                         _p(status), threads or default_threads())
    return owner, hops, status


def hex_value(s: str) -> int:
    """GenericKey(s, hashed = true).value_ = uint256("0x" + s) (key.h:73-75) as
    a Python int: Boost's unchecked 256-bit cpp_int keeps the value mod 2^256
    (strings over 64 hex digits are parity unpinned: no reference fixture
    holds one).  Raises ValueError where boost's parse throws."""
    if not s or any(c not in "0123456789abcdefABCDEF" for c in s):
        raise ValueError(f"not a hex key: {s!r}")
    return int(s, 16) & ((1 << 256) - 1)


def route_raw(peers: Peers, src, values):
    """or_route on raw uint256 key values (Python ints < 2^256)."""
    values = [int(v) for v in values]
    lo = keys_from_ints([v & ((1 << 128) - 1) for v in values])
    hi = keys_from_ints([v >> 128 for v in values])
    src = np.ascontiguousarray(src, dtype=np.uint32)
    q = len(values)
    owner = np.empty(q, dtype=np.uint32)
    hops = np.empty(q, dtype=np.uint8)
    status = np.empty(q, dtype=np.uint8)
    lib().or_route_raw_batch(ctypes.byref(peers.s), _p(src), _p(lo), _p(hi), q, _p(owner),
                             _p(hops), _p(status))
    return owner, hops, status


def nsucc(peers: Peers, keys, n, src=None, threads=None):
    keys = _keys(keys)
    q = len(keys)
    lists = np.empty((q, n), dtype=np.uint32)
    count = np.empty(q, dtype=np.uint8)
    src = None if src is None else np.ascontiguousarray(src, dtype=np.uint32)
    lib().or_nsucc_batch(ctypes.byref(peers.s), _p(src), _p(keys), q, n, _p(lists),
                         _p(count), threads or default_threads())
    return lists, count


def churn(old_ring, joins, leaves):
    old_ring, joins, leaves = _keys(old_ring), _keys(joins), _keys(leaves)
    new_ring = np.empty((len(old_ring) + len(joins), 2), dtype=np.uint64)
    o2n = np.empty(len(old_ring), dtype=np.uint32)
    m = lib().or_churn(_p(old_ring), len(old_ring), _p(joins), len(joins), _p(leaves),
                       len(leaves), _p(new_ring), _p(o2n))
    return new_ring[:m].copy(), o2n


def misplaced(old_ring, new_ring, o2n, keys, n, threads=None):
    old_ring, new_ring, keys = _keys(old_ring), _keys(new_ring), _keys(keys)
    o2n = np.ascontiguousarray(o2n, dtype=np.uint32)
    q = len(keys)
    lists = np.empty((q, n), dtype=np.uint32)
    count = np.empty(q, dtype=np.uint8)
    mask = np.empty(q, dtype=np.uint16)
    target = np.empty((q, n), dtype=np.uint8)
    lib().or_misplaced(_p(old_ring), len(old_ring), _p(new_ring), len(new_ring), _p(o2n),
                       _p(keys), q, n, _p(lists), _p(count), _p(mask), _p(target),
                       threads or default_threads())
    return lists, count, mask, target


def maintenance_routed(P_old: Peers, P_new: Peers, o2n, keys, n, threads=None):
    """C5 by routed lookups (or_maintenance_routed): (old_lists, old_count,
    new_lists, count, mask, target), lookups from peer q mod n of each ring."""
    keys = _keys(keys)
    o2n = np.ascontiguousarray(o2n, dtype=np.uint32)
    q = len(keys)
    old_lists = np.empty((q, n), dtype=np.uint32)
    old_count = np.empty(q, dtype=np.uint8)
    lists = np.empty((q, n), dtype=np.uint32)
    count = np.empty(q, dtype=np.uint8)
    mask = np.empty(q, dtype=np.uint16)
    target = np.empty((q, n), dtype=np.uint8)
    lib().or_maintenance_routed(ctypes.byref(P_old.s), ctypes.byref(P_new.s), _p(o2n), _p(keys), q,
                                n, _p(old_lists), _p(old_count), _p(lists), _p(count), _p(mask),
                                _p(target), threads or default_threads())
    return old_lists, old_count, lists, count, mask, target


def misplaced_holders(ring, keys, holders, n, threads=None):
    ring, keys = _keys(ring), _keys(keys)
    holders = np.ascontiguousarray(holders, dtype=np.uint32)
    q, nh = holders.shape
    lists = np.empty((q, n), dtype=np.uint32)
    count = np.empty(q, dtype=np.uint8)
    mask = np.empty(q, dtype=np.uint16)
    target = np.empty((q, nh), dtype=np.uint8)
    lib().or_misplaced_holders(_p(ring), len(ring), _p(keys), q, _p(holders), nh, n, _p(lists),
                               _p(count), _p(mask), _p(target), threads or default_threads())
    return lists, count, mask, target


def splitmix_keys(seed: int, count: int, offset: int = 0) -> np.ndarray:
    out = np.empty((count, 2), dtype=np.uint64)
    lib().or_splitmix_keys(seed, offset, count, _p(out))
    return out


# ---------------------------------------------------------------------------
# Rabin IDA (ida_oracle.c): ida.cpp / matrix_math.cpp restated.
# ---------------------------------------------------------------------------
def ida_segments(lengths, m):
    """seg_offsets (blocks + 1,) uint64 of ceil(len / m) segments per block."""
    S = [(int(n) + m - 1) // m for n in lengths]
    out = np.zeros(len(S) + 1, dtype=np.uint64)
    out[1:] = np.cumsum(S, dtype=np.uint64)
    return out


def ida_encode(blocks, n=14, m=10, p=257):
    """Fragments of each datum: list of (n, S_b) uint16 arrays (IDA::Encode)."""
    blocks = [bytes(b) for b in blocks]
    offs = np.zeros(len(blocks) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(b) for b in blocks], dtype=np.uint64)
    data = np.frombuffer(b"".join(blocks) + b"\0", dtype=np.uint8)
    seg = ida_segments([len(b) for b in blocks], m)
    frags = np.zeros(max(1, int(seg[-1]) * n), dtype=np.uint16)
    lib().or_ida_encode_batch(_p(data), _p(offs), len(blocks), n, m, p, _p(frags))
    out = []
    for b in range(len(blocks)):
        S = int(seg[b + 1] - seg[b])
        out.append(frags[n * int(seg[b]): n * int(seg[b]) + n * S].reshape(n, S).copy())
    return out


def ida_decode(frag_rows, indices, m=10, p=257):
    """IDA::Decode of each block from m fragment rows ((m, S_b) arrays) with
    1-based indices: list of uint16 value arrays (trailing zeros dropped)."""
    seg = ida_segments([np.asarray(f).shape[1] * m for f in frag_rows], m)
    flat = np.concatenate([np.asarray(f, dtype=np.uint16).reshape(-1) for f in frag_rows] +
                          [np.zeros(1, np.uint16)])
    idx = np.ascontiguousarray(np.asarray(indices, dtype=np.uint8).reshape(-1, m))
    out = np.zeros(max(1, int(seg[-1]) * m), dtype=np.uint16)
    ln = np.zeros(len(frag_rows), dtype=np.uint64)
    if lib().or_ida_decode_batch(_p(flat), _p(seg), _p(idx), len(frag_rows), m, p, _p(out),
                                 _p(ln)) != 0:
        raise RuntimeError("N is not invertible")
    return [out[m * int(seg[b]): m * int(seg[b]) + int(ln[b])].copy()
            for b in range(len(frag_rows))]


def ida_inverse(basis, p=257):
    m = len(basis)
    b = np.asarray(basis, dtype=np.int32)
    out = np.zeros((m, m), dtype=np.int32)
    if lib().or_ida_vandermonde_inverse(_p(b), m, p, _p(out)) != 0:
        raise RuntimeError("N is not invertible")
    return out
