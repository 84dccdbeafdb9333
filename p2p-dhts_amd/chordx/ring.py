"""Ring handle: the batched replacement for a converged Chord ring of peers.

Mirrors what a ChordPeer/DHashPeer exposes on the lookup path
(abstract_chord_peer.h:113-160, finger_table.h:30-288, dhash_peer.h:54-81),
batched over keys and source peers:

  ChordPeer API (reference)                      Ring method
  ---------------------------------------------  -----------------------------
  converged successor ring (Join/Stabilize)      Ring(ids)  (GPU radix sort)
  StoredLocally / owner of a key                 successor(keys)
  GetPredecessor(key)                            predecessor(keys)
  PopulateFingerTable (converged)                build_fingers()
  EditNthFinger / AdjustFingers (hand edits)     upload_fingers(F)
  min_key_ / predecessor_ (white-box state)      upload_peer_state(...)
  GetSuccessor(key) from peer src (+ hops)       route(src, keys)
  GetNSuccessors(key, n)                         nsucc(keys, n)
  batched Join/Leave                             churn(joins, leaves)
  RunGlobalMaintenance misplaced check           misplaced(...), misplaced_holders(...)
  ChordKey::InBetween                            in_between(...)

Buffers: numpy arrays are host memory (staged by the library); torch CUDA
tensors are device memory, and the call is ordered on torch's current stream.
128-bit values are (q, 2) arrays of uint64 (numpy) / int64 (torch):
column 0 = low 64 bits, column 1 = high 64 bits.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L

try:  # torch is optional plumbing (device memory, streams)
    import torch
except Exception:  # pragma: no cover
    torch = None


def _is_dev(x) -> bool:
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def _keys_np(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64).reshape(-1, 2))


def _check_dev(t, esize: int, name: str, device=None, count=None):
    """A device tensor handed to the library as a raw pointer must have the
    element width the C ABI reads/writes, be contiguous, live on the ring's
    GPU and hold `count` elements (first dimension); anything else would be an
    out-of-bounds or misread GPU access, so it is rejected here."""
    if not _is_dev(t):
        return
    if t.element_size() != esize or t.is_floating_point() or t.is_complex():
        raise TypeError(f"{name}: expected a {8 * esize}-bit integer tensor, got {t.dtype}")
    if not t.is_contiguous():
        raise TypeError(f"{name}: tensor must be contiguous")
    if device is not None and (t.device.index or 0) != device:
        raise TypeError(f"{name}: tensor on cuda:{t.device.index}, ring on cuda:{device}")
    if count is not None and (t.dim() == 0 or t.shape[0] != count):
        raise TypeError(f"{name}: expected first dimension {count}, got {tuple(t.shape)}")


def _ptr(a):
    if a is None:
        return None
    if _is_dev(a):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


class Ring:
    """Sorted, de-duplicated ring of 128-bit peer IDs on one GPU."""

    arc_hints = True  # arc_partition_regions(..., hints=True) / arc_route(..., hint=)

    def __init__(self, ids, device: int = 0, _handle=None):
        self._h = None
        if _handle is not None:
            self._h = _handle
        else:
            h = ctypes.c_void_p()
            if _is_dev(ids):
                ids = ids.contiguous()
                assert ids.dim() == 2 and ids.shape[1] == 2 and ids.element_size() == 8
                device = ids.device.index or 0
                # the build runs on the handle's own stream: order it after torch's
                torch.cuda.current_stream(device).synchronize()
                L.check(L.lib().cx_ring_create(_ptr(ids), ids.shape[0], L.CX_MEM_DEVICE, device,
                                               ctypes.byref(h)))
            else:
                ids = _keys_np(ids)
                L.check(L.lib().cx_ring_create(_ptr(ids), len(ids), L.CX_MEM_HOST, device,
                                               ctypes.byref(h)))
            self._h = h
        self.device = device
        n = ctypes.c_size_t()
        L.check(L.lib().cx_ring_size(self._h, ctypes.byref(n)))
        self.n = n.value

    # ---- lifecycle -------------------------------------------------------
    def close(self):
        if self._h is not None:
            L.lib().cx_ring_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self.n

    def _torch_stream(self):
        """Order the library's work on torch's current stream (one ABI call
        only when that stream changed: small batches are host-bound)."""
        cs = torch.cuda.current_stream(self.device).cuda_stream
        if self.__dict__.get("_stream_set") != cs:
            L.check(L.lib().cx_ring_set_stream(self._h, ctypes.c_void_p(cs)))
            self._stream_set = cs

    def _mem(self, *arrays) -> int:
        dev = [_is_dev(a) for a in arrays if a is not None]
        if dev and all(dev):
            self._torch_stream()
            return L.CX_MEM_DEVICE
        if any(dev):
            raise TypeError("mix of device tensors and host arrays")
        L.check(L.lib().cx_ring_use_own_stream(self._h))
        self._stream_set = None
        return L.CX_MEM_HOST

    def _empty(self, like, shape, np_dtype, th_dtype):
        if _is_dev(like):
            return torch.empty(shape, dtype=th_dtype, device=like.device)
        return np.empty(shape, dtype=np_dtype)

    def _prep_keys(self, keys, name="keys"):
        if _is_dev(keys):
            if keys.element_size() != 8 or keys.is_floating_point() or keys.numel() % 2:
                raise TypeError(f"{name}: 128-bit values are (q, 2) int64 device tensors, "
                                f"got {keys.dtype} {tuple(keys.shape)}")
            keys = keys.contiguous().view(-1, 2)
            _check_dev(keys, 8, name, self.device)
            return keys
        return _keys_np(keys)

    def _prep_u32(self, a, name="indices", count=None):
        if _is_dev(a):
            a = a.contiguous()
            _check_dev(a, 4, name, self.device, count)
            return a
        a = np.ascontiguousarray(a, dtype=np.uint32)
        if count is not None and a.shape[0] != count:
            raise TypeError(f"{name}: expected first dimension {count}, got {a.shape}")
        return a

    def _check_out(self, arrays, q):
        """Caller-supplied outputs: (array, element bytes, name) triples."""
        for a, esize, name in arrays:
            if a is None:
                continue
            if _is_dev(a):
                _check_dev(a, esize, name, self.device, q)
            elif (not isinstance(a, np.ndarray) or a.dtype.itemsize != esize
                  or not a.flags.c_contiguous or a.shape[0] != q):
                raise TypeError(f"{name}: expected a contiguous ({q}, ...) array of "
                                f"{esize}-byte integers")

    def ids(self) -> np.ndarray:
        out = np.empty((self.n, 2), dtype=np.uint64)
        L.check(L.lib().cx_ring_ids(self._h, _ptr(out), L.CX_MEM_HOST))
        return out

    def ids_device(self):
        """Zero-copy view of the ring's sorted IDs as a torch int64 (n, 2) tensor."""
        p = ctypes.c_void_p()
        L.check(L.lib().cx_ring_ids_device(self._h, ctypes.byref(p)))
        return _wrap_device(p.value, (self.n, 2), torch.int64, self.device, self)

    def sync(self):
        L.check(L.lib().cx_ring_sync(self._h))

    # ---- a5/a7 -----------------------------------------------------------
    def successor(self, keys, out=None):
        keys = self._prep_keys(keys)
        q = keys.shape[0]
        owner = out if out is not None else self._empty(keys, (q,), np.uint32, torch and torch.int32)
        self._check_out([(owner, 4, "owner")], q)
        mk = self._mem(keys, owner)
        L.check(L.lib().cx_successor(self._h, _ptr(keys), q, _ptr(owner), mk))
        return owner

    def predecessor(self, keys, out=None):
        """GetPredecessor(key) on the converged ring: the owner's predecessor."""
        keys = self._prep_keys(keys)
        q = keys.shape[0]
        pred = out if out is not None else self._empty(keys, (q,), np.uint32, torch and torch.int32)
        self._check_out([(pred, 4, "pred")], q)
        mk = self._mem(keys, pred)
        L.check(L.lib().cx_predecessor(self._h, _ptr(keys), q, _ptr(pred), mk))
        return pred

    # ---- a4/a6 -----------------------------------------------------------
    def build_fingers(self, copy_out: bool = False):
        """Converged PopulateFingerTable; returns the n x 128 table if copy_out."""
        if copy_out:
            F = np.empty((self.n, L.CX_FINGERS), dtype=np.uint32)
            L.check(L.lib().cx_fingers_build(self._h, _ptr(F), L.CX_MEM_HOST))
            return F
        L.check(L.lib().cx_fingers_build(self._h, None, L.CX_MEM_HOST))
        return None

    def upload_fingers(self, F):
        F = self._prep_u32(F, "fingers", self.n)
        assert tuple(F.shape) == (self.n, L.CX_FINGERS)
        mk = self._mem(F)
        L.check(L.lib().cx_fingers_upload(self._h, _ptr(F), mk))

    def upload_peer_state(self, min_keys=None, preds=None):
        mk_arr = None if min_keys is None else self._prep_keys(min_keys, "min_keys")
        pr = None if preds is None else self._prep_u32(preds, "preds", self.n)
        if mk_arr is not None and mk_arr.shape[0] != self.n:
            raise TypeError(f"min_keys: expected {self.n} values, got {mk_arr.shape[0]}")
        mk = self._mem(*(a for a in (mk_arr, pr) if a is not None)) if (mk_arr is not None or pr is not None) else L.CX_MEM_HOST
        L.check(L.lib().cx_peer_state_upload(self._h, _ptr(mk_arr), _ptr(pr), mk))

    def upload_liveness(self, alive=None, succs=None, ns: int = 0, rule: int = 0):
        """Peer liveness (n bytes, None = all alive) and successors_ lists
        ((n, ns) indices in list order, CX_NONE-padded; None = the converged
        next-ns window) for ForwardRequest's dead-finger branch; rule =
        CX_FWD_CHORD (chord_peer.cpp:201-208) or CX_FWD_DHASH
        (dhash_peer.cpp:516-526).  Switches route() to the literal walk.
        With alive=None and succs=None the ring is reset to the converged
        walk (no liveness state); ns and rule are then ignored."""
        al = None
        if alive is not None:
            al = alive.contiguous() if _is_dev(alive) else np.ascontiguousarray(alive, np.uint8)
            _check_dev(al, 1, "alive", self.device, self.n)
            if al.shape[0] != self.n:
                raise TypeError(f"alive: expected {self.n} entries")
        sl = None
        if succs is not None:
            sl = self._prep_u32(succs, "succs", self.n)
            ns = 1 if sl.ndim == 1 else int(sl.shape[1])
        arrs = [a for a in (al, sl) if a is not None]
        mk = self._mem(*arrs) if arrs else L.CX_MEM_HOST
        L.check(L.lib().cx_liveness_upload(self._h, _ptr(al), _ptr(sl), int(ns), int(rule), mk))

    def fingers_device(self):
        p = ctypes.c_void_p()
        L.check(L.lib().cx_fingers_device(self._h, ctypes.byref(p)))
        if not p.value:
            return None
        return _wrap_device(p.value, (self.n, L.CX_FINGERS), torch.int32, self.device, self)

    def set_route_variant(self, v: int):
        """Internal A/B switch: 0 = finger + ring gather per hop, 1 = route table,
        2/3 = packed table, 4 = lookahead tree, 5 = pattern-keyed window table,
        -1 = automatic (5 up to 2^24 peers, else 4)."""
        f = L.lib().cxi_set_route_variant
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.check(f(self._h, v))

    def route_info(self):
        """(variant in effect, variant-5 nodes not representable, route-table bytes)."""
        f = L.lib().cxi_route_info
        f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                      ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        v, e, b = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
        L.check(f(self._h, ctypes.byref(v), ctypes.byref(e), ctypes.byref(b)))
        return v.value, e.value, b.value

    def route_counters(self, enable: bool):
        """Internal: gather counters of the default route kernel.  enable=True
        zeroes them and makes later route() calls run the counting build of
        the walk; enable=False switches back and returns
        (64-B table gathers, exact 16-B ring gathers, exact hops, lookups)."""
        f = L.lib().cxi_route_counters
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
        out = np.zeros(4, dtype=np.uint64)
        L.check(f(self._h, int(bool(enable)), _ptr(out)))
        return None if enable else tuple(int(x) for x in out)

    def gather_probe(self, lanes: int = 1 << 19, hops: int = 64, span: int = 0) -> float:
        """Internal: dependent random 64-B gathers/s on this ring's own route
        table (the walk's access pattern without the walk); span > 0: over
        the table's first `span` bytes only (footprint A/B)."""
        if span:
            f = L.lib().cxi_gather_probe_span
            f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                          ctypes.POINTER(ctypes.c_double)]
            r = ctypes.c_double()
            L.check(f(self._h, lanes, hops, span, ctypes.byref(r)))
            return r.value
        f = L.lib().cxi_gather_probe
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                      ctypes.POINTER(ctypes.c_double)]
        r = ctypes.c_double()
        L.check(f(self._h, lanes, hops, ctypes.byref(r)))
        return r.value

    def route_table_hash(self, arc: bool = False) -> int:
        """Internal: order-sensitive 64-bit hash of the built pattern-keyed
        table (arc=True: this rank's arc planes), for A/B identity of builds."""
        f = L.lib().cxi_route_table_hash
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]
        h = ctypes.c_uint64()
        L.check(f(self._h, int(bool(arc)), ctypes.byref(h)))
        return h.value

    def set_table_build(self, v: int):
        """Internal A/B switch for the route-table build: 0 = level + two-hop
        planes, root-centric windows (default), 1 = the row-major finger
        table, 2 = level planes only, 3 = level + two-hop planes, one lane per
        entry (the round-2 build), 4 = root-centric in 256-row blocks (round
        3), 5 = alias of 0, 6 / 7 = as 0 on pair / quad planes, 8 = both
        windows of a root at once, 9 = as 0 with plane 0 stored after the W1
        gathers.  All build the same table."""
        f = L.lib().cxi_set_table_build
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.check(f(self._h, v))

    def set_route_depth(self, R: int):
        """Internal A/B switch: the route table covers levels [128 - R, 128)
        (0 = the default).  Before the first build_fingers only."""
        f = L.lib().cxi_set_route_depth
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.check(f(self._h, int(R)))

    def set_fingers_repair(self, on: bool):
        """Internal A/B switch (row f2): a ring churned from this one remaps its
        parent's finger level planes (True; the ring then keeps its planes for
        its children) or searches them from scratch (False, default: the
        streaming build is faster).  Inherited by churned rings."""
        f = L.lib().cxi_set_fingers_repair
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.check(f(self._h, int(bool(on))))

    def fingers_repair_info(self):
        """(repaired, searched) of the last finger build: whether its planes
        were remapped from the parent ring, and how many fingers the repair
        searched exactly (churn events at the finger, joined peers)."""
        f = L.lib().cxi_fingers_repair_info
        f.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                      ctypes.POINTER(ctypes.c_uint64)]
        r, n = ctypes.c_int(), ctypes.c_uint64()
        L.check(f(self._h, ctypes.byref(r), ctypes.byref(n)))
        return bool(r.value), n.value

    def set_churn_variant(self, v: int):
        """Internal A/B switch: 0 = full re-sort, 1 = merge of sorted joins (default)."""
        f = L.lib().cxi_set_churn_variant
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.check(f(self._h, v))

    def set_search_variant(self, v: int):
        """Internal A/B switch: 0 = Eytzinger (LDS top levels), 1 = bucket directory
        (default; successor / predecessor of >= 2^16 keys and >= 4 n on a ring
        whose slice table fits LDS take the LDS slice table), 2 = wave-cooperative
        16-ary tree (ballot/popcount), 3 = wave-cooperative Eytzinger (16 lanes a
        query, four levels per ballot), 4 = the LDS slice table whenever the ring
        fits (any batch), 5 = directory only; 2 to 5 serve successor and
        predecessor only, the other searches keep the directory."""
        f = L.lib().cxi_set_search_variant
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.check(f(self._h, v))

    def set_misplaced_variant(self, v: int):
        """Internal A/B switch for cx_misplaced on a ring from cx_churn: 0 = two
        searches + the old_to_new window per key, 1 = churn directory (default)."""
        f = L.lib().cxi_set_misplaced_variant
        f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.check(f(self._h, v))

    # ---- a7-a9 -----------------------------------------------------------
    def route(self, src, keys, out=None):
        """GetSuccessor(key) issued at peer src: (owner, hops, status)."""
        keys = self._prep_keys(keys)
        q = keys.shape[0]
        src = self._prep_u32(src, "src", q)
        if out is None:
            owner = self._empty(keys, (q,), np.uint32, torch and torch.int32)
            hops = self._empty(keys, (q,), np.uint8, torch and torch.uint8)
            status = self._empty(keys, (q,), np.uint8, torch and torch.uint8)
        else:
            owner, hops, status = out
        self._check_out([(owner, 4, "owner"), (hops, 1, "hops"), (status, 1, "status")], q)
        mk = self._mem(keys, src, owner, hops)
        L.check(L.lib().cx_route(self._h, _ptr(src), _ptr(keys), q, _ptr(owner), _ptr(hops),
                                 _ptr(status), mk))
        return owner, hops, status

    # ---- a10/a11 ---------------------------------------------------------
    def nsucc(self, keys, n: int, out=None):
        """GetNSuccessors(key, n) on the converged ring: (lists (q, n), count);
        out = (lists, count) to write caller buffers."""
        keys = self._prep_keys(keys)
        q = keys.shape[0]
        if out is None:
            lists = self._empty(keys, (q, n), np.uint32, torch and torch.int32)
            count = self._empty(keys, (q,), np.uint8, torch and torch.uint8)
        else:
            lists, count = out
            self._check_out([(lists, 4, "lists"), (count, 1, "count")], q)
            if tuple(lists.shape) != (q, n):
                raise TypeError(f"lists: expected shape ({q}, {n})")
        mk = self._mem(keys, lists)
        L.check(L.lib().cx_nsucc(self._h, _ptr(keys), q, n, _ptr(lists), _ptr(count), mk))
        return lists, count

    def dhash_check(self, n: int = 14, m: int = 10):
        L.check(L.lib().cx_dhash_check(self._h, n, m))

    # ---- a12 -------------------------------------------------------------
    def churn(self, joins, leaves):
        joins, leaves = self._prep_keys(joins), self._prep_keys(leaves)
        o2n = self._empty(joins, (self.n,), np.uint32, torch and torch.int32)
        mk = self._mem(joins, leaves, o2n)
        h = ctypes.c_void_p()
        L.check(L.lib().cx_churn(self._h, _ptr(joins), joins.shape[0], _ptr(leaves),
                                 leaves.shape[0], mk, ctypes.byref(h), _ptr(o2n)))
        return Ring(None, self.device, _handle=h), o2n

    def misplaced(self, new_ring: "Ring", old_to_new, keys, n: int):
        keys = self._prep_keys(keys)
        o2n = self._prep_u32(old_to_new, "old_to_new", self.n)
        q = keys.shape[0]
        lists = self._empty(keys, (q, n), np.uint32, torch and torch.int32)
        count = self._empty(keys, (q,), np.uint8, torch and torch.uint8)
        mask = self._empty(keys, (q,), np.uint16, torch and torch.int16)
        target = self._empty(keys, (q, n), np.uint8, torch and torch.uint8)
        mk = new_ring._mem(keys, o2n, lists)
        L.check(L.lib().cx_misplaced(self._h, new_ring._h, _ptr(o2n), _ptr(keys), q, n,
                                     _ptr(lists), _ptr(count), _ptr(mask), _ptr(target), mk))
        return lists, count, mask, target

    def dhash_maintenance(self, new_ring: "Ring", old_to_new, keys, n: int):
        """nsucc(keys, n) on this (old) ring + misplaced(new_ring, ...) in one
        pass (cx_dhash_maintenance): (old_lists, old_count, new_lists, count,
        mask, target), each equal to the separate calls' outputs."""
        keys = self._prep_keys(keys)
        o2n = self._prep_u32(old_to_new, "old_to_new", self.n)
        q = keys.shape[0]
        old_lists = self._empty(keys, (q, n), np.uint32, torch and torch.int32)
        old_count = self._empty(keys, (q,), np.uint8, torch and torch.uint8)
        lists = self._empty(keys, (q, n), np.uint32, torch and torch.int32)
        count = self._empty(keys, (q,), np.uint8, torch and torch.uint8)
        mask = self._empty(keys, (q,), np.uint16, torch and torch.int16)
        target = self._empty(keys, (q, n), np.uint8, torch and torch.uint8)
        mk = new_ring._mem(keys, o2n, lists)
        L.check(L.lib().cx_dhash_maintenance(self._h, new_ring._h, _ptr(o2n), _ptr(keys), q, n,
                                             _ptr(old_lists), _ptr(old_count), _ptr(lists),
                                             _ptr(count), _ptr(mask), _ptr(target), mk))
        return old_lists, old_count, lists, count, mask, target

    def misplaced_holders(self, keys, holders, n: int):
        keys = self._prep_keys(keys)
        holders = self._prep_u32(holders, "holders", keys.shape[0])
        if holders.ndim != 2:
            raise TypeError("holders: expected a (q, nh) array")
        q, nh = holders.shape
        lists = self._empty(keys, (q, n), np.uint32, torch and torch.int32)
        count = self._empty(keys, (q,), np.uint8, torch and torch.uint8)
        mask = self._empty(keys, (q,), np.uint16, torch and torch.int16)
        target = self._empty(keys, (q, nh), np.uint8, torch and torch.uint8)
        mk = self._mem(keys, holders, lists)
        L.check(L.lib().cx_misplaced_holders(self._h, _ptr(keys), q, _ptr(holders), nh, n,
                                             _ptr(lists), _ptr(count), _ptr(mask),
                                             _ptr(target), mk))
        return lists, count, mask, target

    # ---- arc-sharded routing (chordx.arc drives the exchange) -------------
    def arc_build(self, world: int, rank: int, top_levels: int = 0):
        """Rank `rank`'s route planes of a `world`-rank arc layout (cx_arc_build):
        replicated top levels, lower levels for its arc + halo."""
        L.check(L.lib().cx_arc_build(self._h, world, rank, top_levels))

    def arc_info(self):
        """(replicated top levels, local rows, route-plane bytes)."""
        t, r, b = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint64()
        L.check(L.lib().cx_arc_info(self._h, ctypes.byref(t), ctypes.byref(r), ctypes.byref(b)))
        return t.value, r.value, b.value

    def _arc_stream(self):
        self._torch_stream()

    def arc_seed(self, rank: int, src, keys):
        """(q, 4) int64 device tensor of NEW records (32 B each)."""
        keys = self._prep_keys(keys)
        src = self._prep_u32(src, "src", keys.shape[0])
        if not (_is_dev(keys) and _is_dev(src)):
            raise TypeError("arc routing takes device tensors")
        q = keys.shape[0]
        out = torch.empty((q, 4), dtype=torch.int64, device=keys.device)
        self._arc_stream()
        L.check(L.lib().cx_arc_seed(self._h, rank, _ptr(src), _ptr(keys), q, _ptr(out)))
        return out

    def arc_start(self, rank: int, src, keys, owner, hops, status=None):
        """arc_seed + the first arc_step in one pass (cx_arc_start): outcome
        records of this rank's new lookups."""
        keys = self._prep_keys(keys)
        src = self._prep_u32(src, "src", keys.shape[0])
        if not (_is_dev(keys) and _is_dev(src)):
            raise TypeError("arc routing takes device tensors")
        q = keys.shape[0]
        out = torch.empty((q, 4), dtype=torch.int64, device=keys.device)
        self._arc_stream()
        L.check(L.lib().cx_arc_start(self._h, rank, _ptr(src), _ptr(keys), q, _ptr(out),
                                     _ptr(owner), _ptr(hops), _ptr(status)))
        return out

    def arc_step(self, rank: int, recs, owner, hops, status=None):
        """One walk step over `recs`; returns the outcome records (same count)."""
        q = recs.shape[0]
        out = torch.empty_like(recs)
        self._arc_stream()
        L.check(L.lib().cx_arc_step(self._h, rank, _ptr(recs), q, _ptr(out), _ptr(owner),
                                    _ptr(hops), _ptr(status)))
        return out

    def arc_send_ahead(self, world: int, rank: int, src, keys):
        """(send, counts): this rank's new lookups as NEW records grouped by the
        rank of their key's arc (cx_arc_send_ahead; no origin walk)."""
        keys = self._prep_keys(keys)
        src = self._prep_u32(src, "src", keys.shape[0])
        if not (_is_dev(keys) and _is_dev(src)):
            raise TypeError("arc routing takes device tensors")
        q = keys.shape[0]
        send = torch.empty((q, 4), dtype=torch.int64, device=keys.device)
        counts = np.zeros(world, dtype=np.uint64)
        self._arc_stream()
        L.check(L.lib().cx_arc_send_ahead(self._h, world, rank, _ptr(src), _ptr(keys), q,
                                          _ptr(send), _ptr(counts)))
        return send[: int(counts.sum())], [int(c) for c in counts]

    def arc_partition(self, world: int, src, keys):
        """(send_keys, send_src, perm, counts): this rank's lookups grouped by
        the rank of their key's arc (cx_arc_partition).  send_keys / send_src
        are exchanged; perm (lookup index -> send slot) stays here."""
        keys = self._prep_keys(keys)
        src = self._prep_u32(src, "src", keys.shape[0])
        if not (_is_dev(keys) and _is_dev(src)):
            raise TypeError("arc routing takes device tensors")
        q = keys.shape[0]
        skeys = torch.empty((q, 2), dtype=torch.int64, device=keys.device)
        ssrc = torch.empty(q, dtype=torch.int32, device=keys.device)
        perm = torch.empty(q, dtype=torch.int32, device=keys.device)
        counts = np.zeros(world, dtype=np.uint64)
        self._arc_stream()
        L.check(L.lib().cx_arc_partition(self._h, world, _ptr(src), _ptr(keys), q, _ptr(skeys),
                                         _ptr(ssrc), _ptr(perm), _ptr(counts)))
        return skeys, ssrc, perm, [int(c) for c in counts]

    def arc_partition_regions(self, world: int, src, keys, cap: int, hints: bool = False):
        """Single-pass partition (cx_arc_partition_regions): (send_keys,
        send_src, perm, counts) with destination d's lookups at rows
        [d cap, d cap + counts[d]) of send_keys / send_src; None when some
        destination exceeds cap (the caller falls back to arc_partition).
        hints=True: (send_keys, send_src, perm, counts, send_hint), the
        origin-resolved source hints for arc_route(..., hint=)."""
        keys = self._prep_keys(keys)
        src = self._prep_u32(src, "src", keys.shape[0])
        if not (_is_dev(keys) and _is_dev(src)):
            raise TypeError("arc routing takes device tensors")
        q = keys.shape[0]
        skeys = torch.empty((world * cap, 2), dtype=torch.int64, device=keys.device)
        ssrc = torch.empty(world * cap, dtype=torch.int32, device=keys.device)
        perm = torch.empty(q, dtype=torch.int32, device=keys.device)
        shint = torch.empty(world * cap, dtype=torch.int64, device=keys.device) if hints else None
        counts = np.zeros(world, dtype=np.uint64)
        self._arc_stream()
        rc = L.lib().cx_arc_partition_regions(self._h, world, _ptr(src), _ptr(keys), q, cap,
                                              _ptr(skeys), _ptr(ssrc), _ptr(shint), _ptr(perm),
                                              _ptr(counts))
        if rc == L.CX_E_STATE and "region" in (L.lib().cx_last_error() or b"").decode():
            return None
        L.check(rc)
        out = (skeys, ssrc, perm, [int(c) for c in counts])
        return out + (shint,) if hints else out

    def arc_partition_regions_async(self, world: int, src, keys, cap: int, counts,
                                    hints: bool = False):
        """cx_arc_partition_regions_async: as arc_partition_regions, but the
        counts (and, at counts[world], the overflow flag) land in `counts`, a
        device int64 tensor of world + 1 elements, with no host
        synchronisation; (send_keys, send_src, perm[, send_hint])."""
        keys = self._prep_keys(keys)
        src = self._prep_u32(src, "src", keys.shape[0])
        if not (_is_dev(keys) and _is_dev(src) and _is_dev(counts)):
            raise TypeError("arc routing takes device tensors")
        if not (counts.dtype == torch.int64 and counts.is_contiguous()
                and counts.numel() == world + 1):
            raise TypeError("counts: a contiguous int64 device tensor of world + 1 elements")
        q = keys.shape[0]
        skeys = torch.empty((world * cap, 2), dtype=torch.int64, device=keys.device)
        ssrc = torch.empty(world * cap, dtype=torch.int32, device=keys.device)
        perm = torch.empty(q, dtype=torch.int32, device=keys.device)
        shint = torch.empty(world * cap, dtype=torch.int64, device=keys.device) if hints else None
        self._arc_stream()
        L.check(L.lib().cx_arc_partition_regions_async(self._h, world, _ptr(src), _ptr(keys), q,
                                                       cap, _ptr(skeys), _ptr(ssrc), _ptr(shint),
                                                       _ptr(perm), _ptr(counts)))
        return (skeys, ssrc, perm, shint) if hints else (skeys, ssrc, perm)

    @staticmethod
    def arc_own_ws_words(q: int) -> int:
        """int32 words of arc_count_async's own_ws scratch for q lookups (the
        own-run cursor: one word whatever q)."""
        return 1

    def arc_count_async(self, world: int, keys, counts, me: int = -1, own_idx=None,
                        own_ws=None):
        """cx_arc_count_async: per-destination counts of the keys' arcs into
        `counts` (device int64, world elements), no host synchronisation; with
        own_idx (device int32, >= q elements) and own_ws (device int32 scratch,
        >= arc_own_ws_words(q) elements): the indices of rank `me`'s own
        lookups in own_idx[:counts[me]] (a permutation of them, ascending
        within each block's run)."""
        keys = self._prep_keys(keys)
        if not (_is_dev(keys) and _is_dev(counts)):
            raise TypeError("arc routing takes device tensors")
        if not (counts.dtype == torch.int64 and counts.is_contiguous()
                and counts.numel() == world):
            raise TypeError("counts: a contiguous int64 device tensor of world elements")
        if own_idx is not None:
            if not (0 <= me < world):
                raise ValueError("me must be in [0, world)")
            for t, n_ in ((own_idx, keys.shape[0]), (own_ws, self.arc_own_ws_words(keys.shape[0]))):
                if t is None or not (_is_dev(t) and t.is_contiguous() and t.element_size() == 4
                                     and t.numel() >= n_):
                    raise TypeError("own_idx (>= q) / own_ws (>= arc_own_ws_words(q)): "
                                    "contiguous 4-byte device tensors")
        self._arc_stream()
        L.check(L.lib().cx_arc_count_async(self._h, world, _ptr(keys), keys.shape[0],
                                           _ptr(counts), int(me), _ptr(own_idx),
                                           _ptr(own_ws)))

    def arc_scatter_async(self, world: int, src, keys, counts, cursor, hints: bool = False,
                          skip: int = -1):
        """cx_arc_scatter_async: the exact-layout partition of (src, keys) by the
        device counts of arc_count_async over the same keys; cursor: device
        int32 scratch of world elements (one per concurrent scatter); skip: a
        destination left out (its lookups' perm = -1, its count taken as 0).
        Returns (send_keys, send_src, perm[, send_hint]), destination d's
        lookups at rows [sum(counts[:d]), sum(counts[:d + 1]))."""
        keys = self._prep_keys(keys)
        src = self._prep_u32(src, "src", keys.shape[0])
        for t, n, w in ((counts, world, 8), (cursor, world, 4)):
            if not (_is_dev(t) and t.is_contiguous() and t.numel() == n and t.element_size() == w):
                raise TypeError("counts (int64) / cursor (int32): contiguous device tensors of "
                                "world elements")
        if not (_is_dev(keys) and _is_dev(src)):
            raise TypeError("arc routing takes device tensors")
        if not -1 <= skip < world:
            raise ValueError("skip must be -1 or a rank")
        q = keys.shape[0]
        skeys = torch.empty((q, 2), dtype=torch.int64, device=keys.device)
        ssrc = torch.empty(q, dtype=torch.int32, device=keys.device)
        perm = torch.empty(q, dtype=torch.int32, device=keys.device)
        shint = torch.empty(q, dtype=torch.int64, device=keys.device) if hints else None
        self._arc_stream()
        L.check(L.lib().cx_arc_scatter_async(self._h, world, _ptr(src), _ptr(keys), q,
                                             _ptr(counts), _ptr(cursor), _ptr(skeys), _ptr(ssrc),
                                             _ptr(shint), _ptr(perm), int(skip)))
        return (skeys, ssrc, perm, shint) if hints else (skeys, ssrc, perm)

    def arc_route_local(self, src, keys, idx, owner, hops, status=None):
        """cx_arc_route_local: the lookups keys[idx[j]] from src[idx[j]] of this
        rank's own arc walked in place; owner / hops / status written at
        idx[j] (status may be None)."""
        keys = self._prep_keys(keys)
        src = self._prep_u32(src, "src", keys.shape[0])
        if not (_is_dev(keys) and _is_dev(src) and _is_dev(idx)):
            raise TypeError("arc routing takes device tensors")
        if not (idx.is_contiguous() and idx.element_size() == 4):
            raise TypeError("idx: a contiguous 4-byte device tensor")
        q0 = keys.shape[0]
        for t, w, name in ((owner, 4, "owner"), (hops, 1, "hops"), (status, 1, "status")):
            if t is not None and not (_is_dev(t) and t.element_size() == w and t.numel() >= q0
                                      and t.is_contiguous()):
                raise TypeError(f"{name}: contiguous device tensor of {w}-byte elements, >= "
                                "len(keys)")
        self._arc_stream()
        L.check(L.lib().cx_arc_route_local(self._h, _ptr(src), _ptr(keys), _ptr(idx), idx.numel(),
                                           _ptr(owner), _ptr(hops), _ptr(status)))

    def arc_route(self, src, keys, res=None, hint=None):
        """Packed results (int64: owner | hops << 32 | status << 40 | 1 << 63)
        of lookups received from every rank, in input order (cx_arc_route;
        with the origins' source hints: cx_arc_route_hinted)."""
        keys = self._prep_keys(keys)
        src = self._prep_u32(src, "src", keys.shape[0])
        if not (_is_dev(keys) and _is_dev(src)):
            raise TypeError("arc routing takes device tensors")
        q = keys.shape[0]
        if res is None:
            res = torch.empty(q, dtype=torch.int64, device=keys.device)
        elif not (_is_dev(res) and res.element_size() == 8 and res.numel() == q
                  and res.is_contiguous()):
            raise TypeError("res must be a contiguous 8-byte device tensor of q elements")
        if hint is not None:
            if not (_is_dev(hint) and hint.element_size() == 8 and hint.is_contiguous()
                    and hint.numel() == q):
                raise TypeError("hint must be a contiguous 8-byte device tensor of q elements")
            self._arc_stream()
            L.check(L.lib().cx_arc_route_hinted(self._h, _ptr(src), _ptr(keys), _ptr(hint), q,
                                                _ptr(res)))
            return res
        self._arc_stream()
        L.check(L.lib().cx_arc_route(self._h, _ptr(src), _ptr(keys), q, _ptr(res)))
        return res

    def arc_deliver(self, res, perm, owner, hops, status=None):
        """owner/hops/status of lookup i from the returned results (send
        order, or the region layout of arc_partition_regions) at perm[i]
        (None: identity) (cx_arc_deliver).  perm's entries must index res
        (they do when perm comes from the partition that laid res out)."""
        if not (_is_dev(res) and res.element_size() == 8 and res.is_contiguous()):
            raise TypeError("res must be a contiguous 8-byte device tensor")
        q = res.shape[0] if perm is None else perm.numel()
        if perm is not None and not (_is_dev(perm) and perm.element_size() == 4
                                     and perm.is_contiguous() and perm.numel() <= res.numel()):
            raise TypeError("perm must be a contiguous 4-byte device tensor, no longer than res")
        for t, w, name in ((owner, 4, "owner"), (hops, 1, "hops"), (status, 1, "status")):
            if t is not None and not (_is_dev(t) and t.element_size() == w and t.numel() >= q):
                raise TypeError(f"{name}: device tensor of {w}-byte elements, >= q")
        self._arc_stream()
        L.check(L.lib().cx_arc_deliver(self._h, _ptr(res), _ptr(perm) if perm is not None
                                       else None, q, _ptr(owner), _ptr(hops), _ptr(status)))

    def arc_local_ring(self, lo: int, hi: int) -> "Ring":
        """Peers [lo, hi) of this ring as a ring of their own (the arc a rank
        holds in the arc layout's exact-successor mode); its successor()
        answers indices relative to lo."""
        if not 0 <= lo < hi <= self.n:
            raise ValueError("arc must be a non-empty range of peers")
        return Ring(self.ids_device()[lo:hi].contiguous(), device=self.device)

    def arc_bucket(self, world: int, recs):
        """(send, counts): records grouped by destination rank, NONE dropped."""
        q = recs.shape[0]
        send = torch.empty_like(recs)
        counts = np.zeros(world, dtype=np.uint64)
        self._arc_stream()
        L.check(L.lib().cx_arc_bucket(self._h, world, _ptr(recs), q, _ptr(send), _ptr(counts)))
        return send[: int(counts.sum())], [int(c) for c in counts]


def in_between(v, lb, ub, inclusive: bool = True) -> np.ndarray:
    """Batched ChordKey::InBetween on raw uint256 operands ((q, 4) uint64 each)."""
    v, lb, ub = (np.ascontiguousarray(np.asarray(a, dtype=np.uint64).reshape(-1, 4))
                 for a in (v, lb, ub))
    out = np.empty(len(v), dtype=np.uint8)
    L.check(L.lib().cx_in_between(_ptr(v), _ptr(lb), _ptr(ub), len(v), int(inclusive),
                                  _ptr(out), L.CX_MEM_HOST))
    return out


def uuid5_dns(names, device: int = 0) -> np.ndarray:
    """IDs of plaintext names (peer "ip:port" strings or keys), hashed on the GPU:
    (q, 2) uint64 [lo, hi] = UUIDv5(DNS, name) big-endian (key.h:29-33,76-79)."""
    enc = [n.encode() if isinstance(n, str) else bytes(n) for n in names]
    offs = np.zeros(len(enc) + 1, dtype=np.uint64)
    if enc:
        offs[1:] = np.cumsum([len(b) for b in enc])
    buf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
    out = np.empty((len(enc), 2), dtype=np.uint64)
    L.check(L.lib().cx_uuid5_dns(_ptr(buf), _ptr(offs), len(enc), _ptr(out), L.CX_MEM_HOST,
                                 device))
    return out


def sort_time(ids, variant: int = 0):
    """Internal A/B: (ms, sorted) of cx_ring_create's (ID, index) sort over the
    device IDs `ids` ((n, 2) int64), variant 0 = the default (MSD buckets +
    LDS bucket sort), 1 = the 16-pass LSD sort (cxi_sort_time)."""
    assert _is_dev(ids) and ids.dim() == 2 and ids.shape[1] == 2
    ids = ids.contiguous()
    f = L.lib().cxi_sort_time
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
    torch.cuda.current_stream(ids.device).synchronize()
    ms, ok = ctypes.c_double(), ctypes.c_int()
    L.check(f(_ptr(ids), ids.shape[0], ids.device.index or 0, int(variant), ctypes.byref(ms),
              ctypes.byref(ok)))
    return ms.value, bool(ok.value)


def fill_splitmix(out, seed: int, offset: int = 0):
    """Synthetic uniform 128-bit keys written on the device into `out` ((q, 2) int64)."""
    assert _is_dev(out) and out.dim() == 2 and out.shape[1] == 2
    L.check(L.lib().cx_fill_splitmix(_ptr(out), out.shape[0], seed, offset,
                                     out.device.index or 0,
                                     ctypes.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)))
    return out


class _DevArray:
    """__cuda_array_interface__ shim so torch can view engine-owned memory."""

    def __init__(self, ptr, shape, typestr, owner):
        self._owner = owner
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr,
                                         "data": (ptr, False), "version": 2, "strides": None}


def _wrap_device(ptr, shape, dtype, device, owner):
    typestr = {torch.int64: "<i8", torch.int32: "<i4"}[dtype]
    with torch.cuda.device(device):
        return torch.as_tensor(_DevArray(ptr, shape, typestr, owner), device=f"cuda:{device}")
