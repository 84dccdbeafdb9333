"""Rabin IDA on the GPU: DHash's payload coding (src/ida/ida.cpp, data_block.cpp).

encode / decode are batched over ragged blocks (cx_ida_encode / cx_ida_decode);
DataBlock mirrors the reference class of the same name: a value is split into
n fragments (indices 1..n, data_block.cpp:12-13) of which any m rebuild it
(DHashPeer::Read decodes from the m lowest indices it collected,
dhash_peer.cpp:163-197 via std::set ordering).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def _is_dev(x) -> bool:
    return torch is not None and isinstance(x, torch.Tensor) and x.is_cuda


def _ptr(a):
    if a is None:
        return None
    if _is_dev(a):
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


def _need(t, esize: int, name: str, numel: int, dev):
    """Device-tensor argument check: element size, contiguity, size, device
    (the kernels read and write these through raw pointers)."""
    if not _is_dev(t):
        raise TypeError(f"{name}: expected a device tensor like the others")
    if t.element_size() != esize:
        raise TypeError(f"{name}: expected {esize}-byte elements, got {t.dtype}")
    if not t.is_contiguous():
        raise TypeError(f"{name}: must be contiguous")
    if t.numel() < numel:
        raise TypeError(f"{name}: needs {numel} elements, has {t.numel()}")
    if t.device != dev:
        raise TypeError(f"{name}: on {t.device}, expected {dev}")


def segments(lengths, m: int) -> np.ndarray:
    """seg_offsets (blocks + 1,) uint64: prefix sums of ceil(len / m)."""
    offs = np.zeros(len(lengths) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(np.asarray(lengths, dtype=np.uint64))
    seg = np.zeros_like(offs)
    L.check(L.lib().cx_ida_segments(_ptr(offs), len(lengths), m, _ptr(seg)))
    return seg


def _on_default_stream(t):
    """The IDA entry points run on the device's null stream: when the caller
    works on another (non-blocking) torch stream, its pending writes to the
    inputs are waited for before the call (and _after_call orders the
    outputs back), so no kernel reads a buffer another stream is filling."""
    cur = torch.cuda.current_stream(t.device)
    if cur.cuda_stream != 0:
        cur.synchronize()
        return False
    return True


def _after_call(t, was_default):
    if not was_default:
        torch.cuda.synchronize(t.device)


def encode_flat(data, offsets, n=14, m=10, p=257, device: int = 0, seg_offsets=None, out=None):
    """Raw batched encode.  data: uint8 bytes, offsets: (blocks + 1,) uint64
    (numpy, or torch device tensors).  Returns (frags uint16, seg_offsets);
    pass seg_offsets (same memory kind) to skip computing them."""
    blocks = offsets.shape[0] - 1
    if _is_dev(data):
        _need(data, 1, "data", 0, data.device)
        _need(offsets, 8, "offsets", blocks + 1, data.device)
    if seg_offsets is None:
        off_h = offsets.cpu().numpy() if _is_dev(offsets) else np.asarray(offsets, np.uint64)
        seg = np.zeros(blocks + 1, dtype=np.uint64)
        L.check(L.lib().cx_ida_segments(_ptr(np.ascontiguousarray(off_h)), blocks, m,
                                        _ptr(seg)))
        seg_offsets = torch.from_numpy(seg.astype(np.int64)).to(offsets.device) \
            if _is_dev(offsets) else seg
    if _is_dev(data):
        total = int(seg_offsets[-1])
        _need(seg_offsets, 8, "seg_offsets", blocks + 1, data.device)
        frags = out if out is not None else torch.empty(
            max(total * n, 1), dtype=torch.int16, device=data.device)
        _need(frags, 2, "out", total * n, data.device)
        mk = L.CX_MEM_DEVICE
        dflt = _on_default_stream(data)
    else:
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        frags = np.zeros(max(int(seg_offsets[-1]) * n, 1), dtype=np.uint16)
        mk = L.CX_MEM_HOST
    L.check(L.lib().cx_ida_encode(_ptr(data), _ptr(offsets), _ptr(seg_offsets), blocks, n, m,
                                  p, _ptr(frags), mk, device))
    if mk == L.CX_MEM_DEVICE:
        _after_call(data, dflt)
    return frags, seg_offsets


def decode_flat(frags, seg_offsets, indices, m=10, p=257, device: int = 0, total=None,
                out=None):
    """Raw batched decode; returns (values uint16, out_len uint64).  With
    device tensors, pass total (= seg_offsets[-1]) to avoid reading it back."""
    blocks = seg_offsets.shape[0] - 1
    if _is_dev(frags):
        dev = frags.device
        total = int(seg_offsets[-1].item()) if total is None else int(total)
        _need(frags, 2, "frags", total * m, dev)
        _need(seg_offsets, 8, "seg_offsets", blocks + 1, dev)
        _need(indices, 1, "indices", blocks * m, dev)
        if out is None:
            out = (torch.empty(max(total * m, 1), dtype=torch.int16, device=dev),
                   torch.empty(max(blocks, 1), dtype=torch.int64, device=dev))
        out, ln = out
        _need(out, 2, "out", total * m, dev)
        _need(ln, 8, "out_len", blocks, dev)
        mk = L.CX_MEM_DEVICE
        dflt = _on_default_stream(frags)
    else:
        frags = np.ascontiguousarray(frags, dtype=np.uint16)
        seg_offsets = np.ascontiguousarray(seg_offsets, dtype=np.uint64)
        indices = np.ascontiguousarray(indices, dtype=np.uint8)
        out = np.zeros(max(int(seg_offsets[-1]) * m, 1), dtype=np.uint16)
        ln = np.zeros(max(blocks, 1), dtype=np.uint64)
        mk = L.CX_MEM_HOST
    L.check(L.lib().cx_ida_decode(_ptr(frags), _ptr(seg_offsets), _ptr(indices), blocks, m, p,
                                  _ptr(out), _ptr(ln), mk, device))
    if mk == L.CX_MEM_DEVICE:
        _after_call(frags, dflt)
    return out, ln


def encode(blocks, n=14, m=10, p=257, device: int = 0):
    """List of (n, S_b) uint16 fragment matrices, one per datum (bytes)."""
    blocks = [bytes(b) for b in blocks]
    offs = np.zeros(len(blocks) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(b) for b in blocks], dtype=np.uint64)
    data = np.frombuffer(b"".join(blocks) + b"\0", dtype=np.uint8)
    frags, seg = encode_flat(data, offs, n, m, p, device)
    return [frags[n * int(seg[b]): n * int(seg[b + 1])].reshape(n, -1).copy()
            for b in range(len(blocks))]


def decode(frag_rows, indices, m=10, p=257, device: int = 0):
    """Values (uint16 arrays) decoded from m fragment rows per block with their
    1-based indices; None for a block whose indices have no inverse."""
    S = [np.asarray(f).shape[1] for f in frag_rows]
    seg = np.zeros(len(S) + 1, dtype=np.uint64)
    seg[1:] = np.cumsum(S, dtype=np.uint64)
    flat = np.concatenate([np.asarray(f, dtype=np.uint16).reshape(-1) for f in frag_rows] +
                          [np.zeros(1, np.uint16)])
    idx = np.asarray(indices, dtype=np.uint8).reshape(len(frag_rows), m)
    out, ln = decode_flat(flat, seg, idx, m, p, device)
    res = []
    for b in range(len(frag_rows)):
        if int(ln[b]) == 0xFFFFFFFFFFFFFFFF:
            res.append(None)
        else:
            res.append(out[m * int(seg[b]): m * int(seg[b]) + int(ln[b])].copy())
    return res


class DataBlock:
    """DataBlock (data_block.cpp:4-97): a value and its n IDA fragments."""

    def __init__(self, value, n=14, m=10, p=257, device: int = 0):
        self.n, self.m, self.p, self.device = n, m, p, device
        raw = value.encode() if isinstance(value, str) else bytes(value)
        f = encode([raw], n, m, p, device)[0]
        self.fragments = [(i + 1, f[i]) for i in range(n)]  # (INDEX, FRAGMENT)
        self.original = np.frombuffer(raw, dtype=np.uint8).astype(np.uint16)

    @classmethod
    def from_fragments(cls, fragments, n=14, m=10, p=257, device: int = 0):
        """DataBlock(vector<DataFragment>) (data_block.cpp:30-54): decode from
        the first m fragments given, then re-encode all n."""
        if len(fragments) < m:
            raise L.ChordError(L.CX_E_INSUFFICIENT, f"{m} frags are required to decode.")
        first = fragments[:m]
        vals = decode([np.stack([np.asarray(v, np.uint16) for _, v in first])],
                      [[i for i, _ in first]], m, p, device)[0]
        if vals is None:
            raise L.ChordError(L.CX_E_INVALID, "N is not invertible")
        self = cls.__new__(cls)
        self.n, self.m, self.p, self.device = n, m, p, device
        self.original = vals
        if vals.max(initial=0) >= 256:
            # the reference re-encodes its int values (data_block.cpp:52-53);
            # the GPU encoder takes bytes, and a value of 256 or more (only
            # from fragments that were not encoded from bytes) has no byte
            # form: refuse rather than return a wrong or empty fragment list
            raise L.ChordError(L.CX_E_INVALID,
                               "decoded value >= 256: cannot re-encode from bytes")
        f = encode([bytes(vals.astype(np.uint8))], n, m, p, device)[0]
        self.fragments = [(i + 1, f[i]) for i in range(n)]
        return self

    def decode(self) -> str:
        """DataBlock::Decode (data_block.cpp:81-97): chars, trailing NULs dropped."""
        s = "".join(chr(int(c) & 0xFF) for c in self.original)
        return s.rstrip("\0")
