"""Wire bridge: the reference's GET_SUCC request objects answered by the engine.

Wire(["127.0.0.1:5000", ...]) builds the ring of those peers (IDs = UUIDv5 of
the names, abstract_chord_peer.cpp:21) with its converged finger table;
Wire.handle(request) takes the JSON object a peer's server receives
({"COMMAND":"GET_SUCC","KEY":hex} or the batched GET_SUCC_BATCH) and returns
the JSON reply (RemotePeer fields ID / MIN_KEY / IP_ADDR / PORT + SUCCESS,
remote_peer.cpp:83-91; failures as server.h:156-165).  Parsing, dispatch and
reply assembly are C++ (csrc/cx_wire.cpp); key parsing and hex formatting run
on the GPU.  Also exposes the batched hex codec (cx_hex_parse / cx_hex_format).
"""
from __future__ import annotations

import ctypes
import json

import numpy as np

from . import _lib as L


class Wire:
    def __init__(self, addrs, device: int = 0):
        names = [a.encode() for a in addrs]
        arr = (ctypes.c_char_p * len(names))(*names)
        h = ctypes.c_void_p()
        L.check(L.lib().cx_wire_create(arr, len(names), device, ctypes.byref(h)))
        self._h = h

    def close(self):
        if self._h:
            L.lib().cx_wire_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def handle_raw(self, request: bytes) -> bytes:
        out = ctypes.c_void_p()
        n = ctypes.c_size_t()
        L.check(L.lib().cx_wire_handle(self._h, request, len(request), ctypes.byref(out),
                                       ctypes.byref(n)))
        try:
            return ctypes.string_at(out, n.value)
        finally:
            L.lib().cx_wire_free(out)

    def handle(self, request) -> dict:
        raw = request if isinstance(request, (bytes, str)) else json.dumps(request)
        if isinstance(raw, str):
            raw = raw.encode()
        return json.loads(self.handle_raw(raw))


def hex_parse(strings, device: int = 0):
    """(values (q, 2) uint64 lo/hi, ok (q,) uint8) of hex key strings."""
    enc = [s.encode() if isinstance(s, str) else bytes(s) for s in strings]
    offs = np.zeros(len(enc) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(e) for e in enc])
    buf = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
    out = np.zeros((len(enc), 2), dtype=np.uint64)
    ok = np.zeros(len(enc), dtype=np.uint8)
    L.check(L.lib().cx_hex_parse(buf.ctypes.data_as(ctypes.c_void_p),
                                 offs.ctypes.data_as(ctypes.c_void_p), len(enc),
                                 out.ctypes.data_as(ctypes.c_void_p),
                                 ok.ctypes.data_as(ctypes.c_void_p), L.CX_MEM_HOST, device))
    return out, ok


def hex_format(keys, device: int = 0) -> list:
    """std::string(key) of each (lo, hi) key: lowercase hex, no leading zeros."""
    k = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64).reshape(-1, 2))
    txt = np.zeros((k.shape[0], 32), dtype=np.uint8)
    ln = np.zeros(k.shape[0], dtype=np.uint8)
    L.check(L.lib().cx_hex_format(k.ctypes.data_as(ctypes.c_void_p), k.shape[0],
                                  txt.ctypes.data_as(ctypes.c_void_p),
                                  ln.ctypes.data_as(ctypes.c_void_p), L.CX_MEM_HOST, device))
    return [bytes(txt[i, :ln[i]]).decode() for i in range(k.shape[0])]
