"""ctypes binding of libchordx.so (include/chordx.h).

The shared library is built in-tree by `make -C p2p-dhts_amd/csrc` (or
__graft_entry__.build()).  Loading it needs no GPU; every compute entry point
fails with CX_E_HIP when no HIP device is visible -- there is no host fallback.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# CHORDX_LIB: an alternative build of the same library (A/B kernel experiments).
LIB_PATH = os.environ.get("CHORDX_LIB") or os.path.join(HERE, "libchordx.so")

CX_OK = 0
CX_E_INVALID = 1
CX_E_NOT_FOUND = 2
CX_E_LOOKUP_FAILED = 3
CX_E_INSUFFICIENT = 4
CX_E_HIP = 5
CX_E_RCCL = 6
CX_E_NOMEM = 7
CX_E_STATE = 8

CX_MEM_HOST = 0
CX_MEM_DEVICE = 1

CX_FINGERS = 128
CX_NONE = 0xFFFFFFFF
CX_HOP_CAP = 255
CX_MAX_NSUCC = 16
CX_Q_OK, CX_Q_HOPCAP, CX_Q_BADPEER, CX_Q_FAILED, CX_Q_NOT_FOUND = 0, 1, 2, 3, 4
CX_FWD_CHORD, CX_FWD_DHASH = 0, 1

# Every symbol include/chordx.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "cx_version", "cx_last_error", "cx_device_count", "cx_pool_trim", "cx_pool_info",
    "cx_ring_create", "cx_ring_destroy", "cx_ring_size", "cx_ring_ids",
    "cx_ring_ids_device", "cx_ring_set_stream", "cx_ring_use_own_stream", "cx_ring_sync",
    "cx_successor", "cx_predecessor", "cx_fingers_build", "cx_fingers_upload", "cx_fingers_device",
    "cx_peer_state_upload", "cx_liveness_upload", "cx_route", "cx_nsucc", "cx_dhash_check",
    "cx_churn", "cx_misplaced", "cx_dhash_maintenance", "cx_misplaced_holders", "cx_in_between",
    "cx_uuid5_dns", "cx_fill_splitmix",
    "cx_arc_build", "cx_arc_info", "cx_arc_seed", "cx_arc_start", "cx_arc_step",
    "cx_arc_bucket", "cx_arc_send_ahead",
    "cx_arc_partition", "cx_arc_partition_regions", "cx_arc_partition_regions_async",
    "cx_arc_count_async", "cx_arc_scatter_async", "cx_arc_route_local",
    "cx_arc_route", "cx_arc_route_hinted",
    "cx_arc_deliver",
    "cx_hex_parse", "cx_hex_format",
    "cx_ida_segments", "cx_ida_encode", "cx_ida_decode",
    "cx_wire_create", "cx_wire_destroy", "cx_wire_ring", "cx_wire_handle", "cx_wire_free",
)

CX_ARC_NEW, CX_ARC_RESULT, CX_ARC_WALK, CX_ARC_NONE = 0, 1, 2, 3
CX_ARC_MAX_RANKS = 64
CX_ARC_TOP_LEVELS = 6


class ChordError(RuntimeError):
    """A CX_E_* failure; .code is the cx_err value."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ChordError(CX_E_HIP, f"{LIB_PATH} is missing: build it with "
                                   "`make -C p2p-dhts_amd/csrc` (no host fallback exists)")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    pp = ctypes.POINTER(ctypes.c_void_p)
    sig = {
        "cx_version": ([], i),
        "cx_last_error": ([], ctypes.c_char_p),
        "cx_device_count": ([ctypes.POINTER(ctypes.c_int)], i),
        "cx_pool_trim": ([], i),
        "cx_pool_info": ([ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)], i),
        "cx_ring_create": ([vp, sz, i, i, pp], i),
        "cx_ring_destroy": ([vp], i),
        "cx_ring_size": ([vp, ctypes.POINTER(ctypes.c_size_t)], i),
        "cx_ring_ids": ([vp, vp, i], i),
        "cx_ring_ids_device": ([vp, pp], i),
        "cx_ring_set_stream": ([vp, vp], i),
        "cx_ring_use_own_stream": ([vp], i),
        "cx_ring_sync": ([vp], i),
        "cx_successor": ([vp, vp, sz, vp, i], i),
        "cx_predecessor": ([vp, vp, sz, vp, i], i),
        "cx_fingers_build": ([vp, vp, i], i),
        "cx_fingers_upload": ([vp, vp, i], i),
        "cx_fingers_device": ([vp, pp], i),
        "cx_peer_state_upload": ([vp, vp, vp, i], i),
        "cx_liveness_upload": ([vp, vp, vp, i, i, i], i),
        "cx_route": ([vp, vp, vp, sz, vp, vp, vp, i], i),
        "cx_nsucc": ([vp, vp, sz, i, vp, vp, i], i),
        "cx_dhash_check": ([vp, i, i], i),
        "cx_churn": ([vp, vp, sz, vp, sz, i, pp, vp], i),
        "cx_misplaced": ([vp, vp, vp, vp, sz, i, vp, vp, vp, vp, i], i),
        "cx_dhash_maintenance": ([vp, vp, vp, vp, sz, i, vp, vp, vp, vp, vp, vp, i], i),
        "cx_misplaced_holders": ([vp, vp, sz, vp, i, i, vp, vp, vp, vp, i], i),
        "cx_in_between": ([vp, vp, vp, sz, i, vp, i], i),
        "cx_uuid5_dns": ([vp, vp, sz, vp, i, i], i),
        "cx_fill_splitmix": ([vp, sz, u64, u64, i, vp], i),
        "cx_ida_segments": ([vp, sz, i, vp], i),
        "cx_ida_encode": ([vp, vp, vp, sz, i, i, i, vp, i, i], i),
        "cx_ida_decode": ([vp, vp, vp, sz, i, i, vp, vp, i, i], i),
        "cx_hex_parse": ([vp, vp, sz, vp, vp, i, i], i),
        "cx_hex_format": ([vp, sz, vp, vp, i, i], i),
        "cx_wire_create": ([ctypes.POINTER(ctypes.c_char_p), sz, i, pp], i),
        "cx_wire_destroy": ([vp], i),
        "cx_wire_ring": ([vp, pp], i),
        "cx_wire_handle": ([vp, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_void_p),
                            ctypes.POINTER(ctypes.c_size_t)], i),
        "cx_wire_free": ([vp], None),
        "cx_arc_build": ([vp, i, i, i], i),
        "cx_arc_info": ([vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint64),
                         ctypes.POINTER(ctypes.c_uint64)], i),
        "cx_arc_seed": ([vp, i, vp, vp, sz, vp], i),
        "cx_arc_step": ([vp, i, vp, sz, vp, vp, vp, vp], i),
        "cx_arc_start": ([vp, i, vp, vp, sz, vp, vp, vp, vp], i),
        "cx_arc_bucket": ([vp, i, vp, sz, vp, vp], i),
        "cx_arc_send_ahead": ([vp, i, i, vp, vp, sz, vp, vp], i),
        "cx_arc_partition": ([vp, i, vp, vp, sz, vp, vp, vp, vp], i),
        "cx_arc_partition_regions": ([vp, i, vp, vp, sz, u64, vp, vp, vp, vp, vp], i),
        "cx_arc_partition_regions_async": ([vp, i, vp, vp, sz, u64, vp, vp, vp, vp, vp], i),
        "cx_arc_count_async": ([vp, i, vp, sz, vp, i, vp, vp], i),
        "cx_arc_scatter_async": ([vp, i, vp, vp, sz, vp, vp, vp, vp, vp, vp, i], i),
        "cx_arc_route_local": ([vp, vp, vp, vp, sz, vp, vp, vp], i),
        "cx_arc_route_hinted": ([vp, vp, vp, vp, sz, vp], i),
        "cx_arc_route": ([vp, vp, vp, sz, vp], i),
        "cx_arc_deliver": ([vp, vp, vp, sz, vp, vp, vp], i),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != CX_OK:
        msg = lib().cx_last_error()
        raise ChordError(rc, msg.decode() if msg else f"chordx error {rc}")


def pool_trim() -> None:
    """Release the table pool's idle HBM blocks (cx_pool_trim)."""
    check(lib().cx_pool_trim())


def pool_info():
    """(idle blocks, idle bytes) held by the table pool (cx_pool_info)."""
    b, n = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().cx_pool_info(ctypes.byref(b), ctypes.byref(n)))
    return b.value, n.value


POOL_STAT_KEYS = ("fresh_bytes", "fresh_allocs", "reused_bytes", "reused_allocs", "trims",
                  "trimmed_bytes", "retries", "failures")


def pool_stats() -> dict:
    """Internal: allocation-path counters since the process started
    (cxi_pool_stats): bytes / allocations fresh from hipMalloc, handed back by
    the table pool, idle blocks trimmed to retry a failed allocation, retries
    and failures.  Differences of two snapshots give one epoch's path."""
    import numpy as np
    out = np.zeros(8, dtype=np.uint64)
    f = lib().cxi_pool_stats
    f.argtypes = [ctypes.c_void_p]
    check(f(out.ctypes.data_as(ctypes.c_void_p)))
    return {k: int(v) for k, v in zip(POOL_STAT_KEYS, out)}


def pool_stats_delta(before: dict, after: dict) -> dict:
    return {k: after[k] - before[k] for k in POOL_STAT_KEYS}


def set_fault(mask: int) -> None:
    """Internal, tests only: fault injection (cxi_set_fault; bit 0 = the
    route-table build's finger-plane allocation fails)."""
    f = lib().cxi_set_fault
    f.argtypes = [ctypes.c_int]
    check(f(int(mask)))


def device_count() -> int:
    c = ctypes.c_int(0)
    check(lib().cx_device_count(ctypes.byref(c)))
    return c.value
