"""chordx -- MI355X batched Chord/DHash lookup engine (Python face of libchordx).

The engine is a C-ABI shared library (include/chordx.h) over hand-written
gfx950 HIP kernels (p2p-dhts_amd/csrc/).  This package binds it with ctypes and
mirrors the reference's lookup-path interface (see ring.py).
"""
from ._lib import (CX_FINGERS, CX_FWD_CHORD, CX_FWD_DHASH, CX_HOP_CAP, CX_MAX_NSUCC, CX_NONE,
                   CX_Q_BADPEER, CX_Q_FAILED, CX_Q_HOPCAP, CX_Q_NOT_FOUND, CX_Q_OK, ChordError,
                   device_count, lib, pool_info, pool_stats, pool_stats_delta, pool_trim)
from .key import ChordKey
from .ring import Ring, fill_splitmix, in_between, uuid5_dns
from .wire import Wire, hex_format, hex_parse
from . import ida

__all__ = [
    "Ring", "ChordKey", "ChordError", "in_between", "fill_splitmix", "uuid5_dns", "device_count",
    "pool_trim", "pool_info", "pool_stats", "pool_stats_delta", "Wire", "hex_parse", "hex_format",
    "lib",
    "CX_FINGERS", "CX_NONE", "CX_HOP_CAP", "CX_MAX_NSUCC", "CX_Q_OK", "CX_Q_HOPCAP",
    "CX_Q_BADPEER", "CX_Q_FAILED", "CX_Q_NOT_FOUND", "CX_FWD_CHORD", "CX_FWD_DHASH",
]
