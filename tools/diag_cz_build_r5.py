"""Diagnostic (round 6): the one-lane-per-entry route-table
build outside the engine (tests/hip/libcxtest.so cxt_cz_build: k_cz_build's
chained path, row-major (mode 0) or level-plane (mode 1) fingers, round-5 or
current encode), on the all-escape cluster ring and a uniform ring, each
variant built three times.  Prints per build the words that are not CZ_NONE and
a hash of the table."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + "/oracle"]
import oracle as O  # noqa: E402

LIBN = sys.argv[1] if len(sys.argv) > 1 else "libcxtest.so"  # or libcxtest_nop.so / _wz.so
T = ctypes.CDLL(os.path.join(R, "tests", "hip", LIBN))
vp, u32, i = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int
T.cxt_cz_build.argtypes = [i, i, vp, vp, u32, i, i, i, vp, vp]


def p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


for kind in ("cluster", "uniform"):
    if kind == "cluster":
        base = 0x3C3C_5A5A_0F0F_1234 << 64
        ids = O.keys_from_ints([base + k * 7919 for k in range(6000)])
    else:
        ids = O.splitmix_keys(0xE17C1, 6000)
    ring = O.ring_build(ids)
    F = np.ascontiguousarray(O.fingers(ring), dtype=np.uint32)
    n = len(ring)
    ib = max(1, (n - 1).bit_length())
    Rl = ((ib + 8 + 3) // 4) * 4
    l0, gs = 128 - Rl, 116 - ib
    rc = np.ascontiguousarray(ring, dtype=np.uint64)
    for mode in (0, 1):
        for r5 in (1, 0):
            for rep in range(3):
                out = np.zeros(Rl * 2 * n * 16, dtype=np.uint32)
                esc = np.zeros(2, dtype=np.uint32)
                e = T.cxt_cz_build(mode, r5, p(rc), p(F), n, l0, Rl, gs, p(out), p(esc))
                rec = {"lib": LIBN, "ring": kind, "mode": mode, "encode": "r5" if r5 else "r6",
                       "rep": rep, "rc": e, "not_none": int((out != 0xFFFFFFFF).sum()),
                       "esc": int(esc[0]), "oob": int(esc[1]),
                       "hash": hashlib.sha1(out.tobytes()).hexdigest()[:12]}
                if kind == "cluster" and rec["not_none"]:
                    # where the representable words are: word w of entry (plane, row)
                    idx = np.nonzero(out != 0xFFFFFFFF)[0]
                    slot, ent = idx % 16, idx // 16
                    plane, row = ent // n, ent % n
                    rec["by_slot"] = np.bincount(slot, minlength=16).tolist()
                    rec["by_level"] = {int(l0 + k): int(c) for k, c in
                                       enumerate(np.bincount(plane // 2, minlength=Rl)) if c}
                    rec["by_b"] = np.bincount(plane % 2, minlength=2).tolist()
                    rec["lane_hist"] = np.bincount(row % 64, minlength=64).tolist()
                    rec["wave_in_block"] = np.bincount((row % 256) // 64, minlength=4).tolist()
                    rec["sample"] = [[int(plane[k]), int(row[k]), int(slot[k]),
                                      hex(int(out[idx[k]]))] for k in range(0, len(idx),
                                                                        max(1, len(idx) // 12))]
                print(json.dumps(rec), flush=True)
