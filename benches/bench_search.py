#!/usr/bin/env python3
"""Exact successor search variants (rows a5/a7): bucket directory (default),
Eytzinger with LDS top levels, wave-cooperative 16-ary tree, wave-cooperative
Eytzinger (16 lanes a query, ballot over four levels) -- kernel time by
HIP events on the launch stream, at C2 (2^16 ring, 2^20 keys) and C4 sizes
(2^24 ring, 2^25 keys); every variant's output is compared with the default.
    python benches/bench_search.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def keys_dev(n, seed):
    k = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(k, seed)
    return k


def timed(fn, reps=5):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    out = {}
    for name, lg, lq, s1, s2 in (("C2", 16, 20, 0x5EED0001, 0x5EED0002),
                                 ("C4", 24, 25, 0x5EED0005, 0x5EED0006)):
        ring = chordx.Ring(keys_dev(1 << lg, s1))
        keys = keys_dev(1 << lq, s2)
        res = torch.empty(1 << lq, dtype=torch.int32, device="cuda")
        ref = None
        row = {}
        for v, vn in ((1, "directory"), (0, "eytzinger"), (2, "wave16"), (3, "eyt_wave16")):
            ring.set_search_variant(v)
            ms = timed(lambda: ring.successor(keys, out=res))
            same = True if ref is None else bool((res == ref).all())
            if ref is None:
                ref = res.clone()
            pms = timed(lambda: ring.predecessor(keys, out=res))
            row[vn] = {"successor_ms": ms, "lookups_per_s": (1 << lq) / (ms * 1e-3),
                       "predecessor_ms": pms, "identical": same}
        out[name] = row
        del ring, keys, res, ref
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
