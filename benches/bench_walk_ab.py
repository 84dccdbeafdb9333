#!/usr/bin/env python3
"""Round-5 walk A/B: the straight-line walk (k_walk, cx_walk.hip) against the
round-4 walk (k_route_tree<false, true>) on the same C4 batch (2^24-peer ring
0x5EED0005, 2^25 keys 0x5EED0006, src = q mod N), alternating ABAB... rounds
of `reps` launches timed with HIP events on the ring's stream.  Checks owner
and hops equal between the two and owner == exact successor, and counts the
gathers of each (counting builds).  Prints one JSON line.
    python benches/bench_walk_ab.py [reps] [rounds] [log2 peers] [log2 keys]
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402
from chordx import _lib as L  # noqa: E402


def main():
    argv = sys.argv[1:]
    reps = int(argv[0]) if len(argv) > 0 else 10
    rounds = int(argv[1]) if len(argv) > 1 else 6
    lg = int(argv[2]) if len(argv) > 2 else 24
    lq = int(argv[3]) if len(argv) > 3 else 25
    N, Q = 1 << lg, 1 << lq
    ab = L.lib().cxi_ab_old_walk
    ab.argtypes = [ctypes.c_int]
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    del ids
    ring.build_fingers()
    keys = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0006)
    src = (torch.arange(Q, device="cuda", dtype=torch.int64) % ring.n).to(torch.int32)
    outs = {}
    for name, old in (("new", 0), ("old", 1)):
        ab(old)
        o = (torch.empty(Q, dtype=torch.int32, device="cuda"),
             torch.empty(Q, dtype=torch.uint8, device="cuda"),
             torch.empty(Q, dtype=torch.uint8, device="cuda"))
        ring.route(src, keys, out=o)
        ring.route_counters(True)
        ring.route(src, keys, out=o)
        cnt = ring.route_counters(False)
        outs[name] = (o, cnt)
    succ = torch.empty(Q, dtype=torch.int32, device="cuda")
    ring.successor(keys, out=succ)
    (on, cn), (oo, co) = outs["new"], outs["old"]
    res = {"peers": N, "keys": Q,
           "owner_equal": bool((on[0] == oo[0]).all()), "hops_equal": bool((on[1] == oo[1]).all()),
           "status_equal": bool((on[2] == oo[2]).all()),
           "owner_is_successor": bool((on[0] == succ).all()),
           "bad_status_new": int((on[2] != 0).sum()),
           "mean_hops": float(on[1].float().mean()),
           "counters_new": cn, "counters_old": co}
    if not res["hops_equal"]:
        bad = (on[1] != oo[1]).nonzero().flatten()[:8].tolist()
        res["hops_diff_first"] = [(i, int(on[1][i]), int(oo[1][i]), int(on[0][i]), int(oo[0][i]))
                                  for i in bad]
    ms = {"new": [], "old": []}
    stream = torch.cuda.current_stream()
    o = outs["new"][0]
    for r in range(rounds):
        for name, old in (("new", 0), ("old", 1)) if r % 2 == 0 else (("old", 1), ("new", 0)):
            ab(old)
            ring.route(src, keys, out=o)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ring.sync()
            a.record(stream)
            for _ in range(reps):
                ring.route(src, keys, out=o)
            ring.sync()
            b.record(stream)
            torch.cuda.synchronize()
            ms[name].append(a.elapsed_time(b) / reps)
    ab(0)
    res["ms"] = ms
    res["ms_median"] = {k: statistics.median(v) for k, v in ms.items()}
    res["lookups_per_s_median"] = {k: Q / (v * 1e-3) for k, v in res["ms_median"].items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
