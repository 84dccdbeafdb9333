#!/usr/bin/env python3
"""Default walk timer for A/B work (k_walk, cx_walk.hip): the C4 batch
(2^24-peer ring 0x5EED0005, 2^25 keys 0x5EED0006, src = q mod N), `rounds`
rounds of `reps` launches timed around the ring's stream.  Checks owner and
hops against the per-hop walk without a table (route variant 0) and owner ==
exact successor, and counts the walk's gathers (counting build).  Two builds
of the library are compared by running this under each (CHORDX_LIB,
tools/ab_lib.sh).  Prints one JSON line.
    python benches/bench_walk.py [reps] [rounds] [log2 peers] [log2 keys]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def main():
    argv = sys.argv[1:]
    reps = int(argv[0]) if len(argv) > 0 else 10
    rounds = int(argv[1]) if len(argv) > 1 else 6
    lg = int(argv[2]) if len(argv) > 2 else 24
    lq = int(argv[3]) if len(argv) > 3 else 25
    N, Q = 1 << lg, 1 << lq
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    del ids
    ring.build_fingers()
    keys = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0006)
    src = (torch.arange(Q, device="cuda", dtype=torch.int64) % ring.n).to(torch.int32)
    o = (torch.empty(Q, dtype=torch.int32, device="cuda"),
         torch.empty(Q, dtype=torch.uint8, device="cuda"),
         torch.empty(Q, dtype=torch.uint8, device="cuda"))
    ring.route(src, keys, out=o)
    ring.route_counters(True)
    ring.route(src, keys, out=o)
    cnt = ring.route_counters(False)
    succ = torch.empty(Q, dtype=torch.int32, device="cuda")
    ring.successor(keys, out=succ)
    ring.set_route_variant(0)  # per-hop finger + ring gathers, no table
    r0 = ring.route(src, keys)
    ring.set_route_variant(-1)
    res = {"peers": N, "keys": Q, "lib": os.environ.get("CHORDX_LIB", "in-tree"),
           "owner_equal_per_hop_walk": bool((o[0] == r0[0]).all()),
           "hops_equal_per_hop_walk": bool((o[1] == r0[1]).all()),
           "owner_is_successor": bool((o[0] == succ).all()),
           "bad_status": int((o[2] != 0).sum()),
           "mean_hops": float(o[1].float().mean()),
           "counters": cnt}
    del r0
    ms = []
    stream = torch.cuda.current_stream()
    for r in range(rounds):
        ring.route(src, keys, out=o)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ring.sync()
        a.record(stream)
        for _ in range(reps):
            ring.route(src, keys, out=o)
        ring.sync()
        b.record(stream)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b) / reps)
    res["ms"] = ms
    res["ms_median"] = statistics.median(ms)
    res["lookups_per_s_median"] = Q / (res["ms_median"] * 1e-3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
