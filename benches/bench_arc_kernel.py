#!/usr/bin/env python3
"""A/B of the replicated cz walk (cx_route) and the key-first arc walk
(cx_arc_route) on ONE rank (world 1: the arc layout holds every row), same
ring, same lookups (C4 per GPU: 2^24 peers, 2^25 keys, src = q mod N).
Prints one JSON object; run under rocprofv3 for per-kernel PMC."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def timed(fn, reps=5):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    N, Q = 1 << int(os.environ.get("PEERS_LOG2", 24)), 1 << int(os.environ.get("KEYS_LOG2", 25))
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    keys = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0006)
    src = (torch.arange(Q, device="cuda") % N).to(torch.int32)
    out = {"peers": N, "keys": Q}
    ring = chordx.Ring(ids)
    ring.build_fingers()
    o = (torch.empty(Q, dtype=torch.int32, device="cuda"),
         torch.empty(Q, dtype=torch.uint8, device="cuda"),
         torch.empty(Q, dtype=torch.uint8, device="cuda"))
    out["replicated_ms"] = timed(lambda: ring.route(src, keys, out=o))
    del ring
    torch.cuda.empty_cache()
    arc = chordx.Ring(ids)
    arc.arc_build(1, 0)
    res = torch.empty(Q, dtype=torch.int64, device="cuda")
    out["arc_route_ms"] = timed(lambda: arc.arc_route(src, keys, res))
    perm = torch.randperm(Q, device="cuda")
    s2, k2 = src[perm].contiguous(), keys[perm].contiguous()
    out["arc_route_shuffled_ms"] = timed(lambda: arc.arc_route(s2, k2, res))
    ow = (res & 0xFFFFFFFF).to(torch.int32)
    o2 = arc.arc_route(src, keys, res)
    out["equal"] = bool(torch.equal((o2 & 0xFFFFFFFF).to(torch.int32), o[0]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
