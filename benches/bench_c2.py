#!/usr/bin/env python3
"""C2 exact successor (2^16-peer ring 0x5EED0001, 2^20 keys 0x5EED0002):
300 back-to-back cx_successor calls, HIP-event timed (us per call, GPU side),
outputs checked against the first call.  Run under rocprofv3 --kernel-trace
--stats for the kernel-only time.  With several search variants (round 6:
1 = default, the LDS slice table at this size; 5 = the bucket directory
alone) they alternate in rounds of 300 calls, each checked against the
directory's answers.  Prints one JSON line.
    python benches/bench_c2.py [variant ...] [--rounds R]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def main():
    argv = sys.argv[1:]
    rounds = 1
    if "--rounds" in argv:
        i = argv.index("--rounds")
        rounds = int(argv[i + 1])
        del argv[i:i + 2]
    variants = [int(v) for v in argv] or [1]
    ids = torch.empty((1 << 16, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0001)
    ring = chordx.Ring(ids)
    keys = torch.empty((1 << 20, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0002)
    out = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    ring.set_search_variant(5)
    want = ring.successor(keys).clone()
    s = torch.cuda.current_stream()
    us = {v: [] for v in variants}
    same = {v: True for v in variants}
    for r in range(rounds):
        for v in (variants if r % 2 == 0 else variants[::-1]):
            ring.set_search_variant(v)
            ring.successor(keys, out=out)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record(s)
            for _ in range(300):
                ring.successor(keys, out=out)
            b.record(s)
            torch.cuda.synchronize()
            us[v].append(a.elapsed_time(b) / 300 * 1e3)
            same[v] = same[v] and bool(torch.equal(out, want))
    print(json.dumps({"us_per_call": min(us[variants[0]]), "identical": all(same.values()),
                      "us_per_call_by_variant": us, "identical_by_variant": same,
                      "lib": os.environ.get("CHORDX_LIB", "in-tree")}))

if __name__ == "__main__":
    main()
