#!/usr/bin/env python3
"""C2 exact successor (2^16-peer ring 0x5EED0001, 2^20 keys 0x5EED0002):
300 back-to-back cx_successor calls, HIP-event timed (us per call, GPU side),
outputs checked against the first call.  Run under rocprofv3 --kernel-trace
--stats for the kernel-only time.  Prints one JSON line.
    python benches/bench_c2.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def main():
    ids = torch.empty((1 << 16, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0001)
    ring = chordx.Ring(ids)
    keys = torch.empty((1 << 20, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0002)
    out = torch.empty(1 << 20, dtype=torch.int32, device="cuda")
    want = ring.successor(keys).clone()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(300):
        ring.successor(keys, out=out)
    b.record(s)
    torch.cuda.synchronize()
    print(json.dumps({"us_per_call": a.elapsed_time(b) / 300 * 1e3,
                      "identical": bool(torch.equal(out, want)),
                      "lib": os.environ.get("CHORDX_LIB", "in-tree")}))


if __name__ == "__main__":
    main()
