#!/usr/bin/env python3
"""Exact successor at C4 size (2^24-peer ring 0x5EED0005, 2^25 keys
0x5EED0006): `reps` cx_successor launches (the bucket-directory search; the
ring is too large for the LDS slice table), HIP-event timed, with the
request model of bench.dir_search_requests (directory entries + the ring IDs
the in-bucket binary search reads, replayed on the host and checked: the
replay's answers equal the GPU's).  Run under rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE for the measured traffic.  Prints one JSON line.
    python benches/bench_succ.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import chordx  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    N, Q = 1 << 24, 1 << 25
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    del ids
    keys = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0006)
    out = torch.empty(Q, dtype=torch.int32, device="cuda")
    ring.successor(keys, out=out)
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(reps):
        ring.successor(keys, out=out)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    m = bench.exact_successor_record(ring, keys, out, ms, 1, torch.device("cuda"))
    print(json.dumps({"peers": N, "keys": Q, "ms": ms, "record": m}), flush=True)


if __name__ == "__main__":
    main()
