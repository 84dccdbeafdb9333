#!/usr/bin/env python3
"""n-successor lists and the misplaced scan at config C5 (2^24-peer ring,
2^26 keys, n = 14, 1 % joins + 1 % leaves): HIP-event kernel times and an
output checksum, one JSON line (A/B of row-store variants)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


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
    N, Q, n = 1 << 24, 1 << 26, 14
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0007)
    old = chordx.Ring(ids)
    del ids
    keys = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0008)
    joins = torch.empty((N // 100, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(joins, 0x5EED0009)
    pick = (torch.arange(N // 100, device="cuda", dtype=torch.int64) * 0x9E3779B1) % N
    leaves = old.ids_device()[pick].contiguous()
    new, o2n = old.churn(joins, leaves)
    t_ns = timed(lambda: old.nsucc(keys, n))
    lists, count = old.nsucc(keys, n)
    h1 = int((lists.to(torch.int64) * 3 + 1).sum())
    t_mp = timed(lambda: old.misplaced(new, o2n, keys, n))
    l2, c2, m2, t2 = old.misplaced(new, o2n, keys, n)
    h2 = int(l2.to(torch.int64).sum()) + int(m2.to(torch.int64).sum()) + int(t2.to(torch.int64).sum())
    print(json.dumps({"lib": os.path.basename(os.environ.get("CHORDX_LIB", "default")),
                      "nsucc_ms": t_ns, "misplaced_ms": t_mp, "nsucc_hash": h1,
                      "misplaced_hash": h2}), flush=True)


if __name__ == "__main__":
    main()
