#!/usr/bin/env python3
"""Misplaced scan at config C5 (2^24-peer ring, 2^26 keys, n = 14, 1 % joins
+ 1 % leaves): average cx_misplaced time over 5 calls (HIP events), keys/s and
a checksum of the outputs.  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


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
    pick = torch.empty((N // 100, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(pick, 0x5EED0009, offset=1 << 40)
    leaves = old.ids_device()[pick[:, 0].remainder(N)].contiguous()
    new, o2n = old.churn(joins, leaves)
    out = old.misplaced(new, o2n, keys, n)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(5):
        out = old.misplaced(new, o2n, keys, n)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 5
    lists, count, mask, target = out
    ck = [int(lists.to(torch.int64).sum()), int(count.to(torch.int64).sum()),
          int(mask.to(torch.int64).sum()), int(target.to(torch.int64).sum())]
    print(json.dumps({"ms": ms, "keys_per_s": Q / (ms * 1e-3), "checksum": ck,
                      "misplaced_keys": int((mask != 0).sum())}))


if __name__ == "__main__":
    main()
