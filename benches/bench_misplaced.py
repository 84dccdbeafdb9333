#!/usr/bin/env python3
"""Misplaced scan at config C5 (2^24-peer ring, 2^26 keys, n = 14, 1 % joins
+ 1 % leaves): average cx_misplaced time over 5 calls (HIP events), keys/s and
a checksum of the outputs, for the churn directory (variant 1, its build in
the first call) and the two-search path (variant 0).  One JSON line."""
import json
import os
import sys
import time

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
    s = torch.cuda.current_stream()
    res = {}
    # variant 1 (churn directory) first: its first call includes the build
    for v in [int(x) for x in os.environ.get("CX_MISPLACED_VARIANTS", "1,0").split(",")]:
        new.set_misplaced_variant(v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = old.misplaced(new, o2n, keys, n)
        torch.cuda.synchronize()
        first_ms = (time.perf_counter() - t0) * 1e3
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
        res[f"variant{v}"] = {"ms": ms, "keys_per_s": Q / (ms * 1e-3), "first_call_ms": first_ms,
                              "checksum": ck, "misplaced_keys": int((mask != 0).sum())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
