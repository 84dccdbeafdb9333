#!/usr/bin/env python3
"""Does the ring built first route slower?  (benches/bench_depth.py found the
first-built ring ~2.5 % slower in both build orders.)  Same IDs, same default
depth: ring 1 and ring 2 timed in interleaved rounds; then ring 1 is closed and
ring 3 built (its tables come back from the pool or fresh HBM) and ring 2 vs 3
timed the same way.  Results must be identical.  Per ring: (median ms, the
request-rate probe on its table in 10^9 gathers/s); CX_DEBUG_TABLE_VA=1 prints
each table's address.
    python benches/bench_place.py [rounds] [reps]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def timed(rings, outs, src, keys, rounds, reps):
    ms = {k: [] for k in rings}
    s = torch.cuda.current_stream()
    names = list(rings)
    for r in range(rounds):
        for k in (names if r % 2 == 0 else names[::-1]):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(reps):
                rings[k].route(src, keys, out=outs[k])
            b.record(s)
            torch.cuda.synchronize()
            ms[k].append(a.elapsed_time(b) / reps)
    return {k: (round(statistics.median(v), 4), round(rings[k].gather_probe() / 1e9, 2)) for k, v in ms.items()}


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    N, Q = 1 << 24, 1 << 25
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    keys = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0006)
    src = (torch.arange(Q, device="cuda", dtype=torch.int64) % N).to(torch.int32)

    def make():
        r = chordx.Ring(ids)
        r.build_fingers()
        o = (torch.empty(Q, dtype=torch.int32, device="cuda"),
             torch.empty(Q, dtype=torch.uint8, device="cuda"),
             torch.empty(Q, dtype=torch.uint8, device="cuda"))
        for _ in range(3):
            r.route(src, keys, out=o)
        return r, o

    # PLACE_DUMMY=1: a 1000-peer ring made first and kept alive takes the
    # process's first ring stream (and first small blocks); r1 then gets the
    # second stream, as r2 does without it
    dummy = None
    if os.environ.get("PLACE_DUMMY"):
        dids = torch.empty((1000, 2), dtype=torch.int64, device="cuda")
        chordx.fill_splitmix(dids, 0x5EED0999)
        dummy = chordx.Ring(dids)
        dummy.build_fingers()
    rings, outs = {}, {}
    rings["r1"], outs["r1"] = make()
    rings["r2"], outs["r2"] = make()
    torch.cuda.synchronize()
    rec = {"first_pair": timed(rings, outs, src, keys, rounds, reps)}
    same = bool((outs["r1"][0] == outs["r2"][0]).all()) and bool((outs["r1"][1] == outs["r2"][1]).all())
    rings["r1"].close()
    del rings["r1"], outs["r1"]
    rings["r3"], outs["r3"] = make()
    torch.cuda.synchronize()
    rec["after_replacing_r1"] = timed(rings, outs, src, keys, rounds, reps)
    same = same and bool((outs["r3"][0] == outs["r2"][0]).all()) and bool((outs["r3"][1] == outs["r2"][1]).all())
    rec["identical_results"] = same
    # a ring made by the churn path (one join, one leave: same size, near-identical
    # IDs) beside the fresh ones: is it the construction path, not the build order?
    j = torch.empty((1, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(j, 0x5EED0777)
    lv = rings["r2"].ids_device()[12345:12346].contiguous()
    ch, _ = rings["r2"].churn(j, lv)
    ch.build_fingers()
    rings["churned"] = ch
    outs["churned"] = tuple(torch.empty_like(x) for x in outs["r2"])
    for _ in range(3):
        ch.route(src, keys, out=outs["churned"])
    torch.cuda.synchronize()
    rec["with_churned"] = timed(rings, outs, src, keys, rounds, reps)
    rec["pool"] = chordx.pool_info() if hasattr(chordx, "pool_info") else None
    rec["dummy_first"] = dummy is not None
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
