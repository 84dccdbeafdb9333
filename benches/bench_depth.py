#!/usr/bin/env python3
"""Route-table depth A/B in one process (same HBM state for every variant):
C4 per GPU (2^24-peer ring, 2^25 keys, src = q mod N), one ring per depth R
(cxi_set_route_depth: table levels [128 - R, 128)), the route kernel timed
with HIP events in interleaved rounds (ring A, ring B, ring A, ...), plus each
ring's churn -> route-ready on a 1 %/1 % churn.  Owners, hops and statuses
must be identical for every depth (the walk is the same; only where exact
hops replace table gathers changes).
    python benches/bench_depth.py [R,R,...] [rounds] [reps]
"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def main():
    depths = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "32,28").split(",")]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    N, Q = 1 << 24, 1 << 25
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    keys = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0006)
    src = (torch.arange(Q, device="cuda", dtype=torch.int64) % N).to(torch.int32)
    rings, outs = {}, {}
    for R in depths:
        r = chordx.Ring(ids)
        r.set_route_depth(R)
        r.build_fingers()
        rings[R] = r
        o = (torch.empty(Q, dtype=torch.int32, device="cuda"),
             torch.empty(Q, dtype=torch.uint8, device="cuda"),
             torch.empty(Q, dtype=torch.uint8, device="cuda"))
        for _ in range(3):
            r.route(src, keys, out=o)
        outs[R] = o
    torch.cuda.synchronize()
    ms = {R: [] for R in depths}
    s = torch.cuda.current_stream()
    for k in range(rounds):
        order = depths if k % 2 == 0 else depths[::-1]
        for R in order:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(reps):
                rings[R].route(src, keys, out=outs[R])
            b.record(s)
            torch.cuda.synchronize()
            ms[R].append(a.elapsed_time(b) / reps)
    base = depths[0]
    same = all(bool((outs[R][0] == outs[base][0]).all()) and bool((outs[R][1] == outs[base][1]).all())
               and int((outs[R][2] != 0).sum()) == 0 for R in depths)
    succ = rings[base].successor(keys)
    ok = bool((outs[base][0] == succ).all())
    rec = {"depths": depths, "rounds": rounds, "reps": reps, "identical_results": same,
           "owner_equals_successor": ok, "route": {}}
    for R in depths:
        v, esc, tb = rings[R].route_info()
        rings[R].route_counters(True)
        rings[R].route(src, keys, out=outs[R])
        g64, r16, xc, _ = rings[R].route_counters(False)
        rec["route"][R] = {"ms_min": min(ms[R]), "ms_median": statistics.median(ms[R]),
                           "lookups_per_s_median": Q / (statistics.median(ms[R]) * 1e-3),
                           "table_bytes": tb, "table_gathers": g64 / Q,
                           "exact_id_gathers": r16 / Q, "exact_hops": xc / Q}
    del outs
    # churn -> route-ready per depth (the churned ring inherits nothing: set R)
    nj = N // 100
    joins = torch.empty((nj, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(joins, 0x5EED0009)
    pick = (torch.arange(nj, device="cuda", dtype=torch.int64) * 0x9E3779B1) % N
    for R in depths:
        leaves = rings[R].ids_device()[pick].contiguous()
        t = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            new, _ = rings[R].churn(joins, leaves)
            new.set_route_depth(R)
            new.build_fingers()
            new.sync()
            t.append((time.perf_counter() - t0) * 1e3)
            new.close()
            del new
        rec["route"][R]["route_ready_ms"] = t
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
