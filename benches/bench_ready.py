#!/usr/bin/env python3
"""Churn -> route-ready wall time, stage by stage, repeated (the warm steady
state of a membership epoch): cx_churn (1 % joins + 1 % leaves of a 2^24-peer
ring, bench.py's churn leg) then cx_fingers_build on the new ring.  Run under
rocprofv3 --kernel-trace --hip-trace --stats to see where the wall time that
is not kernel time goes.
    python benches/bench_ready.py [log2 peers] [repeats]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    N = 1 << lg
    dev = torch.device("cuda")
    ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    # CX_READY_REPAIR=1: the churned rings remap the parent's finger planes
    # (the f2 repair A/B) instead of searching them from scratch
    ring.set_fingers_repair(os.environ.get("CX_READY_REPAIR", "0") == "1")
    ring.build_fingers()
    ring.sync()
    nj = N // 100
    joins = torch.empty((nj, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(joins, 0x5EED0009)
    pick = (torch.arange(nj, device=dev, dtype=torch.int64) * 0x9E3779B1) % N
    leaves = ring.ids_device()[pick].contiguous()
    rows = []
    hashes = set()
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        new, _ = ring.churn(joins, leaves)
        new.sync()
        t1 = time.perf_counter()
        new.build_fingers()
        new.sync()
        t2 = time.perf_counter()
        hashes.add(new.route_table_hash())
        repaired, searched = new.fingers_repair_info()
        new.close()
        del new
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        rows.append({"churn_ms": (t1 - t0) * 1e3, "fingers_and_table_ms": (t2 - t1) * 1e3,
                     "route_ready_ms": (t2 - t0) * 1e3, "close_ms": (t3 - t2) * 1e3,
                     "fingers_repaired": repaired, "repair_searched": searched})
    print(json.dumps({"log2_peers": lg, "reps": rows, "hashes_equal": len(hashes) == 1,
                      "hash": hashes.pop()}), flush=True)


if __name__ == "__main__":
    main()
