#!/usr/bin/env python3
"""Route-table build timer (row f2): a 2^24-peer ring (seed 0x5EED0007), the
converged fingers + pattern-keyed table built `rounds` times per build input
(alternating ABAB...), wall time and route_table_hash of each; kernel-level A/Bs
use two builds of the library (CHORDX_LIB, tools/ab_lib.sh) under rocprofv3
--kernel-trace --stats.  Routes 2^22 keys through the result.
    python benches/bench_czbuild.py [log2 peers] [table_builds, e.g. 0,3] [rounds]
(table_build 0: root-centric, blocks sized by distinct roots (default); 3: one
lane per entry; 1: from the row-major fingers; 2: level planes only)
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
    # cxi_set_table_build variants, comma-separated: built alternately into the
    # same ring (ABAB...), `rounds` times each, so box and placement are shared
    tbs = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0").split(",")]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ids = torch.empty((1 << lg, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0007)
    ring = chordx.Ring(ids)
    del ids
    ts = {tb: [] for tb in tbs}
    hashes = {}
    ring.build_fingers()  # first touch of the tables, untimed
    for r in range(rounds):
        for tb in (tbs if r % 2 == 0 else tbs[::-1]):
            ring.set_table_build(tb)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ring.build_fingers()
            ring.sync()
            ts[tb].append((time.perf_counter() - t0) * 1e3)
            hashes[tb] = ring.route_table_hash()
    v, esc, table_bytes = ring.route_info()
    out = {"log2_peers": lg, "table_builds": tbs, "rounds": rounds,
           "lib": os.environ.get("CHORDX_LIB", "in-tree"),
           "fingers_and_table_ms": ts,
           "median_ms": {tb: sorted(v)[len(v) // 2] for tb, v in ts.items()},
           "route_table_hash": hashes, "hashes_equal": len(set(hashes.values())) == 1,
           "route_variant": v, "escapes": esc}
    if True:
        q = 1 << 22
        keys = torch.empty((q, 2), dtype=torch.int64, device="cuda")
        chordx.fill_splitmix(keys, 0x5EED0008)
        src = (torch.arange(q, device="cuda", dtype=torch.int64) % ring.n).to(torch.int32)
        o, h, s = ring.route(src, keys)
        out["route_ok"] = bool((o == ring.successor(keys)).all()) and int((s != 0).sum()) == 0
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
