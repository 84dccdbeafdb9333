#!/usr/bin/env python3
"""Route-table build A/B (row f2): a 2^24-peer ring (seed 0x5EED0007), the
converged fingers + pattern-keyed table built twice (the second into mapped
HBM), wall time and route_table_hash of the second build.  The build variant
comes from the environment (CX_CZ_PAIR, CX_CZ_CHUNK, CX_CZ_STORE: read once
per process), so run one process per variant under rocprofv3 --kernel-trace
--stats for per-kernel times.  With CX_CZ_PAIR in {0, 1} the hash must equal
the default build's.
    python benches/bench_czbuild.py [log2 peers] [table_builds, e.g. 0,4] [rounds]
(table_build 0: root-centric, blocks sized by distinct roots (default); 4:
root-centric, 256-row blocks; 3: one lane per entry)
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
           "variant_env": {k: os.environ.get(k) for k in
                           ("CX_CZ_PAIR", "CX_CZ_CHUNK", "CX_CZ_STORE", "CX_CZ_ROOTS_MODE",
                            "CX_CZ2_WPE", "CX_CZ2_MODE")},
           "fingers_and_table_ms": ts,
           "median_ms": {tb: sorted(v)[len(v) // 2] for tb, v in ts.items()},
           "route_table_hash": hashes, "hashes_equal": len(set(hashes.values())) == 1,
           "route_variant": v, "escapes": esc}
    # probes (stores-only / compute-only) leave an unspecified table: no route
    if os.environ.get("CX_CZ_PAIR", "0") in ("0", "1") and \
            os.environ.get("CX_CZ_ROOTS_MODE", "0") == "0" and \
            os.environ.get("CX_CZ2_MODE", "0") in ("0", "32"):  # 32: streaming stores
        q = 1 << 22
        keys = torch.empty((q, 2), dtype=torch.int64, device="cuda")
        chordx.fill_splitmix(keys, 0x5EED0008)
        src = (torch.arange(q, device="cuda", dtype=torch.int64) % ring.n).to(torch.int32)
        o, h, s = ring.route(src, keys)
        out["route_ok"] = bool((o == ring.successor(keys)).all()) and int((s != 0).sum()) == 0
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
