#!/usr/bin/env python3
"""Churn -> route-ready (row f2, config C5 sizes): 2^24-peer ring, 1 % joins +
1 % leaves, then the new ring's finger table and pattern-keyed route table,
timed wall-clock per stage (run under rocprofv3 --kernel-trace --stats for
per-kernel times).  Both table-build inputs (finger level planes / row-major
fingers) are built and their table hashes compared; the new ring then routes
2^24 keys, checked against its exact successor.
    python benches/bench_churn.py [log2 peers]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def keys_dev(n, seed, offset=0):
    k = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(k, seed, offset)
    return k


def wall(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, r


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    N = 1 << lg
    old = chordx.Ring(keys_dev(N, 0x5EED0007))
    t_old, _ = wall(old.build_fingers)
    joins = keys_dev(N // 100, 0x5EED0009)
    # distinct leaving peers (an odd stride is a bijection mod 2^lg): n stays 2^lg
    pick = (torch.arange(N // 100, device="cuda", dtype=torch.int64) * 0x9E3779B1) % N
    leaves = old.ids_device()[pick].contiguous()
    wall(lambda: old.churn(joins, leaves))  # warm the churn allocations
    t_churn, (new, o2n) = wall(lambda: old.churn(joins, leaves))
    out = {"log2_peers": lg, "ring_new": new.n, "old_fingers_and_table_s": t_old,
           "churn_s": t_churn}
    for name, v in (("rows", 1), ("planes_only", 2), ("planes", 0), ("planes_again", 0)):
        new.set_table_build(v)
        t, _ = wall(new.build_fingers)
        out[f"fingers_and_table_{name}_s"] = t
        out[f"hash_{name}"] = new.route_table_hash()
    out["identical"] = (out["hash_rows"] == out["hash_planes_only"] == out["hash_planes"]
                        == out["hash_planes_again"])
    out["route_ready_after_churn_s"] = t_churn + out["fingers_and_table_planes_again_s"]
    keys = keys_dev(1 << 24, 0x5EED0008)
    src = (torch.arange(1 << 24, device="cuda", dtype=torch.int64) % new.n).to(torch.int32)
    owner, hops, status = new.route(src, keys)
    succ = new.successor(keys)
    torch.cuda.synchronize()
    out["route_ok"] = bool((status == 0).all()) and bool((owner == succ).all())
    out["variant"], out["escapes"], out["table_bytes"] = new.route_info()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
