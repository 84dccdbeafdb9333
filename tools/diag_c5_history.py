"""Diagnostic: C5 step time (cx_dhash_maintenance, 2^24 ring, 2^26 keys, 1 %/1 %
churn) in a fresh process, then after the process has built and closed the
bench ring with its 64 GiB route table (pool trimmed), as bench.py's c5 leg
runs it.  Prints one JSON line."""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + "/p2p-dhts_amd"]
import torch  # noqa: E402
import chordx  # noqa: E402

dev = torch.device("cuda")
N, Q, n = 1 << 24, 1 << 26, 14


def c5(tag, steps=10):
    ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(ids, 0x5EED0007)
    old = chordx.Ring(ids)
    del ids
    nj = N // 100
    joins = torch.empty((nj, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(joins, 0x5EED0009)
    pick = (torch.arange(nj, device=dev, dtype=torch.int64) * 0x9E3779B1) % old.n
    leaves = old.ids_device()[pick].contiguous()
    new, o2n = old.churn(joins, leaves)
    new.sync()
    keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(keys, 0x5EED0008)
    for _ in range(3):
        old.dhash_maintenance(new, o2n, keys, n)
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(steps):
        old.dhash_maintenance(new, o2n, keys, n)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / steps
    old.close()
    new.close()
    del old, new, keys, o2n, joins, leaves
    torch.cuda.empty_cache()
    chordx.pool_trim()
    return ms


res = {"fresh": c5("fresh")}
ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
chordx.fill_splitmix(ids, 0x5EED0005)
ring = chordx.Ring(ids)
del ids
ring.build_fingers()
ring.build_fingers()
ring.close()
del ring
torch.cuda.empty_cache()
chordx.pool_trim()
res["after_bench_ring"] = c5("after")
res["again"] = c5("again")
print(json.dumps(res))
