"""Diagnostic: route time of a churned ring (cx_churn of the bench ring, 1 %/1 %)
against a fresh ring built from the churned ring's IDs and against the bench
ring itself, interleaved rounds on the bench's keys (src = q mod n of each)."""
import json
import os
import statistics
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + "/p2p-dhts_amd", R + "/oracle"]
import torch  # noqa: E402
import chordx  # noqa: E402

N, Q = 1 << 24, 1 << 25
dev = torch.device("cuda")
ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
chordx.fill_splitmix(ids, 0x5EED0005)
a = chordx.Ring(ids)
a.build_fingers()
keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
chordx.fill_splitmix(keys, 0x5EED0006)
joins = torch.empty((N // 100, 2), dtype=torch.int64, device=dev)
chordx.fill_splitmix(joins, 0x5EED0009)
leaves = a.ids_device()[::100][: N // 100].clone()
b, _ = a.churn(joins, leaves)
b.build_fingers()
c = chordx.Ring(b.ids_device().clone())
c.build_fingers()
rings = {"bench": a, "churned": b, "fresh_same_ids": c}
outs = {k: (torch.empty(Q, dtype=torch.int32, device=dev), torch.empty(Q, dtype=torch.uint8, device=dev),
            torch.empty(Q, dtype=torch.uint8, device=dev)) for k in rings}
srcs = {k: (torch.arange(Q, device=dev) % r.n).to(torch.int32) for k, r in rings.items()}
ms = {k: [] for k in rings}
s = torch.cuda.current_stream()
for rnd in range(6):
    order = list(rings) if rnd % 2 == 0 else list(rings)[::-1]
    for k in order:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        rings[k].route(srcs[k], keys, out=outs[k])
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(3):
            rings[k].route(srcs[k], keys, out=outs[k])
        e1.record(s)
        torch.cuda.synchronize()
        ms[k].append(e0.elapsed_time(e1) / 3)
same = bool(torch.equal(outs["churned"][0], outs["fresh_same_ids"][0])) and \
    bool(torch.equal(outs["churned"][1], outs["fresh_same_ids"][1]))
print(json.dumps({"ms_median": {k: statistics.median(v) for k, v in ms.items()},
                  "churned_equals_fresh": same,
                  "route_info": {k: r.route_info() for k, r in rings.items()},
                  "hops_mean": {k: float(outs[k][1].float().mean()) for k in rings}}))
