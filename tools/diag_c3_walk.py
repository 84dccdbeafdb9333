"""Diagnostic: the walk's gather rate against the request ceiling on the C3
ring (2^20 peers, 2^24 lookups) and on the C4 ring (2^24 peers, 2^25 lookups):
gather probe on each ring's own table, walk time, counted gathers."""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + "/p2p-dhts_amd"]
import torch  # noqa: E402
import chordx  # noqa: E402

dev = torch.device("cuda")


def one(lg, lq, s_ids, s_keys):
    N, Q = 1 << lg, 1 << lq
    ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(ids, s_ids)
    ring = chordx.Ring(ids)
    ring.build_fingers()
    keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(keys, s_keys)
    src = (torch.arange(Q, device=dev, dtype=torch.int64) % N).to(torch.int32)
    out = (torch.empty(Q, dtype=torch.int32, device=dev), torch.empty(Q, dtype=torch.uint8, device=dev),
           torch.empty(Q, dtype=torch.uint8, device=dev))
    ring.route_counters(True)
    ring.route(src, keys, out=out)
    torch.cuda.synchronize()
    g = ring.route_counters(False)
    for _ in range(3):
        ring.route(src, keys, out=out)
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(s)
    for _ in range(10):
        ring.route(src, keys, out=out)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / 10
    probe = ring.gather_probe()
    req = (g[0] + g[1]) / (ms * 1e-3)
    rand = ring.route(((torch.arange(Q, device=dev) * 0x9E3779B1) % N).to(torch.int32), keys, out=out)
    res = {"lg": lg, "lq": lq, "ms": ms, "gathers": g, "gathers_per_lookup": (g[0] + g[1]) / Q,
           "requests_per_s": req, "probe": probe, "frac": req / probe,
           "table_gib": ring.route_info()[2] / 2**30}
    ring.close()
    return res


print(json.dumps([one(20, 24, 0x5EED0003, 0x5EED0004), one(24, 25, 0x5EED0005, 0x5EED0006)]))
