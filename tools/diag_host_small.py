"""Host-memory (CX_MEM_HOST) call latency for small batches: cx_route and
cx_successor with numpy inputs on the C4 ring (2^24 peers), wall time per call
averaged over 200 calls.  Prints one JSON line."""
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + "/p2p-dhts_amd"]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import chordx  # noqa: E402

N = 1 << 24
ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
chordx.fill_splitmix(ids, 0x5EED0005)
ring = chordx.Ring(ids)
del ids
ring.build_fingers()
res = {}
for q in (1, 64, 4096, 65536):
    kt = torch.empty((q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(kt, 0x5EED0006)
    keys = kt.cpu().numpy().view(np.uint64).reshape(q, 2).copy()
    src = (np.arange(q) % N).astype(np.uint32)
    for _ in range(5):
        ring.route(src, keys)
    t0 = time.perf_counter()
    for _ in range(200):
        o, h, s = ring.route(src, keys)
    t_route = (time.perf_counter() - t0) / 200 * 1e6
    for _ in range(5):
        ring.successor(keys)
    t0 = time.perf_counter()
    for _ in range(200):
        ring.successor(keys)
    t_succ = (time.perf_counter() - t0) / 200 * 1e6
    res[str(q)] = {"route_us": t_route, "successor_us": t_succ}
print(json.dumps(res))
