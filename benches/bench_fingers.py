#!/usr/bin/env python3
"""Finger-table build (row a6, configs C3 and C4 sizes): wall time of the
streaming window build (fingers + route table) and a checksum of the table.
Run under rocprofv3 --kernel-trace --stats for per-kernel times
(k_fingers_plan / k_fingers_tile); prints one JSON line.
    python benches/bench_fingers.py [log2 peers ...]
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))


def run(lg, seed):
    import torch
    import chordx
    ids = torch.empty((1 << lg, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, seed)
    ring = chordx.Ring(ids)
    del ids
    ring.set_route_variant(0)  # no route table: time the finger kernel alone
    out = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ring.build_fingers()
        ring.sync()
        out.append(time.perf_counter() - t0)
    F = ring.fingers_device().clone()
    return min(out), F


def main():
    if os.environ.get("CX_BENCH_FINGERS_CHILD"):
        lg = int(sys.argv[1])
        t, F = run(lg, 0x5EED0005 if lg == 24 else 0x5EED0003)
        import torch
        h = int(torch.sum(F.to(torch.int64) * torch.arange(1, F.shape[1] + 1, device=F.device)).item())
        print(json.dumps({"log2_peers": lg, "wall_s": t, "checksum": h}), flush=True)
        return
    res = {}
    for lg in [int(x) for x in sys.argv[1:]] or [20, 24]:
        for name, extra in (("tile", {}),):
            env = dict(os.environ, CX_BENCH_FINGERS_CHILD="1", **extra)
            r = subprocess.run([sys.executable, __file__, str(lg)], env=env, capture_output=True,
                               text=True, timeout=600)
            if r.returncode:
                print(r.stderr[-3000:], file=sys.stderr)
                sys.exit(r.returncode)
            res[f"{lg}_{name}"] = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
