#!/usr/bin/env python3
"""Request ceiling of dependent random 64-B gathers on the 2^24 ring's route
table vs the number of chains in flight (cxi_gather_probe, one chain per quad
of lanes): is 46 G/s a memory-system ceiling (flat in the chain count) or a
latency limit of the probe (rising with it)?
    python benches/bench_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def main():
    ids = torch.empty((1 << 24, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    del ids
    ring.build_fingers()
    out = {"chains_in_flight": {}}
    for lg in (15, 16, 17, 18, 19, 20, 21):
        lanes = 1 << (lg + 2)
        out["chains_in_flight"][1 << lg] = max(ring.gather_probe(lanes=lanes, hops=64)
                                              for _ in range(2))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
