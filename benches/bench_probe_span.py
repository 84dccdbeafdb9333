#!/usr/bin/env python3
"""Request ceiling against route-table footprint up to the size the two-bit
pattern key would need (four 64-B entries per (level, peer) at
R = 28 = 112 GiB at 2^24).  A ring built with a 56-level table
(cxi_set_route_depth) holds 2^24 x 56 x 128 B = 112 GiB; the dependent 64-B
gather probe (cxi_gather_probe_span) runs over its first 28 / 56 / 84 / 112
GiB, beside the default 28-level (56 GiB) ring's full table, alternating.
The two-bit key pays only if the 112-GiB rate stays >= 0.919 x the 56-GiB
rate (its 8 % fewer gathers per lookup, tools/cz_window_sim.py).
    python benches/bench_probe_span.py
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
    base = chordx.Ring(ids)
    base.set_route_depth(28)  # the 28-level (56 GiB) table the docstring compares against
    base.build_fingers()
    big = chordx.Ring(ids)
    big.set_route_depth(56)
    big.build_fingers()
    del ids
    GiB = 1 << 30
    tb_base, tb_big = base.route_info()[2], big.route_info()[2]
    spans = [s for s in (28 * GiB, 56 * GiB, 84 * GiB) if s < tb_big] + [0]
    rates = {"base_full": []}
    for s in spans:
        rates[f"big_{(s or tb_big) // GiB}GiB"] = []
    for r in range(3):
        rates["base_full"].append(base.gather_probe())
        for s in spans:
            rates[f"big_{(s or tb_big) // GiB}GiB"].append(big.gather_probe(span=s) if s
                                                           else big.gather_probe())
    med = {k: sorted(v)[len(v) // 2] for k, v in rates.items()}
    full_big = med[f"big_{tb_big // GiB}GiB"]
    print(json.dumps({"table_bytes": {"base": tb_base, "big": tb_big}, "rates": rates,
                      "median": med,
                      "big_full_vs_base_full": full_big / med["base_full"],
                      "two_bit_key_break_even": 0.919,
                      "two_bit_key_pays": full_big / med["base_full"] > 0.919 * 1.05}),
          flush=True)


if __name__ == "__main__":
    main()
