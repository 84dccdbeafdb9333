"""Diagnostic: repeat route-table builds 1 / 2 / 3 on the clustered edge ring and
print the escape counts (every entry of this ring escapes: 6000 * R * 16)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + "/p2p-dhts_amd", R + "/oracle"]
import chordx  # noqa: E402
import oracle as O  # noqa: E402

base = 0x3C3C_5A5A_0F0F_1234 << 64
ids = O.keys_from_ints([base + i * 7919 for i in range(6000)])
for rep in range(3):
    ring = chordx.Ring(ids)
    out = []
    for tb in (0, 1, 2, 3, 1, 2, 1, 2):
        ring.set_table_build(tb)
        ring.build_fingers()
        out.append((tb, ring.route_info()[1], ring.route_table_hash() % 100000))
    print(rep, out, flush=True)
    ring.close()
