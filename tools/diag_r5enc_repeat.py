"""Diagnostic (round 6): route-table builds 0 / 1 / 2 / 3 on
the all-escape cluster ring (every word of its table is CZ_NONE), repeated, with
the package under CHORDX_PKG (ab/old_r5enc/p2p-dhts_amd: the tree before commit
0a5da05 with its library built from that tree's sources; its encode took the
exact-ID branch through a variable u128 shift).
Prints per build the words that came out representable (should be 0) and the
table hash."""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.environ.get("CHORDX_PKG", R + "/p2p-dhts_amd"), R + "/oracle"]
import chordx  # noqa: E402
import oracle as O  # noqa: E402

base = 0x3C3C_5A5A_0F0F_1234 << 64
ids = O.keys_from_ints([base + i * 7919 for i in range(6000)])
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    ring = chordx.Ring(ids)
    out = []
    for tb in (0, 1, 2, 3, 2, 1, 2):
        ring.set_table_build(tb)
        ring.build_fingers()
        v, esc, nbytes = ring.route_info()
        out.append({"tb": tb, "representable": nbytes // 4 - esc,
                    "hash": ring.route_table_hash() % 10**8})
    print(json.dumps({"lib": os.path.basename(chordx._lib.LIB_PATH), "rep": rep, "builds": out}),
          flush=True)
    ring.close()
