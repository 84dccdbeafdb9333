#!/usr/bin/env python3
"""Gathers per lookup of the pattern-keyed window walk (route variant 5,
cx_kernels.hip k_route_tree / cz_plan) as a function of the window depth D.

An entry (cur, i, rb) holds the root A = F[cur][i] and the subtree of
fingers hanging off R0 (rb = 0: R0 = A; rb = 1: R0 = F[A][i-1]) at levels
i-2 .. i-1-D taken in descending order: 2^D nodes for rb = 0, 2^D for rb = 1
(the all-levels node is dropped to make room for A).  D = 4 is the 64-B entry
the engine stores (16 x 4 B); D = 5 would be a 128-B entry.  The walk is
the reference's greedy finger walk (abstract_chord_peer.cpp:318-337,
finger_table.h:115-130): hop to F[cur][msb(key - id_cur)] until the key lies
in (id_cur, id_nxt].  A hop whose node is not in the current entry costs one
gather (exact-ID fix-ups, about 0.03 per lookup on the GPU, are not modelled).

Usage: python tools/cz_window_sim.py [log2 peers] [lookups]
"""
import bisect
import random
import sys

M128 = (1 << 128) - 1


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    Q = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    rng = random.Random(0x5EED0005)
    ids = sorted({rng.getrandbits(128) for _ in range(1 << lg)})
    n = len(ids)

    def succ(x):
        j = bisect.bisect_left(ids, x & M128)
        return 0 if j == n else j

    memo = {}

    def finger(p, l):
        k = (p << 7) | l
        v = memo.get(k)
        if v is None:
            v = succ(ids[p] + (1 << l))
            memo[k] = v
        return v

    res = {}
    for D in (4, 5):
        full = (1 << D) - 1
        gathers = hops = 0
        krng = random.Random(0x5EED0006)
        for q in range(Q):
            key = krng.getrandbits(128)
            cur = q % n
            d = (key - ids[cur]) & M128
            # the source owns the key: no hop (StoredLocally at the source)
            if d == 0 or ((ids[cur] - ids[cur - 1]) & M128) >= ((ids[cur] - key) & M128) > 0:
                continue
            cs = -1  # -1: no entry; 'A': on the root of an rb = 1 entry; else subset bits
            ri = rb = 0
            while True:
                i = d.bit_length() - 1
                hit = False
                if cs == 'A':
                    if ri - i == 1:
                        v, hit = 0, True
                elif cs != -1 and 2 <= ri - i <= 1 + D:
                    v = cs | (1 << (ri - i - 2))
                    hit = not (rb and v == full)
                if hit:
                    cs = v
                else:
                    gathers += 1
                    ri = i
                    rb = ((d - (1 << i)) >> (i - 1)) & 1 if i > 0 else 0
                    cs = 'A' if rb else 0
                nxt = finger(cur, i)
                step = (ids[nxt] - ids[cur]) & M128
                hops += 1
                if d <= step:
                    break
                d -= step
                cur = nxt
        res[D] = (gathers / Q, hops / Q)
        print(f"2^{lg} peers, D={D} ({4 << D} B entry): {gathers / Q:.3f} gathers/lookup, "
              f"{hops / Q:.2f} hops/lookup", flush=True)
    g4, g5 = res[4][0], res[5][0]
    print(f"D=5 vs D=4: {g5 / g4:.3f}x the gathers")


if __name__ == "__main__":
    main()
