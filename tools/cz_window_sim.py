#!/usr/bin/env python3
"""Gathers per lookup of pattern-keyed window walks (route variant 5,
cx_kernels.hip k_route_tree / cz_plan) for other entry shapes.

An entry for (cur, level i) is keyed by j pattern bits: bits i-1 .. i-j of
d - 2^i, d = key - id_cur.  It holds the chain the bits predict: the root
A = F[cur][i], then one finger per set bit.  Hanging off the chain's end is
the full subtree of fingers over the next D levels, i-1-j .. i-j-D, taken in
descending order.  `cap` limits the entry to that many nodes; deeper subsets
are dropped first.

The engine's 64-B entry is j = 1, D = 4, cap = 16.  With rb = 1 the window hangs
off F[A][i-1], and the one four-level subset is dropped to make room for A.

The walk is the reference's greedy finger walk (abstract_chord_peer.cpp:318-337,
finger_table.h:115-130): hop to F[cur][msb(key - id_cur)] until the key lies
in (id_cur, id_nxt].  A hop whose path is not in the current entry costs one
gather.  Exact-ID fix-ups are not modelled; they are about 0.03 per lookup on
the GPU.  Sources are src = q mod N, as in config C4.

Usage: python tools/cz_window_sim.py [log2 peers] [lookups]
At 2^24 and 3 x 10^4 lookups it prints 4.038 for the engine's shape.  The GPU's
counting build measures 4.034 table gathers per lookup.
"""
import bisect
import itertools
import random
import sys

M128 = (1 << 128) - 1

# (j, D, cap, what it would cost)
SHAPES = [
    (1, 4, 16, "engine: 64-B entry, 2 entries per (peer, level), 64 GiB at 2^24"),
    (2, 4, 16, "two-bit key: 64-B entry, 4 entries per (peer, level), 128 GiB"),
    (3, 3, 16, "three-bit key, three-level window: 64-B entry, 256 GiB"),
    (1, 5, 32, "five-level window: 128-B entry, 128 GiB"),
]


def main():
    lg = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    Q = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    rng = random.Random(0x5EED0005)
    ids = sorted({rng.getrandbits(128) for _ in range(1 << lg)})
    n = len(ids)

    def succ(x):
        k = bisect.bisect_left(ids, x & M128)
        return 0 if k == n else k

    memo = {}

    def finger(p, l):
        k = (p << 7) | l
        v = memo.get(k)
        if v is None:
            v = succ(ids[p] + (1 << l))
            memo[k] = v
        return v

    def entry_paths(i, d, j, D, cap):
        """Level sequences (starting at i) whose end node the entry holds."""
        if i <= j:
            return {(i,)}
        bits = [((d - (1 << i)) >> (i - 1 - t)) & 1 for t in range(j)]
        chain = [i] + [i - 1 - t for t in range(j) if bits[t]]
        paths = {tuple(chain[:k]) for k in range(1, len(chain) + 1)}
        window = [i - 1 - j - t for t in range(D) if i - 1 - j - t >= 0]
        subsets = [c for r in range(1, len(window) + 1) for c in itertools.combinations(window, r)]
        subsets.sort(key=len)  # shallow subsets first: the deepest are dropped
        for c in subsets[:cap - len(chain)]:
            paths.add(tuple(chain) + c)
        return paths

    base = None
    for j, D, cap, what in SHAPES:
        gathers = hops = 0
        krng = random.Random(0x5EED0006)
        for q in range(Q):
            key = krng.getrandbits(128)
            cur = q % n
            d = (key - ids[cur]) & M128
            # the source owns the key: no hop (StoredLocally at the source)
            if d == 0 or ((ids[cur] - ids[cur - 1]) & M128) >= ((ids[cur] - key) & M128) > 0:
                continue
            paths, path = None, None
            while True:
                i = d.bit_length() - 1
                if paths is not None and path + (i,) in paths:
                    path = path + (i,)
                else:
                    gathers += 1
                    paths, path = entry_paths(i, d, j, D, cap), (i,)
                nxt = finger(cur, i)
                step = (ids[nxt] - ids[cur]) & M128
                hops += 1
                if d <= step:
                    break
                d -= step
                cur = nxt
        g = gathers / Q
        base = base or g
        print(f"2^{lg} peers, j={j} D={D} cap={cap}: {g:.3f} gathers/lookup "
              f"({g / base:.3f}x), {hops / Q:.2f} hops/lookup  [{what}]", flush=True)


if __name__ == "__main__":
    main()
