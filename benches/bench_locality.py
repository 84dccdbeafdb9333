#!/usr/bin/env python3
"""Does key order in the batch change the walk's rate?  (diagnostic)

The C4 batch (2^24-peer ring 0x5EED0005, 2^25 keys 0x5EED0006) routed by the
default walk in four orders of the same lookups or keys:
  given      src = q mod N, keys in generation order (the bench's workload)
  rand_src   the same keys, sources a random permutation of the given ones
  by_key     the given (src, key) pairs sorted by key (sources travel along)
  by_key_q   keys sorted, src = q mod N (a different workload: upper bound of
             what key locality alone could give)
Rounds alternate the orders; each lookup's owner is checked equal across
orders (through the permutation).  Prints one JSON line.
    python benches/bench_locality.py [reps] [rounds]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def main():
    argv = sys.argv[1:]
    reps = int(argv[0]) if len(argv) > 0 else 10
    rounds = int(argv[1]) if len(argv) > 1 else 4
    N, Q = 1 << 24, 1 << 25
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    del ids
    ring.build_fingers()
    keys = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0006)
    src = (torch.arange(Q, device="cuda", dtype=torch.int64) % ring.n).to(torch.int32)
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    perm_src = torch.randperm(Q, device="cuda", generator=g)
    hi_u = keys[:, 1] ^ torch.tensor(-(1 << 63), dtype=torch.int64, device="cuda")
    order = torch.sort(hi_u, stable=True).indices
    del hi_u
    work = {
        "given": (src, keys, None),
        "rand_src": (src[perm_src].contiguous(), keys, None),
        "by_key": (src[order].contiguous(), keys[order].contiguous(), order),
        "by_key_q": (src, keys[order].contiguous(), order),
    }
    o = (torch.empty(Q, dtype=torch.int32, device="cuda"),
         torch.empty(Q, dtype=torch.uint8, device="cuda"),
         torch.empty(Q, dtype=torch.uint8, device="cuda"))
    ring.route(src, keys, out=o)
    base_owner = o[0].clone()
    res = {"peers": N, "keys": Q, "checks": {}, "counters": {}, "ms": {k: [] for k in work}}
    for name, (s, k, perm) in work.items():
        ring.route_counters(True)
        ring.route(s, k, out=o)
        res["counters"][name] = ring.route_counters(False)
        want = base_owner if perm is None else base_owner[perm]
        res["checks"][name] = bool((o[0] == want).all()) and int((o[2] != 0).sum()) == 0
    stream = torch.cuda.current_stream()
    for r in range(rounds):
        names = list(work) if r % 2 == 0 else list(reversed(work))
        for name in names:
            s, k, _ = work[name]
            ring.route(s, k, out=o)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ring.sync()
            a.record(stream)
            for _ in range(reps):
                ring.route(s, k, out=o)
            ring.sync()
            b.record(stream)
            torch.cuda.synchronize()
            res["ms"][name].append(a.elapsed_time(b) / reps)
    res["ms_median"] = {k: statistics.median(v) for k, v in res["ms"].items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
