#!/usr/bin/env python3
"""Where the arc rank's own-lookup walk loses time (diagnostic, G ranks
simulated on one GPU, rank 0's view; C4 per-rank batch as bench_arc_exact_sim).

  inplace   cx_arc_route_local over own_idx (the default: keys / sources read
            at the lookups' indices, outputs written there)
  compact   the same lookups gathered into contiguous arrays first (not timed),
            walked by cx_arc_route_local over 0..c-1 (contiguous reads and
            outputs, the same index stage)
  packed    the compacted lookups through cx_arc_route (no index stage, packed
            8-B results in order), as a received region is walked
Alternating rounds, HIP-event timed; owners / hops checked equal across the
three.  Prints one JSON line.
    python benches/bench_own_walk.py [G] [rounds]
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def timed(fn):
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b)


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    N, Q = 1 << 24, 1 << 25
    dev = torch.device("cuda")
    ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    del ids
    ring.build_fingers()
    keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(keys, 0x5EED0006)
    src = (torch.arange(Q, device=dev) % N).to(torch.int32)
    ring.arc_build(G, 0)
    row = torch.zeros(G, dtype=torch.int64, device=dev)
    own_idx = torch.empty(Q, dtype=torch.int32, device=dev)
    ws = torch.empty(ring.arc_own_ws_words(Q), dtype=torch.int32, device=dev)
    ring.arc_count_async(G, keys, row, 0, own_idx, ws)
    c = int(row[0])
    idx = own_idx[:c]
    ck, cs = keys[idx.long()].contiguous(), src[idx.long()].contiguous()
    seq = torch.arange(c, dtype=torch.int32, device=dev)
    ow = torch.full((Q,), -1, dtype=torch.int32, device=dev)
    hp = torch.zeros(Q, dtype=torch.uint8, device=dev)
    st = torch.zeros(Q, dtype=torch.uint8, device=dev)
    cow = torch.empty(c, dtype=torch.int32, device=dev)
    chp = torch.empty(c, dtype=torch.uint8, device=dev)
    cst = torch.empty(c, dtype=torch.uint8, device=dev)
    res = torch.empty(c, dtype=torch.int64, device=dev)
    il = idx.long()
    ck2, cs2 = torch.empty_like(ck), torch.empty_like(cs)
    runs = {
        "inplace": lambda: ring.arc_route_local(src, keys, idx, ow, hp, st),
        "compact": lambda: ring.arc_route_local(cs, ck, seq, cow, chp, cst),
        "packed": lambda: ring.arc_route(cs, ck, res=res),
        # torch copies of the same lookups' bytes: where scattered access costs
        "r_gather": lambda: (torch.index_select(keys, 0, il, out=ck2), torch.index_select(src, 0, il, out=cs2)),
        "r_contig": lambda: (ck2.copy_(keys[:c]), cs2.copy_(src[:c])),
        "w_scatter": lambda: (ow.index_copy_(0, il, cow), hp.index_copy_(0, il, chp), st.index_copy_(0, il, cst)),
        "w_contig": lambda: (ow[:c].copy_(cow), hp[:c].copy_(chp), st[:c].copy_(cst)),
    }
    for k in ("inplace", "compact", "packed"):
        runs[k]()
    torch.cuda.synchronize()
    same = bool(torch.equal(ow[idx.long()], cow)) and bool(torch.equal(hp[idx.long()], chp)) \
        and bool(torch.equal((res & 0xFFFFFFFF).to(torch.int32), cow)) \
        and bool(torch.equal(((res >> 32) & 0xFF).to(torch.uint8), chp)) \
        and int((cst != 0).sum()) == 0
    for k in runs:
        runs[k]()
    ms = {k: [] for k in runs}
    for r in range(rounds):
        for k in (runs if r % 2 == 0 else list(reversed(list(runs)))):
            ms[k].append(timed(runs[k]))
    print(json.dumps({"G": G, "own_lookups": c, "same_results": same, "ms": ms,
                      "ms_median": {k: statistics.median(v) for k, v in ms.items()}}), flush=True)


if __name__ == "__main__":
    main()
