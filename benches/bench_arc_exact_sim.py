#!/usr/bin/env python3
"""The exact-layout arc path (ArcRouter.route_exact) with G ranks simulated on
ONE GPU, at C4's per-rank batch: a projection of the per-GPU cost of an
N = G arc-sharded run from one box (SURVEY 8e layout 2).

One engine plays every rank in turn (cx_arc_build(G, g) before rank g's
work).  Per origin rank g (its 2^25 keys, splitmix 0x5EED0006 at offset
g Q, src = q mod N as bench.py): the count pass with its own lookups'
indices, the exact-layout scatter of the others (hints included), and the
in-place walk of its own lookups.  Per destination rank d: the lookups every
other origin sent it (the regions d of their scatters, concatenated as the
all_to_all delivers them) walked from their hints.  Per origin again: the
delivery of its remote answers.  Each piece is HIP-event timed; owners, hops
and statuses of every origin's lookups are checked against the replicated
walk (cx_route on the same ring).

  per-rank compute = count + scatter + own walk + received walk + deliver
                     (the scatter overlaps the walks in route_exact: also
                     reported without it)
  per-rank exchange = 28 B out per remote lookup + 8 B back, over 7 xGMI
                     links at a stated efficiency (no measured xGMI here)

    python benches/bench_arc_exact_sim.py [G] [log2 keys per rank]
Prints one JSON line.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402

XGMI_LINK = 153e9  # B/s per link per direction (MI355X_MICROARCH.md)


def timed(fn):
    s = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    r = fn()
    b.record(s)
    torch.cuda.synchronize()
    return r, a.elapsed_time(b)


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    lq = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    N, Q = 1 << 24, 1 << lq
    dev = torch.device("cuda")
    ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    del ids
    ring.build_fingers()
    keys, srcs = [], []
    for g in range(G):
        k = torch.empty((Q, 2), dtype=torch.int64, device=dev)
        chordx.fill_splitmix(k, 0x5EED0006, offset=g * Q)
        keys.append(k)
        srcs.append((torch.arange(g * Q, (g + 1) * Q, device=dev) % N).to(torch.int32))
    outs = [(torch.full((Q,), -1, dtype=torch.int32, device=dev),
             torch.zeros(Q, dtype=torch.uint8, device=dev),
             torch.full((Q,), 9, dtype=torch.uint8, device=dev)) for _ in range(G)]
    for rep in range(2):  # rep 0 warms every kernel and table (round 6: rank 0's
        # first own walk ran 1.14 ms cold against 0.69-0.77 warm and set the max)
        res = simulate(ring, G, Q, N, keys, srcs, outs, dev)
    print(json.dumps(res))


def simulate(ring, G, Q, N, keys, srcs, outs, dev):
    for ow, hp, st in outs:  # every repetition writes every output afresh
        ow.fill_(-1)
        hp.fill_(0)
        st.fill_(9)
    t = {k: [0.0] * G for k in ("count", "scatter", "own_walk", "recv_walk", "deliver")}
    parts, counts = [], []
    for g in range(G):  # ---- origin side
        ring.arc_build(G, g)
        row = torch.zeros(G, dtype=torch.int64, device=dev)
        own_idx = torch.empty(Q, dtype=torch.int32, device=dev)
        # sized for either build of the count pass (the round-5 two-kernel pass
        # took 2048 + Q / 4 words of scratch; ab/ A/B runs load that library)
        ws = torch.empty(max(ring.arc_own_ws_words(Q), 2048 + (Q + 3) // 4), dtype=torch.int32,
                         device=dev)
        _, t["count"][g] = timed(lambda: ring.arc_count_async(G, keys[g], row, g, own_idx, ws))
        cnt = row.tolist()
        cur = torch.empty(G, dtype=torch.int32, device=dev)
        part, t["scatter"][g] = timed(lambda: ring.arc_scatter_async(G, srcs[g], keys[g], row, cur,
                                                                      hints=True, skip=g))
        ow, hp, st = outs[g]
        _, t["own_walk"][g] = timed(lambda: ring.arc_route_local(
            srcs[g], keys[g], own_idx[:cnt[g]], ow, hp, st))
        parts.append(part)
        counts.append(cnt)
    answers = [[None] * G for _ in range(G)]  # answers[g][d]: rank d's answers to origin g
    for d in range(G):  # ---- destination side
        ring.arc_build(G, d)
        ks, ss, hs, who = [], [], [], []
        for g in range(G):
            if g == d:
                continue
            off = sum(counts[g][j] for j in range(d) if j != g)
            c = counts[g][d]
            sk, ssrc, _, sh = parts[g]
            ks.append(sk[off:off + c])
            ss.append(ssrc[off:off + c])
            hs.append(sh[off:off + c])
            who.append((g, c))
        rk, rs, rh = torch.cat(ks), torch.cat(ss), torch.cat(hs)
        res, t["recv_walk"][d] = timed(lambda: ring.arc_route(rs, rk, hint=rh))
        at = 0
        for g, c in who:
            answers[g][d] = res[at:at + c]
            at += c
    ok = True
    sent = []
    for g in range(G):  # ---- back at the origins
        back = torch.empty(Q, dtype=torch.int64, device=dev)  # >= perm's length
        rem = torch.cat([answers[g][d] for d in range(G) if d != g])
        back[:rem.shape[0]] = rem
        ow, hp, st = outs[g]
        _, t["deliver"][g] = timed(lambda: ring.arc_deliver(back, parts[g][2], ow, hp, st))
        wo, wh, ws_ = ring.route(srcs[g], keys[g])
        ok = ok and bool(torch.equal(ow, wo)) and bool(torch.equal(hp, wh)) and \
            bool(torch.equal(st, ws_))
        sent.append(sum(counts[g]) - counts[g][g])
    per = [sum(t[k][g] for k in t) for g in range(G)]
    per_overlap = [per[g] - t["scatter"][g] for g in range(G)]
    recv = [sum(counts[g][d] for g in range(G) if g != d) for d in range(G)]
    xbytes = [28 * sent[g] + 8 * recv[g] for g in range(G)]  # out per rank (both directions)
    replicated = timed(lambda: ring.route(srcs[0], keys[0], out=outs[0]))[1]
    res = {"G": G, "keys_per_rank": Q, "peers": N, "equal_to_replicated_route": ok,
           "ms_per_rank": {k: [round(v, 4) for v in t[k]] for k in t},
           "compute_ms_max": max(per), "compute_ms_max_scatter_overlapped": max(per_overlap),
           "replicated_walk_ms": replicated,
           "remote_fraction": sum(sent) / (G * Q),
           "xgmi_bytes_out_per_rank_max": max(xbytes),
           "xgmi_ms_at_50pct_of_7_links": max(xbytes) / (0.5 * 7 * XGMI_LINK) * 1e3,
           "projected_lookups_per_s_per_gpu": {
               "serial": Q / ((max(per) + max(xbytes) / (0.5 * 7 * XGMI_LINK) * 1e3) * 1e-3),
               "overlapped": Q / (max(max(per_overlap),
                                      max(xbytes) / (0.5 * 7 * XGMI_LINK) * 1e3) * 1e-3)},
           "note": "one engine plays every rank (cx_arc_build per rank), the whole simulation "
                   "run twice and the second timed; exchange not measured: 28 B out + 8 B back "
                   "per remote lookup over 7 xGMI links at 50 % of 153 GB/s"}
    return res


if __name__ == "__main__":
    main()
