#!/usr/bin/env python3
"""Arc-sharded routing on ONE GPU with G simulated ranks (SURVEY 8e layout 2).

G engine handles share one MI355X; each holds the replicated top-level route
planes and the lower planes of its own arc (+ halo) only (cx_arc_build), and
records are exchanged in-process exactly as chordx.arc.ArcRouter does over
RCCL.  Per round and rank we time the walk step and the bucketing on the GPU
(HIP events) and count the records that would cross xGMI, so the per-GPU cost
of an 8-GPU arc-sharded run can be read off one box:

  per-GPU compute  ~ max over ranks of (step + bucket) per round, summed
  per-GPU exchange ~ records out per rank per round x 32 B over 7 xGMI links
  projected rate   = keys per rank / (compute + exchange)   (no overlap)

Prints one JSON object (profiles/<round>/arc_sim.json).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402
from chordx.arc import MAX_ROUNDS  # noqa: E402

XGMI_LINK = 153e9  # B/s per link per direction (MI355X_MICROARCH.md)


def run(G, N, Q, ids, reps, top, key_first):
    rings = [chordx.Ring(ids) for _ in range(G)]
    for g, r in enumerate(rings):
        r.arc_build(G, g, top)
    info = [r.arc_info() for r in rings]
    q = Q // G
    keys, srcs, outs = [], [], []
    for g in range(G):
        k = torch.empty((q, 2), dtype=torch.int64, device="cuda")
        chordx.fill_splitmix(k, 0x5EED0006, offset=g * q)
        keys.append(k)
        srcs.append((torch.arange(g * q, (g + 1) * q, device="cuda") % N).to(torch.int32))
        outs.append((torch.empty(q, dtype=torch.int32, device="cuda"),
                     torch.empty(q, dtype=torch.uint8, device="cuda"),
                     torch.empty(q, dtype=torch.uint8, device="cuda")))
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    best = None
    for _ in range(reps):
        # origin mode: first step straight from the lookups (cx_arc_start);
        # key_first: seed records, sent ahead by key in round 1 (no origin walk)
        recs = [None] * G
        per_round = []
        t0 = time.perf_counter()
        for rnd in range(MAX_ROUNDS):
            inbox = [[] for _ in range(G)]
            total = 0
            rows = []
            for g in range(G):
                a, b, c = ev(), ev(), ev()
                a.record()
                if key_first and rnd == 0:  # fused seed + bucket (cx_arc_send_ahead)
                    b.record()
                    send, counts = rings[g].arc_send_ahead(G, g, srcs[g], keys[g])
                    c.record()
                else:
                    if recs[g] is None:
                        out = rings[g].arc_start(g, srcs[g], keys[g], *outs[g])
                    else:
                        out = rings[g].arc_step(g, recs[g], *outs[g])
                    b.record()
                    send, counts = rings[g].arc_bucket(G, out)
                    c.record()
                torch.cuda.synchronize()
                rows.append({"in": int(keys[g].shape[0] if recs[g] is None else recs[g].shape[0]),
                             "step_ms": a.elapsed_time(b),
                             "bucket_ms": b.elapsed_time(c),
                             "out_remote": int(sum(counts) - counts[g])})
                total += sum(counts)
                for d, part in enumerate(torch.split(send, counts)):
                    inbox[d].append(part)
            per_round.append(rows)
            if total == 0:
                break
            recs = [torch.cat(b) if b else torch.empty((0, 4), dtype=torch.int64,
                                                       device="cuda") for b in inbox]
        wall = time.perf_counter() - t0
        comp = sum(max(r["step_ms"] + r["bucket_ms"] for r in rows) for rows in per_round)
        xg = sum(max(r["out_remote"] for r in rows) * 32 / (7 * XGMI_LINK) * 1e3
                 for rows in per_round)
        res = {"G": G, "mode": "key_first" if key_first else "origin_walk", "keys_total": Q, "keys_per_rank": q, "rounds": len(per_round),
               "top_levels": info[0][0], "local_rows_max": max(i[1] for i in info),
               "route_plane_bytes_per_gpu_max": max(i[2] for i in info),
               "per_gpu_compute_ms": comp, "per_gpu_xgmi_ms_model": xg,
               "projected_lookups_per_s_per_gpu": q / ((comp + xg) * 1e-3),
               "sim_wall_s": wall,
               "records_in_per_round": [sum(r["in"] for r in rows) for rows in per_round],
               "round_max_ms": [max(r["step_ms"] + r["bucket_ms"] for r in rows)
                                for rows in per_round],
               "round_max_step_ms": [max(r["step_ms"] for r in rows) for rows in per_round],
               "round_max_bucket_ms": [max(r["bucket_ms"] for r in rows) for rows in per_round]}
        if best is None or comp < best["per_gpu_compute_ms"]:
            best = res
    del rings
    torch.cuda.empty_cache()
    return best


def run_soa(G, N, Q, ids, reps, top, want=None, regions=False, hints=False):
    """Key-first SoA protocol (ArcRouter.route_soa): per rank partition, walk
    of the receive buffer, delivery; xGMI = 20 B out + 8 B back per remote
    lookup.  want = replicated (owner, hops) to check against."""
    rings = [chordx.Ring(ids) for _ in range(G)]
    for g, r in enumerate(rings):
        r.arc_build(G, g, top)
    info = [r.arc_info() for r in rings]
    q = Q // G
    keys, srcs, outs = [], [], []
    for g in range(G):
        k = torch.empty((q, 2), dtype=torch.int64, device="cuda")
        chordx.fill_splitmix(k, 0x5EED0006, offset=g * q)
        keys.append(k)
        srcs.append((torch.arange(g * q, (g + 1) * q, device="cuda") % N).to(torch.int32))
        outs.append((torch.empty(q, dtype=torch.int32, device="cuda"),
                     torch.empty(q, dtype=torch.uint8, device="cuda"),
                     torch.empty(q, dtype=torch.uint8, device="cuda")))
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    best = None
    for _ in range(reps):
        part_ms, route_ms, deliv_ms, remote_out, remote_in = [], [], [], [], []
        parts, caps = [], []
        cap = q // G + q // (4 * G) + 4096
        for g in range(G):
            a, b = ev(), ev()
            a.record()
            p = rings[g].arc_partition_regions(G, srcs[g], keys[g], cap, hints=hints) \
                if regions else None
            if p is None:
                p = rings[g].arc_partition(G, srcs[g], keys[g])
            parts.append(p)
            b.record()
            torch.cuda.synchronize()
            caps.append(cap if p[0].shape[0] == G * cap and regions else 0)
            part_ms.append(a.elapsed_time(b))
            remote_out.append(sum(parts[g][3]) - parts[g][3][g])

        def views(t, g):
            c, cnt = caps[g], parts[g][3]
            if c:
                return [t[d * c: d * c + cnt[d]] for d in range(G)]
            return list(torch.split(t, cnt))
        ks = [views(p[0], g) for g, p in enumerate(parts)]
        ss = [views(p[1], g) for g, p in enumerate(parts)]
        hs = [views(p[4], g) for g, p in enumerate(parts)] if hints else None
        back = [[None] * G for _ in range(G)]
        for d in range(G):
            rk = torch.cat([ks[g][d] for g in range(G)])
            rs = torch.cat([ss[g][d] for g in range(G)])
            rh = torch.cat([hs[g][d] for g in range(G)]) if hints else None
            remote_in.append(rk.shape[0] - parts[d][3][d])
            a, b = ev(), ev()
            a.record()
            res = rings[d].arc_route(rs, rk, hint=rh)
            b.record()
            torch.cuda.synchronize()
            route_ms.append(a.elapsed_time(b))
            for g, part in enumerate(torch.split(res, [parts[g][3][d] for g in range(G)])):
                back[g][d] = part
            del rk, rs, res
        for g in range(G):
            if caps[g]:  # answers in their region slots (the return all_to_all's layout)
                bk = torch.empty(G * caps[g], dtype=torch.int64, device="cuda")
                for d in range(G):
                    bk[d * caps[g]: d * caps[g] + parts[g][3][d]] = back[g][d]
            else:
                bk = torch.cat(back[g])
            a, b = ev(), ev()
            a.record()
            rings[g].arc_deliver(bk, parts[g][2], *outs[g])
            b.record()
            torch.cuda.synchronize()
            deliv_ms.append(a.elapsed_time(b))
        del parts, ks, ss, back
        comp = max(part_ms) + max(route_ms) + max(deliv_ms)
        # each rank sends and receives over its 7 links; bound by the larger side
        wire = 28 if hints else 20  # bytes out per remote lookup (+ 8 back)
        xg = (max(max(remote_out), max(remote_in)) * wire + max(max(remote_out), max(remote_in)) * 8) \
            / (7 * XGMI_LINK) * 1e3
        res = {"G": G, "mode": ("soa_hints" if hints else "soa_regions") if regions else "soa",
               "keys_total": Q,
               "keys_per_rank": q,
               "top_levels": info[0][0], "local_rows_max": max(i[1] for i in info),
               "route_plane_bytes_per_gpu_max": max(i[2] for i in info),
               "partition_ms_max": max(part_ms), "route_ms_max": max(route_ms),
               "route_ms": route_ms, "deliver_ms_max": max(deliv_ms),
               "per_gpu_compute_ms": comp, "per_gpu_xgmi_ms_model": xg,
               "projected_lookups_per_s_per_gpu": q / ((comp + xg) * 1e-3),
               "projected_lookups_per_s_per_gpu_overlapped": q / (max(comp, xg) * 1e-3),
               "remote_out_max": max(remote_out)}
        if best is None or comp < best["per_gpu_compute_ms"]:
            best = res
    if want is not None:
        ok = True
        for g in range(G):
            ok &= bool(torch.equal(outs[g][0], want[0][g * q:(g + 1) * q]))
            ok &= bool(torch.equal(outs[g][1], want[1][g * q:(g + 1) * q]))
        best["equals_replicated"] = ok
    del rings
    torch.cuda.empty_cache()
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers-log2", type=int, default=24)
    ap.add_argument("--keys-log2", type=int, default=25, help="keys in total over the G ranks")
    ap.add_argument("--groups", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--top-levels", type=int, default=0, help="0: library default")
    ap.add_argument("--modes", default="soa,key_first,origin_walk")
    a = ap.parse_args()
    N, Q = 1 << a.peers_log2, 1 << a.keys_log2
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    ref = chordx.Ring(ids)
    ref.build_fingers()
    k = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(k, 0x5EED0006)
    s = (torch.arange(Q, device="cuda") % N).to(torch.int32)
    o = (torch.empty(Q, dtype=torch.int32, device="cuda"),
         torch.empty(Q, dtype=torch.uint8, device="cuda"),
         torch.empty(Q, dtype=torch.uint8, device="cuda"))
    ref.route(s, k, out=o)
    a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a0.record()
    ref.route(s, k, out=o)
    a1.record()
    torch.cuda.synchronize()
    out = {"peers": N, "keys": Q, "replicated_route_ms": a0.elapsed_time(a1), "arc": []}
    want = (o[0].clone(), o[1].clone())
    del ref, o, k, s
    torch.cuda.empty_cache()
    for G in [int(x) for x in a.groups.split(",")]:
        for mode in a.modes.split(","):
            if mode in ("soa", "soa_regions", "soa_hints"):
                out["arc"].append(run_soa(G, N, Q, ids, a.reps, a.top_levels, want,
                                          regions=mode != "soa", hints=mode == "soa_hints"))
            else:
                out["arc"].append(run(G, N, Q, ids, a.reps, a.top_levels, mode == "key_first"))
            print(json.dumps(out["arc"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
