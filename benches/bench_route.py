#!/usr/bin/env python3
"""Lean headline-kernel timer for A/B work: C4 per GPU (2^24-peer ring, 2^25
keys, src = q mod N), default route kernel, HIP events over `reps` launches
after warm-up, repeated `rounds` times (min and median reported); checks owner
== successor.  Prints one JSON line.
    python benches/bench_route.py [reps] [rounds] [--variants] [--footprint]
--variants also times the A/B kernels on the same batch (moved out of bench.py,
whose driver run keeps its HBM for the arc and churn legs): route variants
0, 4, 5 (finger + ring gathers, lookahead tree, pattern-keyed window table;
each builds its own table, up to 64 GiB) and the
exact-successor searches (directory, Eytzinger, wave-cooperative 16-ary tree).
CX_ORDER=keysorted routes the batch in key order (sort time reported apart).
CX_SRC=random draws each lookup's source peer uniformly instead (splitmix,
seed 0x5EED000A): the first hops of a wave no longer leave adjacent peers.
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402


def timed(fn, reps=3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def variants(ring, src, keys, owner):
    """A/B kernels on the same batch; every result must equal the default's."""
    Q = keys.shape[0]
    out = {"route_variant_kernel_ms": {}, "search_lookups_per_s": {}}
    res = (torch.empty_like(owner), torch.empty(Q, dtype=torch.uint8, device="cuda"),
           torch.empty(Q, dtype=torch.uint8, device="cuda"))
    same = True
    for v in (0, 4, 5):
        ring.set_route_variant(v)
        out["route_variant_kernel_ms"][v] = timed(lambda: ring.route(src, keys, out=res))
        same = same and bool((res[0] == owner).all())
    ring.set_route_variant(-1)
    succ = torch.empty_like(owner)
    for v, name in ((1, "directory"), (0, "eytzinger"), (2, "wave16"), (3, "eyt16")):
        ring.set_search_variant(v)
        ms = timed(lambda: ring.successor(keys, out=succ))
        out["search_lookups_per_s"][name] = Q / (ms * 1e-3)
        same = same and bool((succ == owner).all())
    ring.set_search_variant(1)
    out["variants_equal_default"] = same
    return out


def main():
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    reps = int(argv[0]) if len(argv) > 0 else 10
    rounds = int(argv[1]) if len(argv) > 1 else 5
    N, Q = 1 << 24, 1 << 25
    ids = torch.empty((N, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    del ids
    ring.build_fingers()
    keys = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(keys, 0x5EED0006)
    src_kind = os.environ.get("CX_SRC", "mod")
    if src_kind == "random":
        r = torch.empty((Q, 2), dtype=torch.int64, device="cuda")
        chordx.fill_splitmix(r, 0x5EED000A)
        src = (r[:, 0] & 0x7FFFFFFFFFFFFFFF).remainder(N).to(torch.int32)
        del r
    else:
        src = (torch.arange(Q, device="cuda", dtype=torch.int64) % N).to(torch.int32)
    order = os.environ.get("CX_ORDER", "input")
    sort_ms = None
    if order == "keysorted":
        # A/B: the batch in key order -- adjacent lookups'
        # last hops share lower-plane lines -- with the sort's own time (a
        # 64-bit sort of the keys' high words, the pairs permuted along)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        hi = keys[:, 1] ^ torch.iinfo(torch.int64).min  # unsigned order as signed
        perm = torch.sort(hi).indices
        keys = keys[perm].contiguous()
        src = src[perm].contiguous()
        b.record()
        torch.cuda.synchronize()
        sort_ms = a.elapsed_time(b)
        del hi, perm
    owner = torch.empty(Q, dtype=torch.int32, device="cuda")
    hops = torch.empty(Q, dtype=torch.uint8, device="cuda")
    status = torch.empty(Q, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(3):
        ring.route(src, keys, out=(owner, hops, status))
    ms = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            ring.route(src, keys, out=(owner, hops, status))
        b.record(s)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b) / reps)
    ok = bool((owner == ring.successor(keys)).all()) and int((status != 0).sum()) == 0
    hops_sum = int(hops.to(torch.int64).sum())
    ring.route_counters(True)  # the counting build: random requests the walk issues
    ring.route(src, keys, out=(owner, hops, status))
    g64, r16, xc, nq = ring.route_counters(False)
    same_counting = hops_sum == int(hops.to(torch.int64).sum())
    rec = {"lib": os.path.basename(os.environ.get("CHORDX_LIB", "default")),
           "src": src_kind, "order": order, "sort_ms": sort_ms,
           "ms_min": min(ms), "ms_median": statistics.median(ms),
           "lookups_per_s": Q / (min(ms) * 1e-3), "probe": ring.gather_probe(),
           "owner_ok": ok, "mean_hops": float(hops.double().mean()), "hops_sum": hops_sum,
           "route_R": ring.route_info()[2] // (ring.n * 128),
           "per_lookup": {"table_gathers": g64 / Q, "exact_id_gathers": r16 / Q,
                          "exact_hops": xc / Q}, "counting_same_hops": same_counting}
    if "--footprint" in sys.argv:
        # request ceiling vs table footprint, on the real route table's memory
        rec["probe_by_span_GiB"] = {g: ring.gather_probe(span=g << 30)
                                    for g in (1, 4, 16, 32, 48, 64)}
    if "--variants" in sys.argv:
        rec.update(variants(ring, src, keys, owner))
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
