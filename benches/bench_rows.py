#!/usr/bin/env python3
"""Per-row measurements of the hot-path scope table at the
BASELINE.json configs, one MI355X.  Prints one JSON object (profiles/<round>/rows.json).

  C2  2^16-peer ring, 2^20 keys: exact successor (directory and Eytzinger)
  C3  2^20-peer ring: m=128 finger build; 2^24 routed lookups with hops
  C5  2^24-peer ring, 2^26 keys, n=14: replica lists; 1 % join + 1 % leave
      churn; global-maintenance misplaced scan

Kernel times are HIP events on the launch stream (torch's current stream, which
the library enqueues on for device buffers); host-synchronous calls (ring
build, churn, finger + route-table build) are wall-clock.  Inputs: splitmix
seeds of SURVEY 8(d).

Every row also carries a "cpu" leg (BASELINE.md:39-49): the oracle's C
restatement (oracle/chord_oracle.c, gcc -O3) of the same operation on this
host, on all usable cores and on one core, over a bounded sample of the same
inputs (named in "sample"); each leg also checks the GPU output on its sample.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-dhts_amd"))

import torch  # noqa: E402

import chordx  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

HBM = 8.0e12
CPU_BUDGET_S = float(os.environ.get("CX_ROWS_CPU_S", "6"))


def cpu_leg(fn, total, unit, what, check=None):
    """Times fn(count, threads) on a sample sized to ~CPU_BUDGET_S (2/3 on all
    usable cores, 1/3 on one core).  Returns the cpu dict."""
    from bench import cpu_model, host_threads
    th = host_threads()
    t0 = time.perf_counter()
    fn(min(total, 1024), 1)
    per = max((time.perf_counter() - t0) / min(total, 1024), 1e-9)
    q1 = int(min(total, max(1024, CPU_BUDGET_S / 3 / per)))
    t0 = time.perf_counter()
    fn(q1, 1)
    d1 = time.perf_counter() - t0
    qa = int(min(total, max(q1, CPU_BUDGET_S * 2 / 3 * th / per)))
    t0 = time.perf_counter()
    r = fn(qa, th)
    da = time.perf_counter() - t0
    out = {"value": qa / da, "value_1core": q1 / d1, "unit": unit, "cores": th,
           "kind": "port", "cpu_model": cpu_model(),
           "sample": f"first {qa} of {total} {what} on {th} threads ({da:.1f} s), "
                     f"first {q1} on 1 thread ({d1:.1f} s)"}
    if check is not None:
        out["parity_on_sample"] = bool(check(r, qa))
    return out


def ev_time(fn, reps=3):
    s = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / 1e3


def keys_dev(n, seed, offset=0):
    k = torch.empty((n, 2), dtype=torch.int64, device="cuda")
    chordx.fill_splitmix(k, seed, offset)
    return k


def main():
    out = {"device": torch.cuda.get_device_name(0)}
    # ---------------- C2 ----------------
    ring = chordx.Ring(keys_dev(1 << 16, 0x5EED0001))
    keys = keys_dev(1 << 20, 0x5EED0002)
    res = {}
    for v, name in ((1, "directory"), (0, "eytzinger"), (2, "wave16")):
        ring.set_search_variant(v)
        t = ev_time(lambda: ring.successor(keys))
        res[name] = {"s": t, "lookups_per_s": (1 << 20) / t,
                     "algo_GBps": (1 << 20) * 20 / t / 1e9}
    import oracle as O
    ring_np = ring.ids()
    keys_np = keys.cpu().numpy().view(np.uint64)
    succ_gpu = ring.successor(keys).cpu().numpy().view(np.uint32)
    res["cpu"] = cpu_leg(lambda q, th: O.successor(ring_np, keys_np[:q], threads=th), 1 << 20,
                         "lookups/s", "keys (binary search over the sorted ring)",
                         lambda r, q: (r == succ_gpu[:q]).all())
    out["C2_exact_successor"] = res
    del ring, keys

    # ---------------- C3 ----------------
    N3 = 1 << 20
    ring = chordx.Ring(keys_dev(N3, 0x5EED0003))
    t0 = time.perf_counter()
    ring.build_fingers()
    ring.sync()
    tf = time.perf_counter() - t0
    q = 1 << 24
    keys = keys_dev(q, 0x5EED0004)
    src = (torch.arange(q, device="cuda", dtype=torch.int64) % N3).to(torch.int32)
    owner = torch.empty(q, dtype=torch.int32, device="cuda")
    hops = torch.empty(q, dtype=torch.uint8, device="cuda")
    status = torch.empty(q, dtype=torch.uint8, device="cuda")
    tr = ev_time(lambda: ring.route(src, keys, out=(owner, hops, status)))
    sh = int(hops.to(torch.int64).sum())
    bad3 = int((status != 0).sum())  # before the a9 run below reuses the buffers
    # bench.py's roofline model: 58 B of streams per lookup + 64 B per random
    # gather the walk issued (counted by the counting build on the same batch)
    ring.route_counters(True)
    ring.route(src, keys, out=(owner, hops, status))
    g64, r16, xc, _ = ring.route_counters(False)
    algo = q * 58 + 64 * (g64 + r16 + 2 * xc)
    ring_np = ring.ids()
    F_gpu = ring.fingers_device().cpu().numpy().view(np.uint32)
    cpu_f = cpu_leg(lambda q, th: O.fingers(ring_np, threads=th, rows=(0, q)), N3,
                    "peers/s", "peers' 128-entry finger rows (PopulateFingerTable restated)",
                    lambda r, q: (r == F_gpu[:q]).all())
    P = O.Peers(ring_np, F_gpu)
    src_np = src.cpu().numpy().view(np.uint32)
    kq_np = keys.cpu().numpy().view(np.uint64)
    own_np = owner.cpu().numpy().view(np.uint32)
    hop_np = hops.cpu().numpy()
    cpu_r = cpu_leg(lambda q, th: O.route(P, src_np[:q], kq_np[:q], threads=th), q,
                    "lookups/s", "routed lookups (or_route, literal ForwardRequest walk)",
                    lambda r, qq: (r[0] == own_np[:qq]).all() and (r[1] == hop_np[:qq]).all())
    # a9: the literal walk with dead peers (every 100th peer dead, converged
    # 8-entry successor lists, DHash forwarding rule), same keys and sources
    alive = np.ones(N3, dtype=np.uint8)
    alive[::100] = 0
    ring.upload_liveness(alive=alive, ns=8, rule=chordx.CX_FWD_DHASH)
    tlit = ev_time(lambda: ring.route(src, keys, out=(owner, hops, status)))
    st_lit = status.cpu().numpy()
    own_l, hop_l = owner.cpu().numpy().view(np.uint32), hops.cpu().numpy()
    PL = O.Peers(ring_np, F_gpu, alive=alive, ns=8, rule=O.FWD_DHASH)
    cpu_lit = cpu_leg(lambda q, th: O.route(PL, src_np[:q], kq_np[:q], threads=th), q,
                      "lookups/s", "routed lookups with 1 % dead peers (or_route, DHash rule)",
                      lambda r, qq: (r[0] == own_l[:qq]).all() and (r[1] == hop_l[:qq]).all()
                      and (r[2] == st_lit[:qq]).all())
    a9 = {"route_s": tlit, "lookups_per_s": q / tlit, "dead_fraction": 0.01,
          "status_counts": {str(k): int((st_lit == k).sum()) for k in np.unique(st_lit)},
          "cpu": cpu_lit}
    del P, PL, F_gpu
    out["C3_a9_dead_peers"] = a9
    out["C3"] = {"fingers_build_s_wall": tf, "cpu_fingers": cpu_f, "cpu_route": cpu_r,
                 "fingers_algo_GBps": N3 * 528 / tf / 1e9,
                 "route_s": tr, "route_lookups_per_s": q / tr, "mean_hops": sh / q,
                 "route_algo_GBps": algo / tr / 1e9, "route_algo_frac_of_hbm": algo / tr / HBM,
                 "route_gathers_per_lookup": (g64 + r16 + 2 * xc) / q,
                 "bad_status": bad3}
    del ring, keys, src, owner, hops, status

    # ---------------- C5 ----------------
    N5, q5, n = 1 << 24, 1 << 26, 14
    old = chordx.Ring(keys_dev(N5, 0x5EED0007))
    keys = keys_dev(q5, 0x5EED0008)
    lists = torch.empty((q5, n), dtype=torch.int32, device="cuda")
    tl = ev_time(lambda: old.nsucc(keys, n), reps=2)
    joins = keys_dev(N5 // 100, 0x5EED0009)
    # distinct leaving peers (odd stride mod 2^24): the new ring keeps 2^24 peers
    pick = (torch.arange(N5 // 100, device="cuda", dtype=torch.int64) * 0x9E3779B1) % N5
    leaves = old.ids_device()[pick].contiguous()
    old.build_fingers()  # the live ring is route-ready when membership changes
    old.sync()
    tcv = {}
    for cv in (0, 1, 1):  # re-sort, merge (twice: the first call warms allocations)
        old.set_churn_variant(cv)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        new, o2n = old.churn(joins, leaves)
        torch.cuda.synchronize()
        tcv[cv] = time.perf_counter() - t0
    tc = tcv[1]
    tm = ev_time(lambda: old.misplaced(new, o2n, keys, n), reps=2)
    lists, count, mask, target = old.misplaced(new, o2n, keys, n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    new.build_fingers()
    new.sync()
    t_first = time.perf_counter() - t0  # fresh HBM for the new ring's 72 GiB of tables
    # steady state: the previous epoch's ring is gone (its tables in the pool)
    del new, o2n
    t0 = time.perf_counter()
    new, o2n = old.churn(joins, leaves)
    new.build_fingers()
    new.sync()
    t_cycle = time.perf_counter() - t0
    t_ready = t_cycle - tc
    old_np, new_np = old.ids(), new.ids()
    o2n_np = o2n.cpu().numpy().view(np.uint32) if hasattr(o2n, "cpu") else np.asarray(o2n)
    j_np = joins.cpu().numpy().view(np.uint64)
    l_np = leaves.cpu().numpy().view(np.uint64)
    t0 = time.perf_counter()
    want_new, want_o2n = O.churn(old_np, j_np, l_np)
    t_churn_cpu = time.perf_counter() - t0
    k5 = keys.cpu().numpy().view(np.uint64)
    lists_np = lists.cpu().numpy().view(np.uint32)
    mask_np = mask.cpu().numpy()
    cpu_m = cpu_leg(lambda qq, th: O.misplaced(old_np, new_np, o2n_np, k5[:qq], n, threads=th),
                    q5, "keys/s", "keys (RunGlobalMaintenance restated, n = 14)",
                    lambda r, qq: (r[0] == lists_np[:qq]).all() and (r[2] == mask_np[:qq]).all())
    out["C5"] = {"ring_old": N5, "ring_new": new.n, "keys": q5, "n": n,
                 "route_ready_after_churn_s_wall": t_cycle,
                 "new_fingers_and_route_table_s_wall": t_ready,
                 "first_fingers_and_route_table_s_wall_fresh_hbm": t_first,
                 "cpu_churn": {"value_s": t_churn_cpu, "cores": 1, "kind": "port",
                               "identical": bool((want_new == new_np).all()
                                                 and (want_o2n == o2n_np).all())},
                 "cpu_misplaced": cpu_m,
                 "nsucc_s": tl, "nsucc_keys_per_s": q5 / tl,
                 "churn_s_wall": tc, "churn_resort_s_wall": tcv[0],
                 "misplaced_s": tm, "misplaced_keys_per_s": q5 / tm,
                 "misplaced_algo_GBps": q5 * 139 / tm / 1e9,
                 "keys_with_misplaced_holder": int((mask != 0).sum()),
                 "misplaced_pairs": int(sum(int(((mask.to(torch.int32) >> j) & 1).sum())
                                            for j in range(n)))}
    del old, new, keys, lists, count, mask, target, joins, leaves, pick, o2n
    torch.cuda.empty_cache()

    # ---------------- f1 UUIDv5 IDs, f3 hex codec (device buffers) ----------------
    import ctypes
    import uuid
    from chordx import _lib as LL
    lib = chordx.lib()
    vp = ctypes.c_void_p
    nq = 1 << 22
    names = [f"127.0.0.1:{5000 + i}" if i % 2 else f"key{i}" for i in range(nq)]
    enc = "".join(names).encode()
    offs = np.zeros(nq + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in names])
    d_bytes = torch.from_numpy(np.frombuffer(enc, dtype=np.uint8).copy()).cuda()
    d_offs = torch.from_numpy(offs.view(np.int64)).cuda()
    d_ids = torch.empty((nq, 2), dtype=torch.int64, device="cuda")
    uu = lambda: LL.check(lib.cx_uuid5_dns(vp(d_bytes.data_ptr()), vp(d_offs.data_ptr()), nq,  # noqa: E731
                                           vp(d_ids.data_ptr()), LL.CX_MEM_DEVICE, 0))
    t_uuid = ev_time(uu)
    ids_np = d_ids.cpu().numpy().view(np.uint64)
    want = [uuid.uuid5(uuid.NAMESPACE_DNS, x).int for x in names[:4096]]
    ok_uuid = all(int(ids_np[i, 1]) << 64 | int(ids_np[i, 0]) == want[i] for i in range(4096))
    t0 = time.perf_counter()
    m1 = 200000
    for x in names[:m1]:
        uuid.uuid5(uuid.NAMESPACE_DNS, x)
    cpu_uuid = m1 / (time.perf_counter() - t0)
    # hex: format 2^24 keys to text, parse the text back (round trip on the GPU)
    nh = 1 << 24
    hk = keys_dev(nh, 0x5EED000A)
    txt = torch.empty((nh, 32), dtype=torch.uint8, device="cuda")
    ln = torch.empty(nh, dtype=torch.uint8, device="cuda")
    fm = lambda: LL.check(lib.cx_hex_format(vp(hk.data_ptr()), nh, vp(txt.data_ptr()),  # noqa: E731
                                            vp(ln.data_ptr()), LL.CX_MEM_DEVICE, 0))
    t_fmt = ev_time(fm)
    back = torch.empty((nh, 2), dtype=torch.int64, device="cuda")
    okb = torch.empty(nh, dtype=torch.uint8, device="cuda")
    # the strings (each slot's first len bytes), packed as the parser takes them
    packed_offs = torch.empty(nh + 1, dtype=torch.int64, device="cuda")
    packed_offs[0] = 0
    packed_offs[1:] = torch.cumsum(ln.to(torch.int64), 0)
    sel = (torch.arange(32, device="cuda")[None, :] < ln[:, None].to(torch.int64))
    packed = txt[sel].contiguous()
    pa = lambda: LL.check(lib.cx_hex_parse(vp(packed.data_ptr()), vp(packed_offs.data_ptr()), nh,  # noqa: E731
                                           vp(back.data_ptr()), vp(okb.data_ptr()),
                                           LL.CX_MEM_DEVICE, 0))
    t_parse = ev_time(pa)
    rt_ok = bool(torch.equal(back, hk)) and bool((okb == 1).all())
    t0 = time.perf_counter()
    hk_np = hk[:200000].cpu().numpy().view(np.uint64)
    for lo, hi in hk_np:
        int(format((int(hi) << 64) | int(lo), "x"), 16)
    cpu_hex = 200000 / (time.perf_counter() - t0)
    out["f1_uuid5_f3_hex"] = {
        "uuid5_names": nq, "uuid5_s": t_uuid, "uuid5_names_per_s": nq / t_uuid,
        "uuid5_matches_python_uuid5_on_4096": ok_uuid,
        "cpu_uuid5": {"value": cpu_uuid, "unit": "names/s", "cores": 1, "kind": "python stdlib",
                      "sample": f"first {m1} names, uuid.uuid5 (DNS namespace)"},
        "hex_keys": nh, "hex_format_s": t_fmt, "hex_format_keys_per_s": nh / t_fmt,
        "hex_parse_s": t_parse, "hex_parse_keys_per_s": nh / t_parse,
        "hex_round_trip_identical": rt_ok,
        "cpu_hex_round_trip": {"value": cpu_hex, "unit": "keys/s", "cores": 1,
                               "kind": "python format/int", "sample": "first 200000 keys"}}
    del d_bytes, d_offs, d_ids, hk, txt, ln, back, okb, packed, packed_offs, sel
    torch.cuda.empty_cache()

    # ---------------- IDA (DHash payload coding, 14/10/257) ----------------
    from chordx import ida
    res = {}
    for name, nb, bl in (("4KiB_blocks", 1 << 18, 4096), ("64B_blocks", 1 << 22, 64)):
        g = torch.Generator(device="cuda").manual_seed(1)
        data = torch.randint(0, 256, (nb * bl,), dtype=torch.uint8, device="cuda", generator=g)
        offs = torch.arange(0, nb * bl + 1, bl, dtype=torch.int64, device="cuda")
        frags, seg = ida.encode_flat(data, offs)
        te = ev_time(lambda: ida.encode_flat(data, offs, seg_offsets=seg, out=frags))
        S = (bl + 9) // 10
        keep = torch.tensor([0, 2, 3, 5, 6, 8, 9, 11, 12, 13], device="cuda")
        rows = frags.view(nb, 14, S)[:, keep, :].contiguous().view(-1)
        idx = (keep + 1).to(torch.uint8).repeat(nb).contiguous()
        dec = ida.decode_flat(rows, seg, idx)
        td = ev_time(lambda: ida.decode_flat(rows, seg, idx, out=dec))
        nbytes = nb * bl
        res[name] = {"bytes": nbytes, "encode_s": te, "encode_GBps_data": nbytes / te / 1e9,
                     "encode_algo_frac_of_hbm": nbytes * (1 + 2.8) / te / HBM,
                     "decode_s": td, "decode_GBps_data": nbytes / td / 1e9,
                     "decode_algo_frac_of_hbm": nbytes * (2 + 2) / td / HBM}
        del data, offs, frags, rows, idx, seg, dec
    out["IDA_14_10_257"] = res
    print(json.dumps(out))


if __name__ == "__main__":
    main()
