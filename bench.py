#!/usr/bin/env python3
"""Headline benchmark: finger-routed successor lookups with hop counts on a
2^24-peer Chord ring (BASELINE.json metric, config C4 per GPU).

One step = one cx_route launch over this rank's batch of keys resident in HBM
(the converged m=128 finger table, ring and Eytzinger copy are built before the
timed region).  Weak scaling: every rank holds a replica of the ring and routes
its own slice of the global key stream (keys[q] = splitmix(seed, q), src[q] =
q mod N), so the data path has no collective; the barrier and the max-over-ranks
timing are the only cross-rank traffic.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no torch.distributed environment, bench.py starts
`torch.distributed.run --nproc-per-node N` itself as a child process (before
anything touches the GPU) and exits with its status; rank 0 of the child job
prints the line.  Rank 0 prints ONE JSON line.

Roofline (per launch of the timed route kernel): `achieved` counts the bytes
the walk must move -- its streams (key, source, (pred, self) pair, owner, hops,
status) plus one 64-B granule per random gather it actually issues (window-table
entries, exact ring IDs, finger entries), counted by the counting build of the
same kernel on the same batch -- over the kernel time from HIP events on the
launch stream.  SURVEY 8(d)'s reference-work model (128 B per hop) is reported
separately as `reference_work_model`: it prices hops the window table resolves
without a gather and is not a byte count of this kernel.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "p2p-dhts_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import chordx  # noqa: E402
from chordx import dist  # noqa: E402

SEED_RING = 0x5EED0005
SEED_KEYS = 0x5EED0006
SEED_RANDOM_SRC = 0x5EED000A  # A/B field only: uniformly random source peers
HBM_PEAK = 8.0e12  # B/s per MI355X (MI355X_MICROARCH.md, HBM3E spec)
# Bytes the walk must move per lookup in streams: key 16 + source 4 +
# (pred, self) ID pair 32 + owner 4 + hops 1 + status 1.
BYTES_STREAM = 58
GRANULE = 64  # one dependent random gather
# SURVEY 8(d) reference-work model: 25 B streamed + 64 B source-peer record +
# 128 B per hop (finger granule + ring granule).
REF_STREAM, REF_SRC, REF_HOP = 25, 64, 128


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--peers-log2", type=int, default=24)
    ap.add_argument("--keys-log2", type=int, default=25, help="keys per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="target wall time of the CPU-oracle baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--mode", choices=("replicated", "arc"), default="replicated",
                    help="replicated: every rank holds the whole tree table and routes its "
                         "own keys (default); arc: each rank holds tree rows for its arc only "
                         "and lookups travel between ranks (chordx.arc)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_route.json"))
    return ap.parse_args()


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args):
    """One process per GPU.  Without a torch.distributed environment and with
    --gpus N > 1, run this script under torch.distributed.run as a CHILD
    process (nothing here has touched the GPU yet) and return its exit
    status; None = run the benchmark in this process."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus <= 1:
            return None
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
               f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
        return subprocess.run(cmd).returncode
    if int(ws) != args.gpus:
        print(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}", file=sys.stderr)
        return 2
    return None


def host_threads() -> int:
    """Host cores this process may use: its CPU affinity, capped by the
    job's thread budget (OMP_NUM_THREADS; 16 on a one-GPU box, whose nproc
    shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(ring, F_host, keys_np, src_np, gpu_owner, gpu_hops, budget_s):
    """Literal restatement (oracle/chord_oracle.c or_route: linear 128-entry
    InBetween scan per hop, StoredLocally, ForwardRequest substitution) timed on
    this host's cores over a bounded sample of the same key stream (about
    2/3 of budget_s on all usable cores, 1/3 on one core); also checks the
    GPU's owner/hops on the sample."""
    import oracle as O

    threads = host_threads()
    ring_np = ring.ids()
    P = O.Peers(ring_np, F_host)

    def timed(q, th):
        t0 = time.perf_counter()
        r = O.route(P, src_np[:q], keys_np[:q], threads=th)
        return r, time.perf_counter() - t0

    _, t_cal = timed(4096, 1)
    per1 = t_cal / 4096
    q1 = int(min(len(keys_np), max(4096, budget_s / 3 / max(per1, 1e-9))))
    _, dt1 = timed(q1, 1)
    qa = int(min(len(keys_np), max(q1, budget_s * 2 / 3 * threads / max(per1, 1e-9))))
    (wo, wh, ws), dta = timed(qa, threads)
    ok = bool((wo == gpu_owner[:qa]).all() and (wh == gpu_hops[:qa]).all() and (ws == 0).all())
    return {"value": qa / dta, "unit": "lookups/s", "cores": threads, "kind": "port",
            "value_1core": q1 / dt1,
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "sample": f"first {qa} keys of the rank-0 stream (of {len(keys_np)}) on {threads} "
                      f"threads ({dta:.1f} s), first {q1} on 1 thread ({dt1:.1f} s); "
                      "oracle/chord_oracle.c or_route, gcc -O3 -march=x86-64-v3",
            "parity_on_sample": ok}


def dry_run(args):
    """CX_BENCH_DRYRUN=1: the launch / rendezvous / timing / reporting flow
    without a GPU (CPU tests of the N > 1 path over gloo)."""
    world, rank, _ = dist.env_rank()
    dist.init("gloo")
    dist.barrier(world)
    t0 = time.perf_counter()
    dist.barrier(world)
    dt_max = dist.max_over_ranks(time.perf_counter() - t0, world)
    if rank == 0:
        print(json.dumps({"metric": "dry run", "value": 0.0, "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": dt_max * 1e3 / max(1, args.steps)}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main_arc(args):
    """Arc-sharded layout (SURVEY 8e layout 2): ring IDs generated in shares
    and all-gathered (RCCL), route planes per arc, lookups sent to their key's
    arc and answered in the key-first structure-of-arrays protocol
    (ArcRouter.route_soa: 20 B out, 8 B back per lookup, pipelined pieces)."""
    from chordx.arc import ArcRouter
    world, rank, local = dist.env_rank()
    local = local % max(1, torch.cuda.device_count())  # rehearsal: ranks share a GPU
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    backend = os.environ.get("CX_DIST_BACKEND", "nccl")
    dist.init(backend, dev)
    N = 1 << args.peers_log2
    Q = 1 << args.keys_log2
    lo, hi = rank * N // world, (rank + 1) * N // world
    t0 = time.perf_counter()
    share = torch.empty((N // world, 2), dtype=torch.int64, device=dev)
    assert N % world == 0
    chordx.fill_splitmix(share, SEED_RING, offset=lo)
    if world > 1:
        cd = torch.device("cpu") if backend == "gloo" else dev
        ids = torch.empty((N, 2), dtype=torch.int64, device=cd)
        torch.distributed.all_gather_into_tensor(ids, share.to(cd))
        ids = ids.to(dev)
    else:
        ids = share
    ring = chordx.Ring(ids, device=local)
    del ids, share
    router = ArcRouter(ring, ring.n, rank, world,
                       comm_device="cpu" if backend == "gloo" else None)
    torch.cuda.synchronize(dev)
    t_setup = time.perf_counter() - t0
    keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    q0, q1 = dist.shard(rank, Q)
    chordx.fill_splitmix(keys, SEED_KEYS, offset=q0)
    src = (torch.arange(q0, q1, device=dev, dtype=torch.int64) % ring.n).to(torch.int32)
    owner = torch.empty(Q, dtype=torch.int32, device=dev)
    hops = torch.empty(Q, dtype=torch.uint8, device=dev)
    status = torch.empty(Q, dtype=torch.uint8, device=dev)
    for _ in range(args.warmup):
        router.route(src, keys, owner, hops, status)
    torch.cuda.synchronize(dev)
    router.records_sent = 0
    dist.barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rounds = router.route(src, keys, owner, hops, status)
    torch.cuda.synchronize(dev)
    dist.barrier(world)
    dt = time.perf_counter() - t0
    dt_max = dist.max_over_ranks(dt, world, dev)
    bad = dist.sum_over_ranks(int((status != 0).sum().item()), world, dev)
    sent = dist.sum_over_ranks(router.records_sent, world, dev)
    sum_hops = dist.sum_over_ranks(int(hops.to(torch.int64).sum().item()), world, dev)
    succ = ring.successor(keys)  # exact successor (directory search) of every key
    mismatch = dist.sum_over_ranks(int((succ != owner).sum().item()), world, dev)
    if rank == 0:
        total = world * Q * args.steps
        line = {
            "metric": "successor lookups/sec (whole node) + % HBM roofline, 2^24-peer ring, "
                      "1/2/4/8 GPUs",
            "value": total / dt_max,
            "unit": "lookups/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u128",
            "data": "synthetic",
            "config": {"workload": "C4 finger-routed lookups with hop counts, arc-sharded: "
                                   f"2^{args.peers_log2}-peer ring, 2^{args.keys_log2} keys/GPU/step",
                       "peers": N, "keys_per_gpu": Q, "global_batch": world * Q,
                       "parallelism": f"arc-sharded route planes x{world}, key-first SoA "
                                      "all_to_all (20 B out, 8 B back per lookup)"},
            "rounds_per_step": rounds,
            "records_exchanged_per_lookup": sent / (world * Q * args.steps),
            "mean_hops": sum_hops / (world * Q),
            "bad_status": bad,
            "route_owner_equals_successor": mismatch == 0,
            "setup_s": t_setup,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    rc = launch(args)
    if rc is not None:
        sys.exit(rc)
    if os.environ.get("CX_BENCH_DRYRUN") == "1":
        return dry_run(args)
    if args.mode == "arc":
        return main_arc(args)
    world, rank, local = dist.env_rank()
    # one rank per GPU; CX_DIST_BACKEND=gloo with more ranks than GPUs is the
    # rehearsal of the N > 1 flow on a one-GPU box (ranks share devices)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    dist.init(os.environ.get("CX_DIST_BACKEND", "nccl"), dev)
    N = 1 << args.peers_log2
    Q = 1 << args.keys_log2

    # ---- setup (untimed): ring, Eytzinger copy, converged finger table ----
    ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(ids, SEED_RING)
    t0 = time.perf_counter()
    ring = chordx.Ring(ids, device=local)
    torch.cuda.synchronize(dev)
    t_ring = time.perf_counter() - t0
    del ids
    t0 = time.perf_counter()
    ring.build_fingers()
    ring.sync()
    t_fing = time.perf_counter() - t0
    keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    q0, q1 = dist.shard(rank, Q)
    chordx.fill_splitmix(keys, SEED_KEYS, offset=q0)
    gq = torch.arange(q0, q1, device=dev, dtype=torch.int64)
    src = (gq % ring.n).to(torch.int32)
    del gq
    owner = torch.empty(Q, dtype=torch.int32, device=dev)
    hops = torch.empty(Q, dtype=torch.uint8, device=dev)
    status = torch.empty(Q, dtype=torch.uint8, device=dev)
    out = (owner, hops, status)

    route_variant, cz_escapes, table_bytes = ring.route_info()
    kernel_name = {5: "k_route_tree<false, true>", 4: "k_route_tree<false, false>"}.get(
        route_variant, f"route variant {route_variant}")

    # ---- warmup ----
    for _ in range(args.warmup):
        ring.route(src, keys, out=out)
    torch.cuda.synchronize(dev)

    # ---- timed: exactly K steps, barrier + sync on both sides ----
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dist.barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        ring.route(src, keys, out=out)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    dist.barrier(world)
    dt = time.perf_counter() - t0
    dt_max = dist.max_over_ranks(dt, world, dev)
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # one cx_route launch per step

    # ---- results ----
    bad = dist.sum_over_ranks(int((status != 0).sum().item()), world, dev)
    sum_hops = int(hops.to(torch.int64).sum().item())
    # gathers the walk issues on this batch: the counting build of the same
    # kernel, run once after the timed region (same inputs, same outputs)
    ring.route_counters(True)
    ring.route(src, keys, out=out)
    g64, r16, xc, nq = ring.route_counters(False)
    gathers = g64 + r16 + 2 * xc
    algo_bytes = Q * BYTES_STREAM + GRANULE * gathers
    achieved = algo_bytes / (kern_ms * 1e-3)
    ref_bytes = Q * (REF_STREAM + REF_SRC) + REF_HOP * sum_hops
    probe = ring.gather_probe()  # request-rate ceiling on this table, this box, this run
    # exact-successor rate on the same keys (row a5, C2 kernel at C4 size)
    succ_out = torch.empty(Q, dtype=torch.int32, device=dev)
    ring.successor(keys, out=succ_out)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(3):
        ring.successor(keys, out=succ_out)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    succ_ms = e0.elapsed_time(e1) / 3
    owner_eq = bool((succ_out == owner).all().item())
    ring.set_search_variant(0)  # A/B: Eytzinger search with LDS top levels
    ring.successor(keys, out=succ_out)
    e0.record(stream)
    for _ in range(3):
        ring.successor(keys, out=succ_out)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    eyt_ms = e0.elapsed_time(e1) / 3
    owner_eq = owner_eq and bool((succ_out == owner).all().item())
    ring.set_search_variant(2)  # A/B: wave-cooperative 16-ary tree (ballot + popcount)
    ring.successor(keys, out=succ_out)
    e0.record(stream)
    for _ in range(3):
        ring.successor(keys, out=succ_out)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wave_ms = e0.elapsed_time(e1) / 3
    owner_eq = owner_eq and bool((succ_out == owner).all().item())
    ring.set_search_variant(1)
    # A/B: the other route kernels on the same batch (bit-identical results)
    variant_ms = {}
    for v in (0, 1, 2, 3, 4, 5):
        ring.set_route_variant(v)
        ring.route(src, keys, out=out)
        e0.record(stream)
        for _ in range(3):
            ring.route(src, keys, out=out)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        variant_ms[v] = e0.elapsed_time(e1) / 3
    ring.set_route_variant(-1)
    # A/B: the same keys from uniformly random source peers (C4 fixes src = q mod N,
    # whose wave-adjacent sources share lines on the first gathers); owners must not change
    rsrc = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(rsrc, SEED_RANDOM_SRC, offset=q0)
    rsrc = (rsrc[:, 0] & 0x7FFFFFFFFFFFFFFF).remainder(ring.n).to(torch.int32)
    rout = (torch.empty_like(owner), torch.empty_like(hops), torch.empty_like(status))
    ring.route(rsrc, keys, out=rout)  # own buffers: owner/hops stay the timed run's
    e0.record(stream)
    for _ in range(3):
        ring.route(rsrc, keys, out=rout)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    rsrc_ms = e0.elapsed_time(e1) / 3
    owner_eq = owner_eq and bool((succ_out == rout[0]).all().item())
    rsrc_bad = int((rout[2] != 0).sum().item())
    del rsrc, rout

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        F_host = np.empty((ring.n, chordx.CX_FINGERS), dtype=np.uint32)
        F_host[:] = ring.fingers_device().cpu().numpy().view(np.uint32)
        cs = Q  # the sample is sized by --cpu-seconds inside cpu_baseline
        cpu = cpu_baseline(ring, F_host, keys[:cs].cpu().numpy().view(np.uint64),
                           src[:cs].cpu().numpy().view(np.uint32),
                           owner[:cs].cpu().numpy().view(np.uint32),
                           hops[:cs].cpu().numpy(), args.cpu_seconds)
        del F_host

    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if tj.get("peers") == N and tj.get("keys") == Q and tj.get("kernel") == kernel_name:
            traffic = tj.get("hbm_bytes_per_launch")
    req = gathers / (kern_ms * 1e-3)
    gather = {"requests_per_s": req, "ceiling": probe, "frac": req / probe,
              "gathers_per_lookup": gathers / Q, "table_gathers": g64, "exact_id_gathers": r16,
              "exact_hops": xc,
              "note": "random 64-B requests the walk issued (counting build, same batch) per "
                      "second of kernel time, vs dependent quad-cooperative 64-B gathers/s "
                      "measured on the same route table in this run"}

    if rank == 0:
        total = world * Q * args.steps
        line = {
            "metric": "successor lookups/sec (whole node) + % HBM roofline, 2^24-peer ring, "
                      "1/2/4/8 GPUs",
            "value": total / dt_max,
            "unit": "lookups/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u128",
            "data": "synthetic",
            "config": {"workload": "C4 finger-routed lookups with hop counts (per GPU): "
                                   f"2^{args.peers_log2}-peer ring, 2^{args.keys_log2} keys/GPU/step, "
                                   "src = q mod N, splitmix seeds 0x5EED0005/0x5EED0006",
                       "peers": N, "keys_per_gpu": Q, "global_batch": world * Q,
                       "parallelism": f"replicated ring, keys sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK, "traffic": traffic,
                         "kernel": kernel_name, "kernel_ms": kern_ms,
                         "algo_bytes_per_launch": algo_bytes,
                         "algo_model": f"{BYTES_STREAM} B streams per lookup + {GRANULE} B per "
                                       "random gather issued (counted)"},
            "reference_work_model": {"bytes_per_launch": ref_bytes,
                                     "GBps": ref_bytes / (kern_ms * 1e-3) / 1e9,
                                     "note": "SURVEY 8(d): 128 B per hop; hops the window "
                                             "table resolves without a gather are priced too, "
                                             "so this is not a byte count of the kernel"},
            "cpu_baseline": cpu,
            "gather_roofline": gather,
            "route_variant": route_variant,
            "route_table_bytes": table_bytes,
            "route_cz_escapes": cz_escapes,
            "mean_hops": sum_hops / Q,
            "bad_status": bad,
            "route_owner_equals_successor": owner_eq,
            "exact_successor_lookups_per_s": Q / (succ_ms * 1e-3),
            "exact_successor_eytzinger_lookups_per_s": Q / (eyt_ms * 1e-3),
            "exact_successor_wave16_lookups_per_s": Q / (wave_ms * 1e-3),
            "route_variant_kernel_ms": variant_ms,
            "route_random_src": {"kernel_ms": rsrc_ms, "lookups_per_s": Q / (rsrc_ms * 1e-3),
                                 "bad_status": rsrc_bad,
                                 "note": "same keys and kernel, src uniform in [0, N) "
                                         "(splitmix 0x5EED000A) instead of q mod N"},
            "setup_s": {"ring_sort": t_ring, "fingers_build": t_fing},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
