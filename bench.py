#!/usr/bin/env python3
"""Headline benchmark: finger-routed successor lookups with hop counts on a
2^24-peer Chord ring (BASELINE.json metric, config C4).

One step = one cx_route launch over this rank's batch of keys resident in HBM
(the converged m=128 finger table, ring and route table are built before the
timed region).  Every rank generates its share of the ring IDs and one
all_gather (RCCL over xGMI) replicates them; every rank then holds a replica of
the ring and routes its own slice of the global key stream (keys[q] =
splitmix(seed, q), src[q] = q mod N): weak scaling, no collective in the timed
data path, the barrier and the max-over-ranks timing are the only cross-rank
traffic.  After the timed region the same run measures, on every rank:

  arc      C4 as BASELINE.json states it -- the ring sharded by key arc, each
           rank holding route rows for its arc only, lookups exchanged with
           all_to_all-v (chordx.arc.ArcRouter, key-first SoA protocol) -- timed
           over the same number of steps on the same keys, results compared
           with the replicated route;
  churn    1 % joins + 1 % leaves of the bench ring (seed 0x5EED0009) ->
           route-ready (merge churn + fingers + route table), cold (fresh HBM)
           then warm (table pool), with the two tables' hashes compared and
           each epoch's allocation path (fresh / pooled bytes, trims,
           retries); then the 28- against the 32-level table in ABBA order;
  cpu      the reference-faithful CPU walk (oracle/, rank 0, every world size),
           with the hop histogram of its sample;
  c5       BASELINE config C5 (DHash n = 14 lists + misplaced scan of 2^26 keys
           after a 1 %/1 % churn of a second 2^24 ring), after the bench ring
           is closed: one cx_dhash_maintenance pass per step, keys sharded
           over ranks (strong scaling), parity against the oracle on a sample.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no torch.distributed environment, bench.py starts
`torch.distributed.run --nproc-per-node N` itself as a child process (before
anything touches the GPU) and exits with its status; rank 0 of the child job
prints the ONE JSON line.

Roofline (whole node): `achieved` = the algorithmic bytes of the timed route
kernel summed over ranks -- its streams (key, source, (pred, self) pair,
owner, hops, status) plus one 64-B granule per random gather it actually
issues, counted by the counting build of the same kernel on the same batch --
over the slowest rank's kernel time (HIP events on the launch stream); `peak`
= 8 TB/s x N.  SURVEY 8(d)'s reference-work model (128 B per hop) is reported
separately as `reference_work_model`: it prices hops the window table resolves
without a gather and is not a byte count of this kernel.
"""
from __future__ import annotations

import argparse
import json
import os
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

METRIC = "successor lookups/sec (whole node) + % HBM roofline, 2^24-peer ring, 1/2/4/8 GPUs"
SEED_RING = 0x5EED0005
SEED_KEYS = 0x5EED0006
SEED_CHURN = 0x5EED0009    # C5's churn batch seed
SEED_RANDOM_SRC = 0x5EED000A  # A/B field only: uniformly random source peers
HBM_PEAK = 8.0e12  # B/s per MI355X (MI355X_MICROARCH.md, HBM3E spec)
# Bytes the walk must move per lookup in streams: key 16 + source 4 +
# (pred, self) ID pair 32 + owner 4 + hops 1 + status 1.
BYTES_STREAM = 58
GRANULE = 64  # one dependent random gather
# SURVEY 8(d) reference-work model: 25 B streamed + 64 B source-peer record +
# 128 B per hop (finger granule + ring granule).
REF_STREAM, REF_SRC, REF_HOP = 25, 64, 128
# C2 / C3 (configs[1], configs[2]): SURVEY 8(d) seeds
SEED_C2_RING, SEED_C2_KEYS = 0x5EED0001, 0x5EED0002
SEED_C3_RING, SEED_C3_KEYS = 0x5EED0003, 0x5EED0004
CX_FINGERS_B = 128
# C5 (configs[4]): a second ring and key stream (SURVEY 8d seeds)
SEED_C5_RING, SEED_C5_KEYS = 0x5EED0007, 0x5EED0008
C5_N = 14
# cx_dhash_maintenance per key: key 16 + one 64-B search line + old 14-list 56
# + count 1 + new 14-list 56 + count 1 + mask 2 + targets 14
C5_BYTES_STREAM = 210
# SURVEY 8(d)'s DHash model: 16 + 64 + 56 + 1 + 2 per key
C5_BYTES_SURVEY = 139


def dir_search_requests(ids, keys, k, want_index=False):
    """Random memory requests of the exact successor search over the bucket
    directory (cx_common.hpp dir_successor, the kernel cx_successor runs on a
    ring too large for the LDS slice table): one 16-B directory entry per key,
    plus the ring IDs (16 B each) that the in-bucket binary search reads when
    the entry alone does not decide -- replayed exactly on the host from the
    sorted ring and the keys (uint64 (n, 2) / (q, 2) arrays {lo, hi}; k = the
    directory's bucket bits, 0 < k < 64).  Returns (directory entries, ring
    reads) and, with want_index, the successor index the replay reaches (the
    test checks it against the oracle)."""
    k = int(k)
    sh, kk = np.uint64(64 - k), np.uint64(k)
    hr, lr = ids[:, 1], ids[:, 0]
    hk, lk = keys[:, 1], keys[:, 0]
    bk = hk >> sh
    br = hr >> sh
    lo = np.searchsorted(br, bk, side="left")
    hi = np.searchsorted(br, bk, side="right")
    n = len(ids)
    nonempty = lo < hi
    loc = np.minimum(lo, n - 1)
    frac = (hr[loc] << kk) | (lr[loc] >> sh)
    xf = (hk << kk) | (lk >> sh)
    search = nonempty & ~(xf < frac) & ~((xf > frac) & (hi - lo == 1))
    a = np.where(xf > frac, lo + 1, lo).astype(np.int64)
    z = hi.astype(np.int64)
    ans = np.where(~nonempty | (xf < frac), lo, hi).astype(np.int64)
    idx = np.nonzero(search)[0]
    a, z = a[idx], z[idx]
    xh, xl = hk[idx], lk[idx]
    reads = 0
    while True:
        act = a < z
        cnt = int(act.sum())
        if cnt == 0:
            break
        reads += cnt
        m = (a + z) // 2
        mm = np.minimum(m, n - 1)
        lt = (hr[mm] < xh) | ((hr[mm] == xh) & (lr[mm] < xl))
        a = np.where(act & lt, m + 1, a)
        z = np.where(act & ~lt, m, z)
    ans[idx] = a
    if want_index:
        return len(keys), reads, np.where(ans == n, 0, ans)
    return len(keys), reads


def exact_successor_record(ring, keys, succ, ms, world, dev, sample=1 << 22):
    """The exact successor search of the bench batch (north_star's
    "exact successor lookups/sec"): its rate, and its roofline on a request
    model -- 16 B key + 4 B owner per lookup and 64 B per random request (the
    directory entry, and the ring IDs of the in-bucket binary search), the
    requests per key replayed on the host over the first `sample` keys
    (dir_search_requests; its answers must equal the GPU's, else no model)."""
    q = keys.shape[0]
    m = min(q, sample)
    n = ring.n
    k = 1
    while (1 << k) < n:
        k += 1
    k = min(k + 1, 29)  # cx_api.hip build_search: ceil(log2 n) + 1 bucket bits
    ks = keys[:m].cpu().numpy().view(np.uint64)
    d, r, ans = dir_search_requests(ring.ids(), ks, k, want_index=True)
    same = bool((ans.astype(np.uint32) == succ[:m].cpu().numpy().view(np.uint32)).all())
    same = dist.all_over_ranks(same, world, dev)
    per_key = (d + r) / m
    algo = q * (20 + GRANULE * per_key)
    achieved = dist.sum_over_ranks(int(algo), world, dev) / (dist.max_over_ranks(ms, world, dev) * 1e-3)
    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic_successor.json")
    if os.path.exists(tf) and n == 1 << 24 and q == 1 << 25:
        with open(tf) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    return {"lookups_per_s": world * q / (dist.max_over_ranks(ms, world, dev) * 1e-3),
            "kernel_ms": ms, "kernel": "k_successor<true, false> (bucket directory)",
            "traffic": None if traffic is None else traffic * world,
            "traffic_note": "PMC FETCH_SIZE + WRITE_SIZE per launch on one GPU "
                            "(profiles/traffic_successor.json) x N",
            "requests_per_key": per_key if same else None,
            "ring_reads_per_key": r / m if same else None,
            "model_replay_equals_gpu": same, "model_sample_keys": m,
            "requests_per_s": world * q * per_key / (dist.max_over_ranks(ms, world, dev) * 1e-3),
            "roofline": None if not same else {
                "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK * world / 1e9,
                "achieved": achieved / 1e9, "frac": achieved / (HBM_PEAK * world),
                "model": "16 B key + 4 B owner per lookup + 64 B per random request (one "
                         "directory entry per key, plus the ring IDs the in-bucket binary search "
                         "reads, replayed on the host); whole node over the slowest rank"}}


class LegGuard:
    """A watchdog per sub-record leg, on every rank.  The headline is measured
    and its line assembled before the legs run; if a leg does not finish in
    its limit (a collective that never completes on a new node, say), rank 0
    prints the line as it stands -- the leg's key null, the leg named in
    `legs_aborted` -- and every rank leaves with os._exit(0) after its own
    limit, so a hung sub-record costs its record, not the headline.  Limits
    are several times a leg's duration on a one-GPU box."""

    def __init__(self, rank: int):
        self.rank = rank
        self.line = None  # rank 0: the line so far
        self.timer = None

    def start(self, name: str, seconds: float) -> None:
        import threading
        self.stop()
        self.timer = threading.Timer(seconds, self._expire, (name, seconds))
        self.timer.daemon = True
        self.timer.start()

    def stop(self) -> None:
        if self.timer is not None:
            self.timer.cancel()
            self.timer = None

    def run(self, name: str, fn):
        """fn() under the watchdog; a leg that raises on this rank (an RCCL
        error on a new node, say) ends the run like a hung one: rank 0 prints
        the line as it stands with the leg and its error in `legs_failed`;
        every rank leaves with status 0 at once (ranks waiting for it in a
        collective leave when their own watchdog fires), so the launcher never
        tears rank 0 down before its line is out."""
        self.start(name, LEG_LIMIT_S)
        try:
            if os.environ.get("CX_BENCH_FAIL_LEG") == name:  # the failure path's own test
                raise RuntimeError(f"injected failure in leg {name!r}")
            return fn()
        except Exception as e:  # noqa: BLE001 -- reported in the line, then exit
            self.stop()
            progress(f"leg {name!r} failed: {type(e).__name__}: {e}")
            if self.rank == 0 and self.line is not None:
                self.line.setdefault("legs_failed", []).append(
                    {"leg": name, "error": f"{type(e).__name__}: {e}"[:500],
                     "note": "the keys of this and later legs are null"})
                print(json.dumps(self.line), flush=True)
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(0 if self.line is not None or self.rank != 0 else 3)

    def _expire(self, name: str, seconds: float) -> None:
        progress(f"leg {name!r} did not finish in {seconds:.0f} s: leaving")
        if self.rank == 0 and self.line is not None:
            self.line.setdefault("legs_aborted", []).append(
                {"leg": name, "limit_s": seconds,
                 "note": "watchdog: the leg did not finish; the keys of this and later legs "
                         "are null"})
            print(json.dumps(self.line), flush=True)
        os._exit(0 if self.line is not None or self.rank != 0 else 3)


# per-leg limit; CX_BENCH_LEG_LIMIT_S overrides it (the watchdog's own test)
LEG_LIMIT_S = float(os.environ.get("CX_BENCH_LEG_LIMIT_S", "300"))


def progress(msg: str) -> None:
    """One line on stderr per leg (the JSON line alone goes to stdout): long
    multi-rank runs show they are alive."""
    print(f"[bench r{os.environ.get('RANK', '0')} {time.strftime('%H:%M:%S')}] {msg}",
          file=sys.stderr, flush=True)


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
    ap.add_argument("--no-arc", action="store_true", help="skip the arc-sharded sub-record")
    ap.add_argument("--no-churn", action="store_true", help="skip the churn -> route-ready leg")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 DHash maintenance leg")
    ap.add_argument("--c5-keys-log2", type=int, default=26, help="C5 keys (all ranks)")
    ap.add_argument("--c5-oracle-keys", type=int, default=1 << 20,
                    help="C5 keys checked against the oracle (rank 0)")
    ap.add_argument("--c5-cpu-keys", type=int, default=1 << 17,
                    help="C5 CPU baseline: largest key sample (routed lists, rank 0; 0 = skip)")
    ap.add_argument("--c5-cpu-seconds", type=float, default=8.0)
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 exact-successor leg")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 fingers + routes leg")
    ap.add_argument("--mode", choices=("replicated", "arc"), default="replicated",
                    help="replicated: every rank holds the whole route table and routes its "
                         "own keys (default; the arc layout is still measured as the `arc` "
                         "sub-record); arc: the arc-sharded layout is the headline value")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_route.json"))
    return ap.parse_args()


def launch(args):
    """One process per GPU.  Without a torch.distributed environment and with
    --gpus N > 1, run this script under torch.distributed.run as a CHILD
    process (nothing here has touched the GPU yet) and return its exit
    status; None = run the benchmark in this process."""
    return dist.launch_self(args.gpus, __file__, sys.argv[1:])


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


def cpu_baseline(ring_np, F_host, keys_np, src_np, gpu_owner, gpu_hops, budget_s, world):
    """Literal restatement (oracle/chord_oracle.c or_route: linear 128-entry
    InBetween scan per hop, StoredLocally, ForwardRequest substitution) timed on
    this host's cores over a bounded sample of rank 0's key stream (about
    2/3 of budget_s on all usable cores, 1/3 on one core); also checks the
    GPU's owner/hops on the sample (gpu_owner None: no GPU outputs, dry run).
    Run on rank 0 after the timed region at every world size: the CPU path is
    one host's, so it is reported next to the whole-node GPU value."""
    import oracle as O

    threads = host_threads()
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
    ok = hist_ok = None
    hist = np.bincount(wh, minlength=1).tolist()
    if gpu_owner is not None:
        ok = bool((wo == gpu_owner[:qa]).all() and (wh == gpu_hops[:qa]).all() and (ws == 0).all())
        hist_ok = hist == np.bincount(gpu_hops[:qa], minlength=1).tolist()
    return {"value": qa / dta, "unit": "lookups/s", "cores": threads, "kind": "port",
            "hops_hist": hist, "hist_equal": hist_ok,
            "value_1core": q1 / dt1,
            "cpu_model": cpu_model(), "nproc": os.cpu_count(),
            "n_gpus_beside": world,
            "sample": f"first {qa} keys of the rank-0 stream (of {len(keys_np)}) on {threads} "
                      f"threads ({dta:.1f} s), first {q1} on 1 thread ({dt1:.1f} s); "
                      "oracle/chord_oracle.c or_route, gcc -O3 -march=x86-64-v3",
            "cores_note": "threads = this process's CPU affinity capped by OMP_NUM_THREADS, the "
                          "job's share of the host (nproc counts the whole machine); the walk "
                          "scales linearly in threads (value / value_1core)",
            "parity_on_sample": ok}


def whole_node_roofline(algo_bytes, kern_ms, world, dev):
    """Sum over ranks of the kernel's algorithmic bytes per launch over the
    slowest rank's kernel time, against N x 8 TB/s."""
    total = dist.sum_over_ranks(int(algo_bytes), world, dev)
    ms = dist.max_over_ranks(float(kern_ms), world, dev)
    achieved = total / (ms * 1e-3) if ms > 0 else 0.0
    peak = HBM_PEAK * world
    return {"bound": "hbm", "achieved": achieved / 1e9, "peak": peak / 1e9, "unit": "GB/s",
            "frac": achieved / peak, "algo_bytes_per_launch": total, "kernel_ms": ms,
            "n_gpus": world}


def line_base(args, world, value, dt_max, config, dtype="u128"):
    return {"metric": METRIC, "value": value, "unit": "lookups/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt_max * 1e3 / max(1, args.steps), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": "synthetic",
            "config": config}


def dry_run(args):
    """CX_BENCH_DRYRUN=1: the launch / rendezvous / timing / reduction /
    reporting flow without a GPU (CPU tests of the N > 1 path over gloo): a
    2^12-peer ring, the whole-node roofline reduction fed with zero bytes, and
    the CPU baseline on rank 0 at every world size, as in the GPU run."""
    world, rank, _ = dist.env_rank()
    dist.init("gloo")
    dist.barrier(world)
    t0 = time.perf_counter()
    dist.barrier(world)
    dt_max = dist.max_over_ranks(time.perf_counter() - t0, world)
    roof = whole_node_roofline(0, 1.0, world, None)
    cpu = None
    if rank == 0 and not args.no_cpu:
        import oracle as O
        ring_np = O.ring_build(O.splitmix_keys(SEED_RING, 1 << 12))
        F = O.fingers(ring_np, threads=2)
        keys_np = O.splitmix_keys(SEED_KEYS, 1 << 14)
        src_np = (np.arange(1 << 14) % len(ring_np)).astype(np.uint32)
        cpu = cpu_baseline(ring_np, F, keys_np, src_np, None, None, args.cpu_seconds, world)
    dist.barrier(world)
    if rank == 0:
        line = line_base(args, world, 0.0, dt_max, {"workload": "dry run"})
        line.update({"metric": "dry run", "roofline": roof, "cpu_baseline": cpu,
                     "arc": {"skipped": "dry run: no GPU"}})
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def setup_ring(args, world, rank, dev, backend):
    """Ring IDs generated in shares and all-gathered, then the ring handle."""
    N = 1 << args.peers_log2
    assert N % world == 0
    lo = rank * N // world
    share = torch.empty((N // world, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(share, SEED_RING, offset=lo)
    t0 = time.perf_counter()
    ids = dist.gather_ids(share, world, backend)
    torch.cuda.synchronize(dev)
    t_gather = time.perf_counter() - t0
    t0 = time.perf_counter()
    ring = chordx.Ring(ids, device=dev.index or 0)
    torch.cuda.synchronize(dev)
    t_ring = time.perf_counter() - t0
    setup_ring.sort_roofline = sort_roofline(ids)
    return ring, t_gather, t_ring


# Ring sort byte models per key (16-B ID + 4-B index tag).  LSD, per pass:
# histogram 16 + scatter 20 in / 20 out = 56.  MSD (round 6) at 2^24 keys:
# two such passes over the top bytes, the bucket bounds (the high word, 8) and
# the LDS bucket sort (20 in / 20 out): 2 x 56 + 8 + 40 = 160.
SORT_LSD_PASS_BYTES = 56
SORT_MSD_BYTES = 2 * SORT_LSD_PASS_BYTES + 8 + 40


def sort_roofline(ids):
    """cx_ring_create's (ID, index) sort of the bench's unsorted ring IDs, both
    variants timed with HIP events (chordx.ring.sort_time), against HBM."""
    from chordx.ring import sort_time
    n = ids.shape[0]
    out = {}
    for name, v, by in (("msd_buckets", 0, SORT_MSD_BYTES), ("lsd_16_pass", 1, 16 * SORT_LSD_PASS_BYTES)):
        ms = []
        ok = True
        for _ in range(3):
            t, good = sort_time(ids, v)
            ms.append(t)
            ok = ok and good
        t = sorted(ms)[1]
        out[name] = {"ms": t, "bytes": by * n, "GBps": by * n / (t * 1e-3) / 1e9,
                     "frac": by * n / (t * 1e-3) / HBM_PEAK, "sorted": ok,
                     "passes": 4 if v == 0 else 16}
    out["keys"] = n
    out["speedup"] = out["lsd_16_pass"]["ms"] / out["msd_buckets"]["ms"]
    out["note"] = ("ms = the sort alone (HIP events, median of 3); bytes: MSD 160 B per key "
                   "(two top-byte passes of 56, bucket bounds 8, LDS bucket sort 40), LSD 56 B "
                   "per key per pass x 16; "
                   "the default is MSD with the LSD sort (4 tag + 16 key passes) as the "
                   "fallback for a bucket above 2048 keys")
    return out


def time_steps(fn, steps, world, dev):
    """Exactly `steps` calls bracketed by barrier + synchronize on both sides;
    (wall seconds of this rank, max over ranks)."""
    dist.barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize(dev)
    dist.barrier(world)
    dt = time.perf_counter() - t0
    return dt, dist.max_over_ranks(dt, world, dev)


def arc_leg(args, ring, src, keys, owner_ref, hops_ref, world, rank, dev, backend):
    """C4 as BASELINE.json states it: arc-sharded route planes and lookups
    exchanged with all_to_all-v, over the same keys and steps as the headline;
    owners/hops/statuses must equal the replicated route's."""
    from chordx.arc import ArcRouter
    Q = keys.shape[0]
    t0 = time.perf_counter()
    # N = 1: a one-rank group (RCCL) and exchange_always, so the leg runs and
    # times the general path -- partition, exchange, walk, exchange back,
    # delivery -- that N ranks run, not the in-place walk
    single = world == 1 and dist.init_single(backend, dev if backend == "nccl" else None)
    router = ArcRouter(ring, ring.n, rank, world,
                       comm_device="cpu" if backend == "gloo" else None, exchange_always=True)
    torch.cuda.synchronize(dev)
    t_build = time.perf_counter() - t0
    top, rows, plane_bytes = ring.arc_info()
    owner = torch.empty(Q, dtype=torch.int32, device=dev)
    hops = torch.empty(Q, dtype=torch.uint8, device=dev)
    status = torch.empty(Q, dtype=torch.uint8, device=dev)
    for _ in range(args.warmup):
        router.route(src, keys, owner, hops, status)
    torch.cuda.synchronize(dev)
    router.records_sent = 0
    _, dt_max = time_steps(lambda: router.route(src, keys, owner, hops, status), args.steps,
                           world, dev)
    sent = dist.sum_over_ranks(router.records_sent, world, dev)
    same = bool((owner == owner_ref).all().item()) and bool((hops == hops_ref).all().item()) \
        and int((status != 0).sum().item()) == 0
    same = dist.all_over_ranks(same, world, dev)
    total = world * Q * args.steps
    # exchange self-test: the same protocol with every rank's own lookups sent
    # through the collectives too (self_exchange), so every lookup crosses
    # RCCL -- at N = 1 the exchange a one-GPU run can time and check
    progress("arc: exchange self-test")
    router.self_exchange = True
    for t in (owner, hops, status):
        t.fill_(0xEE)
    router.route(src, keys, owner, hops, status)
    torch.cuda.synchronize(dev)
    router.records_sent = 0
    _, dt_x = time_steps(lambda: router.route(src, keys, owner, hops, status), args.steps,
                         world, dev)
    sent_x = dist.sum_over_ranks(router.records_sent, world, dev)
    same_x = dist.all_over_ranks(
        bool((owner == owner_ref).all().item()) and bool((hops == hops_ref).all().item())
        and int((status != 0).sum().item()) == 0, world, dev)
    router.self_exchange = False
    selftest = {"value": total / dt_x, "unit": "lookups/s", "ms_per_step": dt_x * 1e3 / args.steps,
                "records_exchanged_per_lookup": sent_x / total, "equals_replicated_route": same_x,
                "bytes_exchanged_per_lookup": 28 + 8,
                "layout": "ArcRouter.route with self_exchange: the exact-layout scatter of EVERY "
                          "lookup (the rank's own included) on the side stream, keys + sources + "
                          "hints (28 B) out and packed answers (8 B) back through RCCL list "
                          "all_to_alls in calls of <= 1 GiB per view, walked on arrival, "
                          "delivered through perm"}
    # DHash placement lists (n = 14) in the same layout (keys to
    # their owner's arc, windows read there from the arc + a 13-peer halo,
    # lists back): the same keys, K steps, equal to the replicated cx_nsucc
    progress("arc: placement lists")
    lists = torch.empty((Q, 14), dtype=torch.int32, device=dev)
    cnt = torch.empty(Q, dtype=torch.uint8, device=dev)
    router.nsucc(keys, 14, lists, cnt)  # builds the halo ring once
    _, dt_ns = time_steps(lambda: router.nsucc(keys, 14, lists, cnt), args.steps, world, dev)
    wl, wc = ring.nsucc(keys, 14)
    ns_same = dist.all_over_ranks(bool(torch.equal(lists, wl.to(torch.int32))) and
                                  bool(torch.equal(cnt, wc)), world, dev)
    del lists, cnt, wl, wc
    # exact-successor mode: the same keys, their owners searched on
    # the owner's arc of the ring only
    progress("arc: exact successors")
    own = torch.empty(Q, dtype=torch.int32, device=dev)
    router.successor(keys, own)  # builds the arc's ring once
    _, dt_sc = time_steps(lambda: router.successor(keys, own), args.steps, world, dev)
    sc_same = dist.all_over_ranks(bool(torch.equal(own, ring.successor(keys))), world, dev)
    del own
    exact_succ = {"value": total / dt_sc, "unit": "lookups/s",
                  "ms_per_step": dt_sc * 1e3 / args.steps, "equals_replicated_successor": sc_same,
                  "layout": "count pass and one all_gather; owners searched on the owner's arc "
                            "of the ring (ArcRouter.successor): own keys in place, the others "
                            "sent to their owner's rank (16 B out, 4 B back per key)"}
    placement = {"value": total / dt_ns, "unit": "keys/s", "ms_per_step": dt_ns * 1e3 / args.steps,
                 "n": 14, "equals_replicated_nsucc": ns_same,
                 "layout": "count pass (device counts, the rank's own keys' indices) and one "
                           "all_gather; windows read from the owner's arc plus a 13-peer halo "
                           "ring (ArcRouter.nsucc): own keys in place, the others sent to their "
                           "owner's rank (exact-layout scatter, all_to_all-v) with 15 int32 "
                           "per key back (window + count); at N = 1 every key is the rank's "
                           "own"}
    group = torch.distributed.get_backend() if torch.distributed.is_initialized() else None
    if single:
        torch.distributed.destroy_process_group()
    return {"value": total / dt_max, "unit": "lookups/s", "ms_per_step": dt_max * 1e3 / args.steps,
            "process_group": {"backend": group, "world": world,
                              "one_rank_group": bool(single)},
            "per_gpu_lookups_per_s": total / dt_max / world,
            "records_exchanged_per_lookup": sent / total,
            "rounds_per_step": router.rounds,
            "equals_replicated_route": same,
            "dhash_placement": placement,
            "exact_successor": exact_succ,
            "exchange_selftest": selftest,
            "top_levels_replicated": top, "local_rows": rows,
            "route_plane_bytes_per_gpu": plane_bytes, "build_s": t_build,
            "layout": f"ring IDs all-gathered; arc-sharded route planes x{world} (top {top} "
                      "levels replicated, lower levels for the arc + halo); key-first SoA "
                      "all_to_all-v with origin-resolved source hints (28 B out, 8 B back per "
                      "lookup crossing ranks); count pass whose device counts travel in one "
                      "all_gather per step, exact-layout scatter on a side stream overlapping "
                      "the walks of earlier pieces; each rank walks the lookups of its own arc "
                      "in place (no collective carries them); at N = 1 the general path runs "
                      "through a one-rank RCCL group (the count all_gather and its host read; "
                      "no lookup crosses ranks, so no all_to_all is issued)",
            "note": "owner, hops and status of every lookup equal the replicated route's "
                    "(checked on every rank)"}


def _route_rounds(rings, keys, srcs, dev, rounds=6, per=3):
    """Median per-launch ms of each ring routing the same keys, in interleaved
    rounds (order reversed every other round); rings: {name: (ring, out)}."""
    ms = {d: [] for d in rings}
    stream = torch.cuda.current_stream(dev)
    for k in range(rounds):
        for d in (list(ms) if k % 2 == 0 else list(ms)[::-1]):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            r, out = rings[d]
            e0.record(stream)
            for _ in range(per):
                r.route(srcs[d], keys, out=out)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ms[d].append(e0.elapsed_time(e1) / per)
    return {d: sorted(v)[len(v) // 2] for d, v in ms.items()}


def overlap_leg(serve, joins, leaves, keys, src, dev, builds=3, q_serve=1 << 23, priority=0):
    """Lookups keep running while the next membership epoch's ring builds
    (double-buffered route tables).  `serve` is epoch e's
    route-ready ring; a serving thread routes batches of q_serve of the bench's
    lookups on it on a stream of its own, keeping two launches queued (a
    server's pipeline), while this thread churns `serve` (the same 1 %/1 %
    event set) into epoch e + 1 and builds its fingers and route table on the
    new handle's stream -- `builds` times back to back, each new ring closed
    after it is route-ready.  Calls on one handle are serialised by a lock
    (the handle's stream is per-handle state: the churn call holds it, each
    route enqueue takes it for microseconds).

    Reports the serving rate alone and during the rebuilds (launches whose
    completion was observed inside a rebuild window), each rebuild's wall time
    under that load, and the serving outputs' equality with a reference route
    of `serve` taken before."""
    import threading
    from collections import deque
    Qs = min(q_serve, keys.shape[0])
    ks = keys[:Qs].contiguous()
    ss = (src[:Qs].to(torch.int64) % serve.n).to(torch.int32)
    ref = serve.route(ss, ks)
    torch.cuda.synchronize(dev)
    outs = [tuple(torch.empty_like(t) for t in ref) for _ in range(2)]
    lock = threading.Lock()
    stop = threading.Event()
    done = []  # host time at which each launch was seen complete
    # priority < 0: the serving stream is a high-priority HIP stream (its
    # launches' workgroups dispatch ahead of the rebuild's)
    stream = torch.cuda.Stream(device=dev, priority=priority)
    err = []

    def serving():
        try:
            with torch.cuda.stream(stream):
                pend, i = deque(), 0
                while not stop.is_set():
                    with lock:
                        serve.route(ss, ks, out=outs[i % 2])
                    ev = torch.cuda.Event()
                    ev.record(stream)
                    pend.append(ev)
                    i += 1
                    if len(pend) >= 2:
                        pend.popleft().synchronize()
                        done.append(time.perf_counter())
                while pend:
                    pend.popleft().synchronize()
                    done.append(time.perf_counter())
        except Exception as e:  # reported; the leg's checks then fail
            err.append(repr(e))

    def rate(t0, t1):
        n = sum(1 for t in done if t0 < t <= t1)
        return n * Qs / (t1 - t0)

    th = threading.Thread(target=serving, daemon=True)
    th.start()
    time.sleep(0.25)
    a0 = time.perf_counter()
    time.sleep(0.3)
    a1 = time.perf_counter()
    recs = []
    build_stream = torch.cuda.Stream(device=dev)
    for b in range(builds):
        with torch.cuda.stream(build_stream):
            t0 = time.perf_counter()
            with lock:
                new, _ = serve.churn(joins, leaves)
            new.sync()
            t1 = time.perf_counter()
            new.build_fingers()
            new.sync()
            t2 = time.perf_counter()
        recs.append({"route_ready_ms": (t2 - t0) * 1e3, "churn_ms": (t1 - t0) * 1e3,
                     "fingers_and_table_ms": (t2 - t1) * 1e3,
                     "serving_lookups_per_s": rate(t0, t2)})
        if b == builds - 1:
            k2 = ks[: 1 << 20]
            o, _, st = new.route((torch.arange(k2.shape[0], device=dev) % new.n).to(torch.int32), k2)
            new_ok = bool((o == new.successor(k2)).all().item()) and int((st != 0).sum().item()) == 0
        new.close()
        del new
    stop.set()
    th.join()
    alone = rate(a0, a1)
    same = not err and all(bool(torch.equal(a, b)) for o in outs for a, b in zip(o, ref))
    during = sorted(r["serving_lookups_per_s"] for r in recs)[len(recs) // 2]
    return {"serving_stream_priority": priority,
            "serving_lookups_per_s_alone": alone,
            "serving_lookups_per_s_during_rebuild": during,
            "serving_during_vs_alone": during / alone if alone else None,
            "rebuild_ms_under_load": sorted(r["route_ready_ms"] for r in recs)[len(recs) // 2],
            "rebuilds": recs, "serving_batch": Qs, "serving_equals_reference": same,
            "new_ring_route_equals_successor": new_ok, "errors": err,
            "layout": "epoch e's ring (route table and all) keeps serving on its own stream "
                      "while epoch e + 1 is churned from it and built on the new handle's "
                      "stream; both tables are resident (2 x 64 GiB of 288 GB)"}


def churn_leg(ring, keys, src, dev, depth_ab=28):
    """1 % joins + 1 % leaves of the bench ring -> route-ready.  Every epoch
    states its allocation path: the table pool's counters around it
    (chordx.pool_stats: bytes fresh from hipMalloc -- first-touch page
    mapping --, bytes handed back by the pool, idle blocks trimmed to retry a
    failed allocation, retries).  The pool is trimmed first, so the first
    epoch of each depth is cold (fresh HBM) and the second warm (the pool
    returns the first one's blocks, as every later membership epoch gets).

    Default depth: cold, warm; the two tables' hashes must be equal and the
    warm ring routes 2^22 keys to their exact successors.  Then the depth A/B
    (default R against `depth_ab` levels, cxi_set_route_depth) in ABBA order,
    so neither depth is always the one built first: order AB keeps the warm
    default ring and builds a `depth_ab` ring (cold, then warm) beside it;
    order BA closes both, builds `depth_ab` first and the default second.  In
    each order the two rings (and the bench ring) route the bench's keys in
    interleaved rounds; `per_launch_vs_default` is the mean over both orders."""
    N = ring.n
    nj = N // 100
    joins = torch.empty((nj, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(joins, SEED_CHURN)
    # distinct leaving peers (an odd stride is a bijection mod 2^k)
    pick = (torch.arange(nj, device=dev, dtype=torch.int64) * 0x9E3779B1) % N
    leaves = ring.ids_device()[pick].contiguous()
    out = {}
    epochs = []

    def epoch(depth, label):
        torch.cuda.synchronize(dev)
        st0 = chordx.pool_stats()
        t0 = time.perf_counter()
        new, _ = ring.churn(joins, leaves)
        new.sync()
        t1 = time.perf_counter()
        if depth:
            new.set_route_depth(depth)
        new.build_fingers()
        new.sync()
        t2 = time.perf_counter()
        alloc = chordx.pool_stats_delta(st0, chordx.pool_stats())
        rec = {"epoch": label, "route_ready_ms": (t2 - t0) * 1e3, "churn_ms": (t1 - t0) * 1e3,
               "fingers_and_table_ms": (t2 - t1) * 1e3,
               "route_levels": new.route_info()[2] // (new.n * 128),
               "alloc": {"fresh_GiB": alloc["fresh_bytes"] / 2**30,
                         "fresh_allocs": alloc["fresh_allocs"],
                         "pooled_GiB": alloc["reused_bytes"] / 2**30,
                         "pooled_allocs": alloc["reused_allocs"],
                         "trimmed_blocks": alloc["trims"],
                         "trimmed_GiB": alloc["trimmed_bytes"] / 2**30,
                         "retries": alloc["retries"], "failures": alloc["failures"]}}
        rec["alloc"]["path"] = ("trim-and-retry" if alloc["retries"] else
                                "fresh hipMalloc" if alloc["fresh_bytes"] > alloc["reused_bytes"]
                                else "pool reuse")
        epochs.append(rec)
        return new, rec

    chordx.pool_trim()
    new, out["cold"] = epoch(0, "default cold")
    h_cold = new.route_table_hash()
    new.close()
    del new
    a1, out["warm"] = epoch(0, "default warm")
    out["table_hash_equal"] = h_cold == a1.route_table_hash()
    q = 1 << 22
    k2 = torch.empty((q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(k2, SEED_KEYS + 0x100)
    s2 = (torch.arange(q, device=dev, dtype=torch.int64) % a1.n).to(torch.int32)
    o, h, st = a1.route(s2, k2)
    out["new_ring_route_equals_successor"] = bool((o == a1.successor(k2)).all().item()) \
        and int((st != 0).sum().item()) == 0
    out["new_ring_peers"] = a1.n
    del k2, s2, o, h, st
    # epoch e (a1) keeps serving while epoch e + 1 builds
    progress("churn: overlapped serving during rebuilds")
    out["overlapped"] = overlap_leg(a1, joins, leaves, keys, src, dev)
    # the same with the serving stream at high priority
    out["overlapped"]["high_priority_serving"] = overlap_leg(a1, joins, leaves, keys, src, dev,
                                                             builds=2, priority=-1)
    out["route_ready_ms"] = {"cold": out["cold"]["route_ready_ms"],
                             "warm": out["warm"]["route_ready_ms"]}
    r_def = out["warm"]["route_levels"]

    if depth_ab:
        progress("churn: table depth ABBA")
        sub = {"route_levels": depth_ab, "route_levels_default": r_def}
        Q = keys.shape[0]
        srcw = (src.to(torch.int64) % a1.n).to(torch.int32)

        def outs():
            return (torch.empty(Q, dtype=torch.int32, device=dev),
                    torch.empty(Q, dtype=torch.uint8, device=dev),
                    torch.empty(Q, dtype=torch.uint8, device=dev))

        # order AB: the warm default ring (built first) beside a depth_ab ring
        new, sub["cold"] = epoch(depth_ab, f"R{depth_ab} cold")
        new.close()
        del new
        b1, sub["warm"] = epoch(depth_ab, f"R{depth_ab} warm")
        ra, rb, rbench = outs(), outs(), outs()
        med_ab = _route_rounds({"A": (a1, ra), "B": (b1, rb), "bench": (ring, rbench)}, keys,
                               {"A": srcw, "B": srcw, "bench": src}, dev)
        same = bool((ra[0] == rb[0]).all().item()) and bool((ra[1] == rb[1]).all().item()) \
            and int((ra[2] != 0).sum().item()) == 0 and int((rb[2] != 0).sum().item()) == 0
        a1.close()
        b1.close()
        del a1, b1
        # order BA: depth_ab first, then the default
        b2, _ = epoch(depth_ab, f"R{depth_ab} (order BA, first)")
        a2, _ = epoch(0, "default (order BA, second)")
        med_ba = _route_rounds({"B": (b2, rb), "A": (a2, ra), "bench": (ring, rbench)}, keys,
                               {"A": srcw, "B": srcw, "bench": src}, dev)
        same = same and bool((ra[0] == rb[0]).all().item()) and \
            bool((ra[1] == rb[1]).all().item()) and int((ra[2] != 0).sum().item()) == 0
        b2.close()
        a2.close()
        del b2, a2, ra, rb, rbench
        d_ab = med_ab["B"] / med_ab["A"] - 1.0
        d_ba = med_ba["B"] / med_ba["A"] - 1.0
        sub.update({
            "route_ms_median": {
                "order_AB": {f"default_R{r_def}": med_ab["A"], f"R{depth_ab}": med_ab["B"],
                             "bench_ring": med_ab["bench"]},
                "order_BA": {f"R{depth_ab}": med_ba["B"], f"default_R{r_def}": med_ba["A"],
                             "bench_ring": med_ba["bench"]}},
            "per_launch_vs_default_by_order": {"AB": d_ab, "BA": d_ba},
            "per_launch_vs_default": (d_ab + d_ba) / 2,
            "results_equal_default": same,
            "note": f"R{depth_ab} against the default R{r_def}: a deeper table is more bytes to "
                    "build and fewer exact hops below it.  ABBA: in order AB the default ring "
                    f"is built first, in order BA the R{depth_ab} ring; per_launch_vs_default "
                    "(< 0: the deeper table routes faster) is the mean of the two orders, which "
                    "cancels a build-order effect"})
        out["table_depth_ab"] = sub
    else:
        a1.close()
        del a1
    out["epochs"] = epochs
    out["workload"] = (f"cx_churn of the bench ring: {nj} joins (splitmix 0x5EED0009) + {nj} "
                       "leaves (distinct peers), then cx_fingers_build (fingers + route table)")
    out["note"] = ("cold = the first epoch of a depth after cx_pool_trim (its tables are fresh "
                   "hipMalloc'd HBM: first-touch page mapping); warm = the table pool returns "
                   "the previous epoch's blocks (the steady state of a membership epoch); each "
                   "epoch's `alloc` states the path its allocations took")
    return out


def c5_leg(args, world, rank, dev, backend):
    """BASELINE config C5 (configs[4]): a 2^24-peer ring (splitmix 0x5EED0007),
    1 % joins (0x5EED0009) + 1 % leaves (distinct peers), and 2^26 keys
    (0x5EED0008) sharded over ranks (strong scaling: rank r scans
    [r Q / N, (r + 1) Q / N)).  One step = cx_dhash_maintenance: each key's
    n = 14 successor list on the old ring (DHashPeer placement,
    dhash_peer.cpp:103-129) and the global-maintenance misplaced scan against
    the new ring (RunGlobalMaintenance, dhash_peer.cpp:298-348) in one pass.
    Old ring IDs are all-gathered and every rank applies the same churn, so
    both rings are whole on every rank and the step needs no collective.
    Checks: old and new lists equal the rings' 14-windows on every key
    (reduced over ranks); on rank 0 the churned ring and map equal the
    oracle's, and lists / counts / masks / targets equal the oracle's
    restatement on the first `c5_oracle_keys` keys."""
    N, Q, n = 1 << args.peers_log2, 1 << args.c5_keys_log2, C5_N
    share = torch.empty((N // world, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(share, SEED_C5_RING, offset=rank * (N // world))
    ids = dist.gather_ids(share, world, backend)
    old = chordx.Ring(ids, device=dev.index or 0)
    del ids, share
    nj = N // 100
    joins = torch.empty((nj, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(joins, SEED_CHURN)
    pick = (torch.arange(nj, device=dev, dtype=torch.int64) * 0x9E3779B1) % old.n
    leaves = old.ids_device()[pick].contiguous()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    new, o2n = old.churn(joins, leaves)
    new.sync()
    t_churn = time.perf_counter() - t0
    k0, k1 = dist.shard_range(rank, world, Q)
    q = k1 - k0
    keys = torch.empty((q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(keys, SEED_C5_KEYS, offset=k0)

    def step():
        return old.dhash_maintenance(new, o2n, keys, n)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dist.barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        res = step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    dist.barrier(world)
    dt = time.perf_counter() - t0
    dt_max = dist.max_over_ranks(dt, world, dev)
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    kern_ms_max = dist.max_over_ranks(kern_ms, world, dev)
    old_lists, old_count, lists, count, mask, target = res
    del res

    # every key: both lists are the rings' 14-windows
    succ = new.successor(keys).to(torch.int64)
    ok_new = bool((lists.to(torch.int64) == (succ[:, None] + torch.arange(n, device=dev))
                   % new.n).all().item()) and bool((count == n).all().item())
    succ = old.successor(keys).to(torch.int64)
    ok_old = bool((old_lists.to(torch.int64) == (succ[:, None] + torch.arange(n, device=dev))
                   % old.n).all().item()) and bool((old_count == n).all().item())
    del succ
    ok_new = dist.all_over_ranks(ok_new, world, dev)
    ok_old = dist.all_over_ranks(ok_old, world, dev)
    n_mis = dist.sum_over_ranks(int((mask != 0).sum().item()), world, dev)
    parity = churn_ok = None
    m = 0
    t_or = 0.0
    if rank == 0 and args.c5_oracle_keys:
        import oracle as O
        t0 = time.perf_counter()
        old_ids, new_ids = old.ids(), new.ids()
        want_new, want_o2n = O.churn(old_ids, joins.cpu().numpy().view(np.uint64),
                                     leaves.cpu().numpy().view(np.uint64))
        o2n_h = o2n.cpu().numpy().view(np.uint32)
        churn_ok = bool((want_new == new_ids).all() and (want_o2n == o2n_h).all())
        m = min(args.c5_oracle_keys, q)
        km = keys[:m].cpu().numpy().view(np.uint64)
        wl, wc, wm, wt = O.misplaced(old_ids, want_new, want_o2n, km, n, threads=host_threads())
        parity = bool((lists[:m].cpu().numpy().view(np.uint32) == wl).all()
                      and (count[:m].cpu().numpy() == wc).all()
                      and (mask[:m].cpu().numpy().view(np.uint16) == wm).all()
                      and (target[:m].cpu().numpy() == wt).all())
        t_or = time.perf_counter() - t0
    cpu = None
    if rank == 0 and args.c5_cpu_keys:
        # SURVEY 8(d)'s CPU baseline: the lists by routed lookups, exactly like
        # GetNSuccessors, on the old ring (placement) and the new ring
        # (maintenance), then the misplaced check (or_maintenance_routed)
        import oracle as O
        th = host_threads()
        Fs = []
        for r in (old, new):
            r.set_route_variant(0)  # the finger rows only: no route table
            r.build_fingers()
            Fs.append(r.fingers_device().cpu().numpy().view(np.uint32))
            r.set_route_variant(-1)
        Po, Pn = O.Peers(old.ids(), Fs[0]), O.Peers(new.ids(), Fs[1])
        mc = min(args.c5_cpu_keys, q)
        kc = keys[:mc].cpu().numpy().view(np.uint64)
        o2n_h = o2n.cpu().numpy().view(np.uint32)
        va, v1, qa, q1, rr, dta, dt1 = _cpu_timed(
            lambda qq, t: O.maintenance_routed(Po, Pn, o2n_h, kc[:qq], n, threads=t), 256, mc,
            args.c5_cpu_seconds, th, q_min=min(mc, 1 << 16))
        gpu = (old_lists[:qa].cpu().numpy().view(np.uint32), old_count[:qa].cpu().numpy(),
               lists[:qa].cpu().numpy().view(np.uint32), count[:qa].cpu().numpy(),
               mask[:qa].cpu().numpy().view(np.uint16), target[:qa].cpu().numpy())
        cpu = {"value": va, "unit": "keys/s", "cores": th, "kind": "port", "value_1core": v1,
               "sample": f"first {qa} keys of the rank-0 shard on {th} threads ({dta:.1f} s), "
                         f"{q1} on 1 thread ({dt1:.1f} s): per key 14 routed GetSuccessor "
                         "lookups on the old ring (placement) and 14 on the new ring "
                         "(maintenance) from peer q mod n, then the misplaced check; "
                         "oracle/chord_oracle.c or_maintenance_routed (or_nsucc, "
                         "misplaced_from_list)",
               "equals_gpu_on_sample": all(bool((a == b).all()) for a, b in zip(rr, gpu)),
               "cpu_model": cpu_model(), "nproc": os.cpu_count()}
        del Fs, Po, Pn, gpu, rr
    dist.barrier(world)
    per_step = dt_max / args.steps
    out = {
        "metric": "C5 keys/s (whole node): n = 14 replica lists + misplaced scan after a "
                  "1 %/1 % churn", "unit": "keys/s", "value": Q / per_step,
        "ms_per_step": per_step * 1e3, "steps": args.steps, "scaling": "strong",
        "config": {"workload": f"C5: 2^{args.peers_log2}-peer ring (splitmix 0x5EED0007), "
                               f"2^{args.c5_keys_log2} keys (0x5EED0008) over {world} rank(s), "
                               f"n = {n}, {nj} joins (0x5EED0009) + {nj} leaves",
                   "peers_old": old.n, "peers_new": new.n, "keys_total": Q, "keys_per_gpu": q,
                   "kernel": "k_misplaced<true, true, true> (churn directory, fused old lists)"},
        "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK * world / 1e9,
                     "kernel_ms": kern_ms_max,
                     "achieved": Q * C5_BYTES_STREAM / (kern_ms_max * 1e-3) / 1e9,
                     "frac": Q * C5_BYTES_STREAM / (kern_ms_max * 1e-3) / (HBM_PEAK * world),
                     "model": f"{C5_BYTES_STREAM} B per key (key, one 64-B search line, old "
                              "and new 14-lists with counts, mask, targets), whole node, over "
                              "the slowest rank's kernel time",
                     "survey_model": {
                         "bytes_per_key": C5_BYTES_SURVEY,
                         "achieved": Q * C5_BYTES_SURVEY / (kern_ms_max * 1e-3) / 1e9,
                         "frac": Q * C5_BYTES_SURVEY / (kern_ms_max * 1e-3) / (HBM_PEAK * world),
                         "note": "SURVEY 8(d): 16 key + 64 search + 56 list + 1 + 2 per key "
                                 "(no old list)"}},
        "churn_ms": t_churn * 1e3,
        "new_lists_equal_new_window": ok_new, "old_lists_equal_old_window": ok_old,
        "keys_with_misplaced_holder": n_mis,
        "churn_equals_oracle": churn_ok,
        "parity_on_sample": parity, "oracle_sample_keys": m, "oracle_s": t_or,
        "cpu_baseline": cpu,
        "box_spread_record": "profiles/r06/c5_r4r5/README.md: round-4 and round-5 code in ABBA "
                             "order on one lease, directory load factor 1/2 and 1/4 on each "
                             "(3.29-3.30 ms at 1/4 for both, 3.44-3.45 ms at 1/2 for both)",
        "note": "both rings whole on every rank (IDs all-gathered, the same churn everywhere); "
                "no collective in the step; oracle: oracle/chord_oracle.c or_churn + "
                "or_misplaced (dhash_peer.cpp:298-348)"}
    old.close()
    new.close()
    return out


def _cpu_timed(fn, q_cal, q_max, budget_s, threads, q_min=0):
    """Calibrate fn(q, threads) on q_cal items (1 thread), then time it on a
    sample sized for ~budget_s / 3 on one core and ~2 budget_s / 3 on all
    `threads`; (items/s all cores, items/s one core, q all, q one, result)."""
    t0 = time.perf_counter()
    fn(q_cal, 1)
    per1 = (time.perf_counter() - t0) / q_cal
    q1 = int(min(q_max, max(q_cal, budget_s / 3 / max(per1, 1e-12))))
    t0 = time.perf_counter()
    fn(q1, 1)
    dt1 = time.perf_counter() - t0
    qa = int(min(q_max, max(q1, q_min, budget_s * 2 / 3 * threads / max(per1, 1e-12))))
    t0 = time.perf_counter()
    res = fn(qa, threads)
    dta = time.perf_counter() - t0
    return qa / dta, q1 / dt1, qa, q1, res, dta, dt1


def c2_leg(args, world, rank, dev):
    """BASELINE config C2 (configs[1]): exact successor resolution
    (StoredLocally / owner = lower_bound with wrap, abstract_chord_peer.cpp:720-725)
    of 2^20 uniform keys (splitmix 0x5EED0002) on a 2^16-peer ring (0x5EED0001),
    one cx_successor launch per step; every rank its own 2^20 keys (weak).
    Roofline on SURVEY 8(d)'s 20 B/query + 16 B/peer; parity on every key."""
    import oracle as O
    N, Q = 1 << 16, 1 << 20
    ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(ids, SEED_C2_RING)
    ring = chordx.Ring(ids, device=dev.index or 0)
    keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(keys, SEED_C2_KEYS, offset=rank * Q)
    out = torch.empty(Q, dtype=torch.int32, device=dev)
    steps = max(args.steps, 100)  # ~10 us kernels: enough launches to time
    for _ in range(max(args.warmup, 10)):
        ring.successor(keys, out=out)
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dist.barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        ring.successor(keys, out=out)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    dist.barrier(world)
    dt_max = dist.max_over_ranks(time.perf_counter() - t0, world, dev)
    ev_ms = dist.max_over_ranks(ev0.elapsed_time(ev1) / steps, world, dev)
    ring_np = ring.ids()
    keys_np = keys.cpu().numpy().view(np.uint64)
    want = O.successor(ring_np, keys_np, threads=host_threads())
    parity = dist.all_over_ranks(bool((out.cpu().numpy().view(np.uint32) == want).all()), world, dev)
    cpu = None
    if rank == 0:
        th = host_threads()
        va, v1, qa, q1, _, dta, dt1 = _cpu_timed(
            lambda q, t: O.successor(ring_np, keys_np[:q], threads=t), 4096, Q, 3.0, th)
        cpu = {"value": va, "unit": "lookups/s", "cores": th, "kind": "port", "value_1core": v1,
               "sample": f"first {qa} keys on {th} threads ({dta:.2f} s), {q1} on 1 ({dt1:.2f} s); "
                         "oracle/chord_oracle.c or_successor_batch (binary search of the sorted ring)",
               "cpu_model": cpu_model()}
    algo = Q * 20 + N * 16
    ring.close()
    total = world * Q * steps
    return {"metric": "C2 exact successor lookups/s (whole node)", "unit": "lookups/s",
            "value": total / dt_max, "ms_per_step": dt_max * 1e3 / steps, "steps": steps,
            "kernel_ms_per_step": ev_ms, "lookups_per_s_event_timed": world * Q / (ev_ms * 1e-3),
            "scaling": "weak",
            "config": {"workload": "C2: 2^16-peer ring (splitmix 0x5EED0001), 2^20 keys per GPU "
                                   "(0x5EED0002), cx_successor (round 6: LDS slice table, "
                                   "k_successor_lds; the bucket directory for other shapes)",
                       "peers": N, "keys_per_gpu": Q},
            "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK * world / 1e9,
                         "achieved": world * algo / (ev_ms * 1e-3) / 1e9,
                         "frac": world * algo / (ev_ms * 1e-3) / (HBM_PEAK * world),
                         "model": "SURVEY 8(d): 20 B per query (16 key + 4 owner) + 16 B per peer "
                                  "once per batch, over the event-timed step (launch gaps "
                                  "included; the kernel alone: profiles/r06/c2_lds)"},
            "parity_on_sample": parity, "oracle_sample_keys": Q, "cpu_baseline": cpu}


def c3_leg(args, world, rank, dev):
    """BASELINE config C3 (configs[2]): a 2^20-peer ring (0x5EED0003), the full
    m = 128 finger table (PopulateFingerTable converged, abstract_chord_peer.cpp:564-613)
    and 2^24 finger-routed lookups with hop counts (0x5EED0004, src = q mod N;
    GetSuccessor + ForwardRequest, abstract_chord_peer.cpp:318-337,
    chord_peer.cpp:185-211) per GPU.  Times: the finger build alone (route
    variant 0: rows only, no route table), fingers + route table (route-ready),
    and the default walk over K steps.  Parity: the whole finger table and the
    owners/hops of a 2^18-key sample against the oracle."""
    import oracle as O
    N, Q = 1 << 20, 1 << 24
    ids = torch.empty((N, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(ids, SEED_C3_RING)
    ring = chordx.Ring(ids, device=dev.index or 0)
    del ids

    def wall(fn, reps=3):
        best = None
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            fn()
            ring.sync()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best
    ring.set_route_variant(0)  # fingers only: rows, no route table
    F = ring.build_fingers(copy_out=True)
    t_fing = wall(ring.build_fingers)
    ring.set_route_variant(-1)
    ring.build_fingers()
    t_ready = wall(ring.build_fingers)
    keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(keys, SEED_C3_KEYS, offset=rank * Q)
    src = (torch.arange(Q, device=dev, dtype=torch.int64) % N).to(torch.int32)
    out = (torch.empty(Q, dtype=torch.int32, device=dev), torch.empty(Q, dtype=torch.uint8, device=dev),
           torch.empty(Q, dtype=torch.uint8, device=dev))
    for _ in range(args.warmup):
        ring.route(src, keys, out=out)
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
    dt_max = dist.max_over_ranks(time.perf_counter() - t0, world, dev)
    kern_ms = dist.max_over_ranks(ev0.elapsed_time(ev1) / args.steps, world, dev)
    ring.route_counters(True)
    ring.route(src, keys, out=out)
    g64, r16, xc, _ = ring.route_counters(False)
    gathers = g64 + r16 + 2 * xc
    sum_hops = int(out[1].to(torch.int64).sum().item())
    owner_eq = bool((ring.successor(keys) == out[0]).all().item()) and int((out[2] != 0).sum()) == 0
    ring_np = ring.ids()
    th = host_threads()
    Fw = O.fingers(ring_np, threads=th)
    fingers_ok = bool((F == Fw).all())
    m = 1 << 18
    P = O.Peers(ring_np, Fw)
    keys_np = keys[:m].cpu().numpy().view(np.uint64)
    src_np = src[:m].cpu().numpy().view(np.uint32)
    wo, wh, ws = O.route(P, src_np, keys_np, threads=th)
    parity = fingers_ok and bool((out[0][:m].cpu().numpy().view(np.uint32) == wo).all()
                                 and (out[1][:m].cpu().numpy() == wh).all() and (ws == 0).all())
    parity = dist.all_over_ranks(parity, world, dev)
    owner_eq = dist.all_over_ranks(owner_eq, world, dev)
    cpu = None
    if rank == 0:
        fa, f1, _, _, _, dfa, df1 = _cpu_timed(
            lambda q, t: O.fingers(ring_np, threads=t, rows=(0, q)), 4096, N, 3.0, th)
        ra, r1, qa, q1, _, dra, dr1 = _cpu_timed(
            lambda q, t: O.route(P, src_np[:q], keys_np[:q], threads=t), 2048, m, 6.0, th)
        cpu = {"fingers_peers_per_s": fa, "fingers_peers_per_s_1core": f1,
               "value": ra, "unit": "lookups/s", "value_1core": r1, "cores": th, "kind": "port",
               "sample": f"fingers: or_fingers_build rows ({dfa:.2f} s on {th} threads, {df1:.2f} s "
                         f"on 1); routes: or_route on the first {qa} keys ({dra:.2f} s on {th} "
                         f"threads), {q1} on 1 ({dr1:.2f} s)",
               "cpu_model": cpu_model()}
    del F, Fw, P
    ring.close()
    fing_bytes = N * (CX_FINGERS_B * 4 + 16)
    algo = Q * BYTES_STREAM + GRANULE * gathers
    ref = Q * (REF_STREAM + REF_SRC) + REF_HOP * sum_hops
    total = world * Q * args.steps
    return {"metric": "C3 finger-routed lookups/s with hop counts (whole node)",
            "unit": "lookups/s", "value": total / dt_max, "ms_per_step": dt_max * 1e3 / args.steps,
            "steps": args.steps, "kernel_ms": kern_ms, "scaling": "weak",
            "config": {"workload": "C3: 2^20-peer ring (splitmix 0x5EED0003), m = 128 fingers, "
                                   "2^24 keys per GPU (0x5EED0004), src = q mod N",
                       "peers": N, "keys_per_gpu": Q},
            "fingers_build_ms": t_fing * 1e3, "fingers_and_route_table_ms": t_ready * 1e3,
            "fingers_roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK / 1e9,
                                 "achieved": fing_bytes / t_fing / 1e9,
                                 "frac": fing_bytes / t_fing / HBM_PEAK,
                                 "model": "SURVEY 8(d): 528 B per peer (128 x 4 B written + 16 B "
                                          "read), over the wall time of cx_fingers_build (rows "
                                          "only, one GPU)"},
            "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK * world / 1e9,
                         "achieved": world * algo / (kern_ms * 1e-3) / 1e9,
                         "frac": world * algo / (kern_ms * 1e-3) / (HBM_PEAK * world),
                         "algo_bytes_per_launch": algo, "gathers_per_lookup": gathers / Q,
                         "model": f"{BYTES_STREAM} B streams per lookup + {GRANULE} B per random "
                                  "gather issued (counted), as the headline"},
            "reference_work_model": {"bytes_per_launch": ref,
                                     "GBps": ref / (kern_ms * 1e-3) / 1e9,
                                     "note": "SURVEY 8(d): 25 + 64 B + 128 B per hop"},
            "mean_hops": sum_hops / Q, "route_owner_equals_successor": owner_eq,
            "parity_on_sample": parity, "fingers_equal_oracle": fingers_ok,
            "oracle_sample_keys": m, "cpu_baseline": cpu}


def headline_line(args, world, N, Q, dt_max, roof, traffic, kernel_name, algo_bytes, kern_ms,
                  ref_bytes, gather, route_variant, table_bytes, cz_escapes, sum_hops, hist,
                  max_hops, bad, owner_eq, counting_same, succ_ms, small, rsrc_ms, rsrc_bad,
                  t_gather, t_ring, t_fing, t_fing_warm, setup_alloc):
    """Rank 0's JSON line with the headline and its checks; the sub-record
    legs (churn_route_ready, arc, cpu_baseline, c5, c2, c3) fill their keys
    as they finish (LegGuard prints the line as it stands if one hangs)."""
    total = world * Q * args.steps
    line = line_base(args, world, total / dt_max, dt_max, {
        "workload": "C4 finger-routed lookups with hop counts (per GPU): "
                    f"2^{args.peers_log2}-peer ring, 2^{args.keys_log2} keys/GPU/step, "
                    "src = q mod N, splitmix seeds 0x5EED0005/0x5EED0006",
        "peers": N, "keys_per_gpu": Q, "global_batch": world * Q,
        "parallelism": f"ring IDs all-gathered, replicated route tables, keys sharded "
                       f"x{world} (arc-sharded all_to_all-v layout: `arc`)"})
    roof.update({
        "traffic": None if traffic is None else traffic * world,
        "traffic_note": "PMC FETCH_SIZE + WRITE_SIZE per launch on one GPU "
                        "(profiles/traffic_route.json) x N",
        "kernel": kernel_name,
        "per_gpu": {"achieved": algo_bytes / (kern_ms * 1e-3) / 1e9,
                    "frac": algo_bytes / (kern_ms * 1e-3) / HBM_PEAK,
                    "kernel_ms": kern_ms, "algo_bytes_per_launch": algo_bytes,
                    "traffic": traffic, "rank": 0},
        "algo_model": f"{BYTES_STREAM} B streams per lookup + {GRANULE} B per random "
                      "gather issued (counted), summed over ranks"})
    line.update({
        "roofline": roof,
        "reference_work_model": {"bytes_per_launch": ref_bytes,
                                 "GBps": ref_bytes / (roof["kernel_ms"] * 1e-3) / 1e9,
                                 "note": "SURVEY 8(d): 128 B per hop, summed over ranks; "
                                         "hops the window table resolves without a gather "
                                         "are priced too, so this is not a byte count of "
                                         "the kernel"},
        "cpu_baseline": None,
        "arc": None,
        "churn_route_ready": None,
        "c5": None,
        "c2": None,
        "c3": None,
        "gather_roofline": gather,
        "route_variant": route_variant,
        "route_table_bytes": table_bytes,
        "route_cz_escapes": cz_escapes,
        "mean_hops": sum_hops / (world * Q),
        "hops_hist": hist,
        "max_hops": max_hops,
        "hops_hist_note": "hops_hist[h] = lookups of the timed batch (all ranks) that took "
                          "h hops; the CPU baseline's sample carries the oracle's histogram "
                          "(cpu_baseline.hist_equal)",
        "bad_status": bad,
        "route_owner_equals_successor": owner_eq,
        "counting_build_same_results": counting_same,
        "exact_successor_lookups_per_s": Q / (succ_ms * 1e-3),
        "route_small_batches": small,
        "route_random_src": {"kernel_ms": rsrc_ms, "lookups_per_s": Q / (rsrc_ms * 1e-3),
                             "bad_status": rsrc_bad,
                             "note": "same keys and kernel, src uniform in [0, N) "
                                     "(splitmix 0x5EED000A) instead of q mod N"},
        "setup_s": {"id_all_gather": t_gather, "ring_sort": t_ring,
                    "ring_sort_roofline": getattr(setup_ring, "sort_roofline", None),
                    "fingers_build": t_fing, "fingers_build_again": t_fing_warm,
                    "alloc": setup_alloc,
                    "note": "fingers_build = converged fingers + route table on fresh "
                            f"HBM (first touch of the {table_bytes / 2**30:.0f} GiB route "
                            "table); fingers_build_again = the same build into the "
                            "now-mapped tables"},
        "ab_variants": "benches/bench_route.py --variants (route and search A/B kernels)",
    })
    return line


def main_arc(args):
    """--mode arc: the arc-sharded layout (SURVEY 8e layout 2) is the headline."""
    world, rank, local = dist.env_rank()
    local = local % max(1, torch.cuda.device_count())  # rehearsal: ranks share a GPU
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    backend = os.environ.get("CX_DIST_BACKEND", "nccl")
    dist.init(backend, dev)
    N = 1 << args.peers_log2
    Q = 1 << args.keys_log2
    ring, t_gather, t_ring = setup_ring(args, world, rank, dev, backend)
    keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    q0, q1 = dist.shard(rank, Q)
    chordx.fill_splitmix(keys, SEED_KEYS, offset=q0)
    src = (torch.arange(q0, q1, device=dev, dtype=torch.int64) % ring.n).to(torch.int32)
    succ = ring.successor(keys)
    from chordx.arc import ArcRouter
    router = ArcRouter(ring, ring.n, rank, world,
                       comm_device="cpu" if backend == "gloo" else None)
    owner = torch.empty(Q, dtype=torch.int32, device=dev)
    hops = torch.empty(Q, dtype=torch.uint8, device=dev)
    status = torch.empty(Q, dtype=torch.uint8, device=dev)
    for _ in range(args.warmup):
        router.route(src, keys, owner, hops, status)
    torch.cuda.synchronize(dev)
    router.records_sent = 0
    _, dt_max = time_steps(lambda: router.route(src, keys, owner, hops, status), args.steps,
                           world, dev)
    bad = dist.sum_over_ranks(int((status != 0).sum().item()), world, dev)
    sent = dist.sum_over_ranks(router.records_sent, world, dev)
    sum_hops = dist.sum_over_ranks(int(hops.to(torch.int64).sum().item()), world, dev)
    mismatch = dist.sum_over_ranks(int((succ != owner).sum().item()), world, dev)
    if rank == 0:
        total = world * Q * args.steps
        line = line_base(args, world, total / dt_max, dt_max, {
            "workload": "C4 finger-routed lookups with hop counts, arc-sharded: "
                        f"2^{args.peers_log2}-peer ring, 2^{args.keys_log2} keys/GPU/step",
            "peers": N, "keys_per_gpu": Q, "global_batch": world * Q,
            "parallelism": f"arc-sharded route planes x{world}, key-first SoA "
                           "all_to_all (20 B out, 8 B back per lookup)"})
        line.update({"rounds_per_step": router.rounds,
                     "records_exchanged_per_lookup": sent / total,
                     "mean_hops": sum_hops / (world * Q), "bad_status": bad,
                     "route_owner_equals_successor": mismatch == 0,
                     "setup_s": {"id_all_gather": t_gather, "ring_sort": t_ring}})
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    args = parse()
    rc = launch(args)
    if rc is not None:
        sys.exit(rc)
    # the depth A/B closes two warm rings (~131 GiB at 2^24) before order BA
    # rebuilds them: a pool cap above that keeps both, so order BA is warm too
    # (at the default 96 GiB the older ring's blocks are freed and its rebuild
    # pays fresh page mapping, 2.2-2.4 s on the boxes measured)
    os.environ.setdefault("CX_POOL_CAP_GIB", "160")
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
    backend = os.environ.get("CX_DIST_BACKEND", "nccl")
    dist.init(backend, dev)
    N = 1 << args.peers_log2
    Q = 1 << args.keys_log2

    # ---- setup (untimed): replicated ring, converged finger + route tables ----
    progress("setup: ring, fingers, route table")
    ring, t_gather, t_ring = setup_ring(args, world, rank, dev, backend)
    st0 = chordx.pool_stats()
    t0 = time.perf_counter()
    ring.build_fingers()
    ring.sync()
    t_fing = time.perf_counter() - t0
    st1 = chordx.pool_stats()
    t0 = time.perf_counter()
    ring.build_fingers()  # same tables again: their HBM is now mapped
    ring.sync()
    t_fing_warm = time.perf_counter() - t0
    setup_alloc = {k: {"fresh_GiB": d["fresh_bytes"] / 2**30, "pooled_GiB": d["reused_bytes"] / 2**30,
                       "retries": d["retries"]}
                   for k, d in (("fingers_build", chordx.pool_stats_delta(st0, st1)),
                                ("fingers_build_again",
                                 chordx.pool_stats_delta(st1, chordx.pool_stats())))}
    keys = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    q0, q1 = dist.shard(rank, Q)
    chordx.fill_splitmix(keys, SEED_KEYS, offset=q0)
    src = (torch.arange(q0, q1, device=dev, dtype=torch.int64) % ring.n).to(torch.int32)
    owner = torch.empty(Q, dtype=torch.int32, device=dev)
    hops = torch.empty(Q, dtype=torch.uint8, device=dev)
    status = torch.empty(Q, dtype=torch.uint8, device=dev)
    out = (owner, hops, status)

    route_variant, cz_escapes, table_bytes = ring.route_info()
    kernel_name = {5: "k_walk<false, false, false>", 4: "k_route_tree<false, false>"}.get(
        route_variant, f"route variant {route_variant}")

    # ---- warmup ----
    progress("warmup")
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

    # ---- results (all reduced over ranks) ----
    progress("timed steps done; checks")
    bad = dist.sum_over_ranks(int((status != 0).sum().item()), world, dev)
    sum_hops = dist.sum_over_ranks(int(hops.to(torch.int64).sum().item()), world, dev)
    # hop histogram (SURVEY 5 metrics), summed over ranks; hops <= 255 (hop cap)
    hist = dist.sum_vec_over_ranks(torch.bincount(hops.to(torch.int64), minlength=256).cpu(),
                                   world, dev)
    max_hops = max(h for h, c in enumerate(hist) if c) if any(hist) else 0
    hist = hist[:max_hops + 1]
    succ = torch.empty(Q, dtype=torch.int32, device=dev)
    ring.successor(keys, out=succ)  # exact successor (directory search) of every key
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(3):
        ring.successor(keys, out=succ)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    succ_ms = e0.elapsed_time(e1) / 3
    owner_eq = dist.all_over_ranks(bool((succ == owner).all().item()), world, dev)
    exact_rec = exact_successor_record(ring, keys, succ, succ_ms, world, dev)
    # gathers the walk issues on this batch: the counting build of the same
    # kernel, run once after the timed region (same inputs, same outputs)
    ref = (owner.clone(), hops.clone())
    ring.route_counters(True)
    ring.route(src, keys, out=out)
    g64, r16, xc, nq = ring.route_counters(False)
    counting_same = bool((owner == ref[0]).all().item()) and bool((hops == ref[1]).all().item())
    gathers = g64 + r16 + 2 * xc
    algo_bytes = Q * BYTES_STREAM + GRANULE * gathers
    roof = whole_node_roofline(algo_bytes, kern_ms, world, dev)
    ref_bytes = dist.sum_over_ranks(Q * (REF_STREAM + REF_SRC), world, dev) + REF_HOP * sum_hops
    probe = ring.gather_probe()  # request-rate ceiling on this table, this box, this run
    # A/B: the same keys from uniformly random source peers (C4 fixes src = q mod N,
    # whose wave-adjacent sources share lines on the first gathers); owners must not change
    rsrc = torch.empty((Q, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(rsrc, SEED_RANDOM_SRC, offset=q0)
    rsrc = (rsrc[:, 0] & 0x7FFFFFFFFFFFFFFF).remainder(ring.n).to(torch.int32)
    rout = (torch.empty_like(owner), torch.empty_like(hops), torch.empty_like(status))
    ring.route(rsrc, keys, out=rout)
    e0.record(stream)
    for _ in range(3):
        ring.route(rsrc, keys, out=rout)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    rsrc_ms = e0.elapsed_time(e1) / 3
    owner_eq = dist.all_over_ranks(owner_eq and bool((succ == rout[0]).all().item()), world, dev)
    rsrc_bad = int((rout[2] != 0).sum().item())
    del rsrc, rout
    # small batches (serving): one launch over the first 2^k lookups of the same
    # batch, HIP events around 20 back-to-back launches; outputs must equal the
    # full batch's (the walk is per lookup)
    small = {}
    for lk in (12, 16, 20):
        m = 1 << lk
        if m > Q:
            continue
        so = (torch.empty(m, dtype=torch.int32, device=dev), torch.empty(m, dtype=torch.uint8, device=dev),
              torch.empty(m, dtype=torch.uint8, device=dev))
        ring.route(src[:m], keys[:m], out=so)
        e0.record(stream)
        for _ in range(20):
            ring.route(src[:m], keys[:m], out=so)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        same = bool(torch.equal(so[0], owner[:m])) and bool(torch.equal(so[1], hops[:m]))
        small[f"2^{lk}"] = {"us_per_launch": e0.elapsed_time(e1) / 20 * 1e3, "equal_to_batch": same}
        del so

    # ---- the headline line (rank 0), before any sub-record leg ----
    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as f:
            tj = json.load(f)
        if tj.get("peers") == N and tj.get("keys") == Q and tj.get("kernel") == kernel_name:
            traffic = tj.get("hbm_bytes_per_launch")
    req = gathers / (kern_ms * 1e-3)
    gather = {"requests_per_s": req, "ceiling": probe, "frac": req / probe,
              "gathers_per_lookup": gathers / Q, "table_gathers": g64, "exact_id_gathers": r16,
              "exact_hops": xc, "rank": 0,
              "note": "random 64-B requests the walk issued (counting build, same batch) per "
                      "second of kernel time, vs dependent quad-cooperative 64-B gathers/s "
                      "(non-temporal, as the walk's) measured on the same route table in this "
                      "run (rank 0)"}
    guard = LegGuard(rank)
    line = None
    if rank == 0:
        line = headline_line(args, world, N, Q, dt_max, roof, traffic, kernel_name, algo_bytes,
                             kern_ms, ref_bytes, gather, route_variant, table_bytes, cz_escapes,
                             sum_hops, hist, max_hops, bad, owner_eq, counting_same, succ_ms,
                             small, rsrc_ms, rsrc_bad, t_gather, t_ring, t_fing, t_fing_warm,
                             setup_alloc)
        line["exact_successor"] = exact_rec
        guard.line = line

    # ---- churn -> route-ready (f2), cold then warm ----
    progress("churn -> route-ready leg")

    def churn_block():
        if args.no_churn:
            return None
        churn = churn_leg(ring, keys, src, dev)
        chordx.pool_trim()  # the new rings' blocks are not needed by the arc leg
        churn["route_ready_ms_max_over_ranks"] = {
            k: dist.max_over_ranks(v, world, dev) for k, v in churn["route_ready_ms"].items()}
        churn["alloc_retries_all_ranks"] = dist.sum_over_ranks(
            sum(e["alloc"]["retries"] for e in churn["epochs"]), world, dev)
        churn["table_hash_equal"] = dist.all_over_ranks(churn["table_hash_equal"], world, dev)
        # one warm membership epoch (churn -> route-ready) amortized over K
        # timed batches of the headline: K Q / (route_ready + K t_batch)
        rr = churn["route_ready_ms_max_over_ranks"]["warm"]
        churn["epoch_amortized"] = {
            f"K{k}": {"lookups_per_s": world * k * Q / ((rr + k * dt_max * 1e3 / args.steps) * 1e-3),
                      "vs_headline": (k * dt_max * 1e3 / args.steps) / (rr + k * dt_max * 1e3 / args.steps)}
            for k in (1, 8)}
        churn["epoch_amortized"]["note"] = (
            "a warm 1 %/1 % churn epoch's route-ready time (max over ranks) plus K timed batches "
            "of the headline (2^25 lookups per GPU each), whole node; `overlapped`: epoch e "
            "keeps serving while epoch e + 1 builds (churn_route_ready.overlapped), so under "
            "back-to-back epochs the serving rate is the rate during a rebuild")
        ov = churn.get("overlapped")
        if ov:
            during = dist.sum_over_ranks(int(ov["serving_lookups_per_s_during_rebuild"]), world, dev)
            churn["epoch_amortized"]["overlapped"] = {
                "lookups_per_s": during, "vs_headline": during / (world * Q * args.steps / dt_max),
                "epoch_ms_under_load": dist.max_over_ranks(ov["rebuild_ms_under_load"], world, dev)}
        if "table_depth_ab" in churn:
            st = churn["table_depth_ab"]
            st["results_equal_default"] = dist.all_over_ranks(st["results_equal_default"], world, dev)
            st["route_ready_ms_warm_max_over_ranks"] = dist.max_over_ranks(
                st["warm"]["route_ready_ms"], world, dev)
        return churn

    churn = guard.run("churn_route_ready", churn_block)
    if line is not None:
        line["churn_route_ready"] = churn

    # ---- arc-sharded C4 (all_to_all-v) on the same keys and steps ----
    progress("arc leg")
    arc = guard.run("arc", lambda: None if args.no_arc else
                    arc_leg(args, ring, src, keys, owner, hops, world, rank, dev, backend))
    if line is not None:
        line["arc"] = arc

    # ---- CPU baseline: rank 0, every world size, after the timed region ----
    progress("cpu baseline")

    def cpu_block():
        cpu = None
        if rank == 0 and not args.no_cpu:
            F_host = np.empty((ring.n, chordx.CX_FINGERS), dtype=np.uint32)
            F_host[:] = ring.fingers_device().cpu().numpy().view(np.uint32)
            cpu = cpu_baseline(ring.ids(), F_host, keys.cpu().numpy().view(np.uint64),
                               src.cpu().numpy().view(np.uint32),
                               owner.cpu().numpy().view(np.uint32), hops.cpu().numpy(),
                               args.cpu_seconds, world)
            del F_host
        dist.barrier(world)
        return cpu

    cpu = guard.run("cpu_baseline", cpu_block)
    if line is not None:
        line["cpu_baseline"] = cpu

    # ---- C5 (configs[4]) after the bench ring's tables are released ----
    progress("c5 leg")

    def c5_block():
        if args.no_c5:
            return None
        ring.close()
        chordx.pool_trim()
        out = c5_leg(args, world, rank, dev, backend)
        chordx.pool_trim()
        return out

    c5 = guard.run("c5", c5_block)
    if line is not None:
        line["c5"] = c5

    # ---- C2 / C3 (configs[1], configs[2]): small rings, after the bench ring ----
    progress("c2 / c3 legs")

    def c23_block():
        c2 = None if args.no_c2 else c2_leg(args, world, rank, dev)
        c3 = None
        if not args.no_c3:
            c3 = c3_leg(args, world, rank, dev)
            chordx.pool_trim()
        return c2, c3

    c2, c3 = guard.run("c2_c3", c23_block)
    guard.stop()

    if rank == 0:
        line.update({"c2": c2, "c3": c3})
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
