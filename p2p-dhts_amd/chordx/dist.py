"""Multi-GPU plumbing for the replicated-ring, key-sharded lookup path.

The lookup path shards by query: every rank holds a replica of the ring (and
its finger/route tables) and routes its own contiguous slice of the global key
stream.  No collective touches the data path; the only cross-rank traffic is
the start/stop barrier and the max-over-ranks timing reduction.  With the
"nccl" backend torch.distributed runs RCCL over xGMI; tests use "gloo" on CPU.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as tdist


def env_rank():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend: str, device=None):
    world, rank, local = env_rank()
    if world > 1 and not tdist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
        tdist.init_process_group(backend, **kw)
    return world, rank, local


def init_single(backend: str, device=None) -> bool:
    """A one-rank process group (no rendezvous: an in-process HashStore).  On
    a one-GPU run this lets the collective path itself run -- the arc
    exchange's all_gather / all_to_all execute on RCCL with the rank as its
    own peer -- instead of being skipped.  Returns True if it created the
    group (the caller destroys it)."""
    if tdist.is_initialized():
        return False
    kw = {"device_id": device} if (backend == "nccl" and device is not None) else {}
    tdist.init_process_group(backend, store=tdist.HashStore(), rank=0, world_size=1, **kw)
    return True


def sum_vec_over_ranks(v, world: int, device=None):
    """Element-wise sum over ranks of an int64 vector (a list or 1-D tensor);
    returns a list of ints."""
    t = torch.as_tensor(v, dtype=torch.int64)
    if world > 1:
        d = _dev(device)
        t = t.to(d) if d is not None else t.cpu()
        tdist.all_reduce(t, op=tdist.ReduceOp.SUM)
    return [int(x) for x in t.cpu().tolist()]


def shard(rank: int, per_rank: int):
    """Global key-stream range [begin, end) routed by `rank` (weak scaling)."""
    return rank * per_rank, (rank + 1) * per_rank


def shard_range(rank: int, world: int, total: int):
    """[begin, end) of a fixed `total` split over `world` ranks (strong
    scaling: C5's 2^26 keys scanned by N ranks)."""
    return rank * total // world, (rank + 1) * total // world


def gather_rows(t, world: int, backend: str = "gloo"):
    """Concatenation over ranks (rank order) of every rank's rows of `t`
    (shards may differ in length): one all_gather of the row counts, one of
    the rows padded to the longest shard.  Returns the full tensor on every
    rank (on t's device)."""
    if world == 1:
        return t
    cd = torch.device("cpu") if backend == "gloo" else t.device
    x = t.to(cd).contiguous()
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=cd)
    ns = torch.empty(world, dtype=torch.int64, device=cd)
    tdist.all_gather_into_tensor(ns, n)
    counts = [int(c) for c in ns.cpu()]
    m = max(counts)
    pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=cd)
    pad[: x.shape[0]] = x
    allp = torch.empty((world * m,) + tuple(x.shape[1:]), dtype=x.dtype, device=cd)
    tdist.all_gather_into_tensor(allp, pad)
    parts = [allp[r * m: r * m + counts[r]] for r in range(world)]
    return torch.cat(parts).to(t.device)


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_self(gpus: int, script: str, argv):
    """One process per GPU: without a torch.distributed environment and with
    gpus > 1, run `script argv` under torch.distributed.run as a CHILD process
    (the caller has not touched the GPU) and return its exit status; None =
    run in this process.  2 when WORLD_SIZE disagrees with gpus."""
    import subprocess
    import sys
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if gpus <= 1:
            return None
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={gpus}", "--master-addr", "127.0.0.1",
               f"--master-port={free_port()}", os.path.abspath(script)] + list(argv)
        return subprocess.run(cmd).returncode
    if int(ws) != gpus:
        print(f"{os.path.basename(script)}: WORLD_SIZE={ws} but --gpus {gpus}", file=sys.stderr)
        return 2
    return None


def barrier(world: int):
    if world > 1:
        tdist.barrier()


def _dev(device):
    """Reduction tensors live on the GPU for RCCL and on the host for gloo."""
    if device is None or tdist.get_backend() == "gloo":
        return None
    return device


def max_over_ranks(x: float, world: int, device=None) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_dev(device))
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: int, world: int, device=None) -> int:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.int64, device=_dev(device))
    tdist.all_reduce(t, op=tdist.ReduceOp.SUM)
    return int(t.item())


def all_over_ranks(ok: bool, world: int, device=None) -> bool:
    """True iff `ok` holds on every rank."""
    return sum_over_ranks(0 if ok else 1, world, device) == 0


def gather_ids(share, world: int, backend: str):
    """The replicated ring's IDs: every rank generates its 1/world share and
    one all_gather (RCCL over xGMI; gloo on the host) replicates them
    (the ring IDs are replicated with one AllGather)."""
    if world == 1:
        return share
    cd = torch.device("cpu") if backend == "gloo" else share.device
    ids = torch.empty((share.shape[0] * world,) + tuple(share.shape[1:]), dtype=share.dtype,
                      device=cd)
    tdist.all_gather_into_tensor(ids, share.to(cd))
    return ids.to(share.device)
