"""Arc-sharded routing across ranks (layout 2).

When a ring's lookahead-tree table (n x R x 64 B: 32 GiB at 2^24 peers,
320 GiB at 2^27) outgrows one GPU, each rank keeps the replicated sorted ring
(16 B per peer) but tree rows only for its own arc of peers,
arc g of G = [g n / G, (g+1) n / G).  A lookup walks on the rank that owns the
row it needs next -- the GET_SUCC request travelling to the peer it was
forwarded to (ChordPeer::ForwardRequest, chord_peer.cpp:185-211) -- and comes
home as a RESULT record when it ends.  Owners, hops and statuses equal the
replicated-ring route's (tests/test_gpu_arc.py).

One bulk-synchronous round = step (walk every record as far as this rank's
rows reach) -> bucket by destination -> exchange.  The exchange is a real
data-path collective: one all_gather of the G x G count matrix (every rank
learns its receive splits and the global in-flight total from the same call)
and one all_to_all_single of the 32-B records.  With the "nccl" backend both
run on RCCL over xGMI; tests drive the same code with "gloo" on CPU.

The engine is any object with arc_build / arc_seed / arc_step / arc_bucket
(chordx.Ring on a GPU; tests/test_multiproc.py plugs in an oracle stand-in).
"""
from __future__ import annotations

import torch
import torch.distributed as tdist

MAX_ROUNDS = 300  # hop cap 255 + seed + result delivery, with margin


def arc_bounds(n: int, world: int, g: int):
    """Peers [lo, hi) of arc g (matches the kernels' destination rule)."""
    return g * n // world, (g + 1) * n // world


def arc_of(peer: int, n: int, world: int) -> int:
    g = min(peer * world // n, world - 1)
    while g > 0 and g * n // world > peer:
        g -= 1
    while g + 1 < world and (g + 1) * n // world <= peer:
        g += 1
    return g


class ArcRouter:
    def __init__(self, engine, n: int, rank: int, world: int, group=None, comm_device=None):
        if not 1 <= world <= 64:
            raise ValueError("arc routing supports 1..64 ranks")
        self.engine, self.n, self.rank, self.world = engine, n, rank, world
        self.group = group
        self.comm_device = comm_device  # device of the collective buffers
        self.lo, self.hi = arc_bounds(n, world, rank)
        engine.arc_build(self.lo, self.hi)
        self.rounds = 0
        self.records_sent = 0

    def _exchange(self, send, counts):
        """Returns (received records, global number of records in flight)."""
        if self.world == 1:
            return send, int(send.shape[0])
        dev = self.comm_device if self.comm_device is not None else send.device
        mine = torch.tensor(counts, dtype=torch.int64, device=dev)
        mat = torch.empty((self.world, self.world), dtype=torch.int64, device=dev)
        tdist.all_gather_into_tensor(mat.view(-1), mine, group=self.group)
        m = mat.cpu()
        inflight = int(m.sum())
        recv_counts = [int(x) for x in m[:, self.rank]]
        if inflight == 0:
            return send[:0], 0
        s = send.to(dev) if send.device != torch.device(dev) else send
        recv = torch.empty((sum(recv_counts), s.shape[1]), dtype=s.dtype, device=dev)
        tdist.all_to_all_single(recv, s.contiguous(), output_split_sizes=recv_counts,
                                input_split_sizes=list(counts), group=self.group)
        return (recv.to(send.device) if recv.device != send.device else recv), inflight

    def route(self, src, keys, owner, hops, status=None) -> int:
        """Routes this rank's lookups (issued at peers src[i]); collective over
        the group.  Writes owner/hops/status at the lookups' indices and
        returns the number of rounds taken."""
        recs = self.engine.arc_seed(self.rank, src, keys)
        for rnd in range(1, MAX_ROUNDS + 1):
            out = self.engine.arc_step(self.rank, recs, owner, hops, status)
            send, counts = self.engine.arc_bucket(self.world, out)
            self.records_sent += int(sum(counts))
            recs, inflight = self._exchange(send, counts)
            if inflight == 0:
                self.rounds = rnd
                return rnd
        raise RuntimeError("arc routing did not drain within MAX_ROUNDS rounds")
