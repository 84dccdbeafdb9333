"""Arc-sharded routing across ranks (layout 2).

Rank g of G owns the arc of peers [g n / G, (g+1) n / G).  Each rank keeps
the replicated sorted ring, the pattern-keyed route planes of the top levels
for all peers (replicated) and the planes below them only for its arc plus a
small halo (cx_arc_build).  A lookup walks on its origin rank while its rows
are replicated; the first time it needs a lower level it is close enough to
its key that every later peer lies in the key's arc or that arc's halo, so it
travels once -- the GET_SUCC request forwarded to the next peer
(ChordPeer::ForwardRequest, chord_peer.cpp:185-211) -- finishes on the rank of
its key's arc, and its result travels home once.  Owners, hops and statuses
equal the replicated-ring route's (tests/test_gpu_arc.py).

Default protocol ("soa", engines with arc_partition): the lookups go straight
to the rank whose arc holds their key's owner as two arrays -- keys (16 B) and
sources (4 B) -- in one all_to_all each; that rank walks them from their
sources over the replicated top planes and its own rows and answers in
receive order, 8 B per lookup; the answers come back with the splits swapped
and land in send order, where the origin scatters them through the
permutation it kept.  One count exchange, three all_to_alls, no origin or
index crossing xGMI, no re-bucketing of results.  With a device engine
(route_exact; gloo test runs stage the exchanges through the host) the
partition runs in two passes: a count pass over the keys (16 B per lookup)
whose device counts travel in the step's one all_gather -- read on the host
once -- and which compacts the indices of the rank's own lookups, then a
scatter that lays each piece's other lookups out by those counts on a side
stream, overlapping the walks of earlier pieces.  A rank walks the lookups
whose key lies in its own arc in place (arc_route_local: they never enter a
collective), and the all_to_alls carry only the other ranks' regions -- none
at all when no lookup of any rank crosses ranks.

DHash placement lists (nsucc) and exact successors (successor) use the same
key partition: the owner's rank reads the answer from its arc (plus a
13-peer halo for the 14-windows) and sends it back.

Record protocol ("records", origin walk or key-first): one bulk-synchronous round = step (walk every record as far as this rank's
rows reach) -> bucket by destination -> exchange: one all_gather of the G x G
count matrix (every rank learns its receive splits and the global in-flight
total from the same call) and one all_to_all_single of the 32-B records.  A
lookup takes three rounds: origin step, arc step, result delivery.  With the
"nccl" backend both collectives run on RCCL over xGMI; tests drive the same
code with "gloo" on CPU.

The engine is any object with arc_build(world, rank) / arc_seed / arc_step /
arc_bucket (chordx.Ring on a GPU; tests/test_multiproc.py plugs in an oracle
stand-in).
"""
from __future__ import annotations

import torch
import torch.distributed as tdist

MAX_ROUNDS = 300  # hop cap 255 + seed + result delivery, with margin
# Largest per-peer view of one all_to_all call (bytes).  Measured on the box
# (tools/diag_rccl_a2a.py, profiles/r06/rccl_a2a/): RCCL 2.26.6 delivers a
# 1 GiB send/recv view whole but only the first half of one of 2,013,265,920 B
# or more, and reports success.  Every exchange is cut into calls of at most
# this many bytes per view (ArcRouter._rounds).
VIEW_CAP = 1 << 30


class _Works:
    """The works of one exchange issued as several all_to_all calls."""

    def __init__(self, works):
        self.works = list(works)

    def wait(self):
        for w in self.works:
            w.wait()


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
    def __init__(self, engine, n: int, rank: int, world: int, group=None, comm_device=None,
                 exchange_always: bool = False):
        if not 1 <= world <= 64:
            raise ValueError("arc routing supports 1..64 ranks")
        self.engine, self.n, self.rank, self.world = engine, n, rank, world
        self.group = group
        self.comm_device = comm_device  # device of the collective buffers
        self.lo, self.hi = arc_bounds(n, world, rank)
        engine.arc_build(world, rank)
        self.rounds = 0
        self.records_sent = 0
        # key-first routing (no origin walk) pays off once lookups cross ranks;
        # a single rank walks them in place
        self.key_first = world > 1
        self._mat_host = None  # pinned landing buffer of the count matrix
        self.chunks = None     # route_soa pipeline depth (None: by batch size)
        self.regions = True    # single-pass partition into destination regions
        self.hints = True      # origin-resolved source hints with the lookups
        self.region_cap = None  # tests: (piece size, world) -> region cap (overflow path)
        # RCCL: count pass + exact-layout scatter on a side stream, own region
        # walked in place (route_exact); False: the single-pass region layout
        self.exact = True
        self._side = None      # side stream of the exact path's scatters
        # exchange_always: a single rank still partitions, exchanges (with
        # itself, through the process group's collectives) and delivers -- the
        # general path, so a one-GPU run executes and times what N ranks run
        self.exchange_always = exchange_always
        # self_exchange: the rank's own lookups / keys travel through the
        # collectives too (to itself) instead of being answered in place -- on a
        # one-rank group every lookup then crosses RCCL, the exchange a one-GPU
        # run can time and check (bench `arc.exchange_selftest`).  Must agree
        # on every rank (checked through the gathered rows).
        self.self_exchange = False
        # largest per-peer view of one all_to_all call (bytes); see _rounds
        self.view_cap = VIEW_CAP

    def _rounds(self, rows: int, row_bytes: int) -> int:
        """all_to_all calls one exchange is issued as: every per-peer view of
        each call stays at or below view_cap bytes (VIEW_CAP: RCCL copies only
        half of a larger one).  `rows` must be the largest per-peer count of
        the exchange over ALL ranks (from the gathered counts), so every rank
        issues the same number of calls."""
        return max(1, -(-int(rows) * int(row_bytes) // self.view_cap))

    def _list_a2a(self, outs, ins, rounds: int = 1):
        """RCCL list all_to_all from the views `ins` (one per destination)
        into `outs` (one per source), as `rounds` calls over consecutive
        slices of every view -- slice j of a view of c rows is rows [c j / R,
        c (j + 1) / R), the same cut on the sending and the receiving side.
        Asynchronous: returns one waitable for all of them."""
        works = []
        for j in range(rounds):
            o = [t[t.shape[0] * j // rounds: t.shape[0] * (j + 1) // rounds] for t in outs]
            i = [t[t.shape[0] * j // rounds: t.shape[0] * (j + 1) // rounds] for t in ins]
            works.append(tdist.all_to_all(o, i, group=self.group, async_op=True))
        return _Works(works)

    def _exchange(self, send, counts):
        """Returns (received records, global number of records in flight)."""
        if self.world == 1:
            return send, int(send.shape[0])
        dev = self.comm_device if self.comm_device is not None else send.device
        mine = torch.tensor(counts, dtype=torch.int64, device=dev)
        mat = torch.empty((self.world, self.world), dtype=torch.int64, device=dev)
        tdist.all_gather_into_tensor(mat.view(-1), mine, group=self.group)
        if mat.is_cuda:
            # the splits must reach the host (all_to_all takes lists): one
            # async copy into a pinned buffer, then wait on that copy only
            if self._mat_host is None or self._mat_host.shape != mat.shape:
                self._mat_host = torch.empty((self.world, self.world), dtype=torch.int64,
                                             pin_memory=True)
            self._mat_host.copy_(mat, non_blocking=True)
            torch.cuda.current_stream(mat.device).synchronize()
            m = self._mat_host
        else:
            m = mat
        inflight = int(m.sum())
        recv_counts = [int(x) for x in m[:, self.rank]]
        if inflight == 0:
            return send[:0], 0
        s = send.to(dev) if send.device != torch.device(dev) else send
        recv = torch.empty((sum(recv_counts), s.shape[1]), dtype=s.dtype, device=dev)
        if recv.is_cuda:
            rows = max(int(x) for x in m.flatten())
            self._list_a2a(list(torch.split(recv, recv_counts)),
                           list(torch.split(s.contiguous(), list(counts))),
                           self._rounds(rows, s.shape[1] * s.element_size())).wait()
        else:
            tdist.all_to_all_single(recv, s.contiguous(), output_split_sizes=recv_counts,
                                    input_split_sizes=list(counts), group=self.group)
        return (recv.to(send.device) if recv.device != send.device else recv), inflight

    def _a2a(self, t, out_splits, in_splits, dev, rounds: int = 1):
        """Asynchronous all-to-all-v of a contiguous buffer: (output, work).
        On RCCL every SoA exchange is a list all_to_all (split views, `rounds`
        calls: _list_a2a), so all ranks issue the same collective kind whether
        their pieces were laid out in regions or packed; gloo takes
        all_to_all_single."""
        s = t.to(dev) if t.device != torch.device(dev) else t
        out = torch.empty((sum(out_splits),) + tuple(s.shape[1:]), dtype=s.dtype, device=dev)
        if out.is_cuda:
            work = self._list_a2a(list(torch.split(out, list(out_splits))),
                                  list(torch.split(s.contiguous(), list(in_splits))), rounds)
        else:
            work = tdist.all_to_all_single(out, s.contiguous(), output_split_sizes=out_splits,
                                           input_split_sizes=in_splits, group=self.group,
                                           async_op=True)
        return out, work

    def _a2a_regions(self, t, counts, cap, out_splits, dev, rounds: int = 1):
        """Asynchronous all_to_all of destination regions: rows [d cap, d cap
        + counts[d]) of t go to rank d (no compaction on RCCL: a list
        all_to_all over region views).  gloo has no list all_to_all: the
        regions are packed first (test path)."""
        views = [t[d * cap: d * cap + counts[d]] for d in range(self.world)]
        if torch.device(dev).type == "cuda" and t.is_cuda:
            out = torch.empty((sum(out_splits),) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
            return out, self._list_a2a(list(torch.split(out, out_splits)), views, rounds)
        return self._a2a(torch.cat(views), out_splits, list(counts), dev)

    def _a2a_into_regions(self, t, in_splits, counts, cap, like, dev, rounds: int = 1):
        """Asynchronous all_to_all whose arrivals from rank d land at rows
        [d cap, d cap + counts[d]) of a world x cap buffer (the answers coming
        home to the region slots perm names)."""
        G = self.world
        if torch.device(dev).type == "cuda" and t.is_cuda:
            back = torch.empty((G * cap,) + tuple(t.shape[1:]), dtype=t.dtype, device=dev)
            outs = [back[d * cap: d * cap + counts[d]] for d in range(G)]
            return back, self._list_a2a(outs, list(torch.split(t, in_splits)), rounds), None
        packed, work = self._a2a(t, list(counts), in_splits, dev)
        return packed, work, (counts, cap)

    @staticmethod
    def _land(t, work, like):
        work.wait()  # the current stream waits for the collective
        return t.to(like.device) if t.device != like.device else t

    def route_soa(self, src, keys, owner, hops, status=None, chunks=None) -> int:
        """Key-first routing in structure-of-arrays form (module docstring);
        returns the number of exchange rounds (1 on a single rank, else 2).

        The batch is cut into pieces (default: one per 2^22 lookups, at most
        4, one on a one-rank group; `chunks` / self.chunks fix the count),
        partitioned up front; one
        all_gather carries every piece's counts.  Piece c + 1's lookups travel
        while piece c is walked, and piece c's answers travel back while piece
        c + 1 is walked (the collectives run on RCCL's stream, the walks on the
        current stream).  Ranks may hold different batch sizes (or none): each
        rank cuts its own batch, the gathered row is padded to a fixed number
        of piece slots, and every rank runs max-over-ranks pieces, the missing
        ones empty -- so all ranks issue the same collectives."""
        eng = self.engine
        if self.world == 1 and not self.exchange_always:
            eng.arc_deliver(eng.arc_route(src, keys), None, owner, hops, status)
            self.rounds = 1
            return 1
        q = int(keys.shape[0])
        fixed = chunks if chunks is not None else self.chunks
        kmax = max(4, int(fixed)) if fixed is not None else 4  # piece slots per rank
        # pieces overlap one piece's exchange with another's walk; a one-rank
        # group exchanges nothing, so its batch is one piece unless fixed
        k = int(fixed) if fixed is not None else (max(1, min(4, q >> 22)) if self.world > 1 else 1)
        k = max(1, min(k, kmax, max(q, 1)))
        if self.exact and hasattr(eng, "arc_count_async") and keys.is_cuda:
            return self.route_exact(src, keys, owner, hops, status, k, kmax)
        if self.self_exchange:
            raise ValueError("self_exchange needs the exact protocol (a device engine)")
        cut = [c * q // k for c in range(k + 1)]
        G = self.world
        # single-pass partition into per-destination regions when the engine
        # has it (cap = 1/G of the piece + slack; a piece whose keys crowd one
        # arc past it is partitioned in two passes instead)
        regions = hasattr(eng, "arc_partition_regions") and self.regions
        # origin-resolved source hints ride along (8 B) when the engine has
        # them: the arc rank's walk then needs no source IDs (a random gather)
        hints = regions and self.hints and getattr(eng, "arc_hints", False)
        dev = self.comm_device if self.comm_device is not None else keys.device
        # counts stay on the device (RCCL): every piece's partition writes its
        # counts and overflow flag into one row, one all_gather carries them
        # all, one pinned copy brings the gathered matrix to the host
        on_dev = regions and hasattr(eng, "arc_partition_regions_async") and \
            torch.device(dev).type == "cuda" and keys.is_cuda
        W = G + 1  # per piece: G counts + overflow flag
        row = torch.zeros(1 + kmax * W, dtype=torch.int64, device=dev)
        parts, caps = [], []

        def piece_cap(c):
            qc = cut[c + 1] - cut[c]
            if self.region_cap is not None:
                return max(1, int(self.region_cap(qc, G)))
            return max(1, qc // G + qc // (4 * G) + 4096)

        for c in range(k):
            ps, pk = src[cut[c]:cut[c + 1]], keys[cut[c]:cut[c + 1]]
            part = None
            cap = 0
            if on_dev:
                cap = piece_cap(c)
                part = eng.arc_partition_regions_async(G, ps, pk, cap, row[1 + c * W: 1 + (c + 1) * W],
                                                       hints=hints)
                part = part[:3] + (None,) + part[3:]  # counts: after the gather
            elif regions:
                cap = piece_cap(c)
                part = eng.arc_partition_regions(G, ps, pk, cap, hints=hints) if hints else \
                    eng.arc_partition_regions(G, ps, pk, cap)
            if part is None:
                part, cap = eng.arc_partition(G, ps, pk), 0
            if part[3] is not None:
                row[1 + c * W: 1 + c * W + G] = torch.tensor(part[3], dtype=torch.int64)
            parts.append(part)
            caps.append(cap)

        def gather(row):
            mat = torch.empty((G, row.numel()), dtype=torch.int64, device=row.device)
            tdist.all_gather_into_tensor(mat.view(-1), row, group=self.group)
            if mat.is_cuda:
                if self._mat_host is None or self._mat_host.shape != mat.shape:
                    self._mat_host = torch.empty(mat.shape, dtype=torch.int64, pin_memory=True)
                self._mat_host.copy_(mat, non_blocking=True)
                torch.cuda.current_stream(mat.device).synchronize()
                return self._mat_host
            return mat

        my_h = bool(hints) and all(len(p) > 4 for p in parts)
        row[0] = k | (int(my_h) << 20)  # bit 21 = 0: the region protocol
        mat = gather(row)
        self._agree(mat[:, 0], 0)
        ovf = [[int(mat[r, 1 + c * W + G]) for c in range(kmax)] for r in range(G)]
        if any(any(o) for o in ovf):
            # a piece crowded one destination past its region: that rank
            # partitions it again in two passes (host counts) and every rank
            # gathers the rows once more (all ranks see the same flags)
            for c in range(k):
                if ovf[self.rank][c]:
                    ps, pk = src[cut[c]:cut[c + 1]], keys[cut[c]:cut[c + 1]]
                    parts[c], caps[c] = eng.arc_partition(G, ps, pk), 0
            row = mat[self.rank].clone()
            for c in range(k):
                if ovf[self.rank][c]:
                    row[1 + c * W: 1 + c * W + G] = torch.tensor(parts[c][3], dtype=torch.int64)
                row[1 + c * W + G] = 0
            my_h = bool(hints) and all(len(p) > 4 for p in parts)
            row[0] = k | (int(my_h) << 20)
            mat = gather(row.to(dev))
        for c in range(k):  # this rank's counts, as host lists (the send splits)
            if parts[c][3] is None:
                parts[c] = parts[c][:3] + ([int(x) for x in mat[self.rank, 1 + c * W: 1 + c * W + G]],) \
                    + parts[c][4:]
        kg = int((mat[:, 0] & 0xFFFFF).max())  # pieces every rank runs
        use_h = bool(int((mat[:, 0] >> 20).min()))  # every rank's pieces carry hints
        recv = [[int(mat[r, 1 + c * W + self.rank]) for r in range(G)] for c in range(kg)]
        # calls per exchange of piece c: its largest per-peer view on any rank
        # (16-B keys out is the widest row; answers and hints are 8 B)
        rnd = [self._rounds(max(int(mat[r, 1 + c * W + d]) for r in range(G) for d in range(G)),
                            16) for c in range(kg)]
        if kg > k:  # this rank's extra pieces are empty
            e = (keys[:0], src[:0], torch.empty(0, dtype=torch.int32, device=keys.device),
                 [0] * G, torch.empty(0, dtype=torch.int64, device=keys.device))
            parts += [e] * (kg - k)
            caps += [0] * (kg - k)
            cut += [q] * (kg - k)
        # every rank exchanges the same arrays: hints travel only when every
        # rank's every piece carries them (bit 20 of the gathered row's first
        # word; a rank whose piece fell back to the two-pass partition has none)

        def send(c):
            sk, ss, _, cnt = parts[c][:4]
            if caps[c]:
                out = [self._a2a_regions(sk, cnt, caps[c], recv[c], dev, rnd[c]),
                       self._a2a_regions(ss, cnt, caps[c], recv[c], dev, rnd[c])]
                if use_h:
                    out.append(self._a2a_regions(parts[c][4], cnt, caps[c], recv[c], dev, rnd[c]))
                return out
            out = [self._a2a(sk, recv[c], cnt, dev, rnd[c]), self._a2a(ss, recv[c], cnt, dev, rnd[c])]
            if use_h:  # an empty piece (kg > k) still takes part in every exchange
                out.append(self._a2a(parts[c][4], recv[c], cnt, dev, rnd[c]))
            return out

        inflight = send(0)
        backs = []
        for c in range(kg):
            got = inflight
            rk = self._land(got[0][0], got[0][1], parts[c][0])
            rs = self._land(got[1][0], got[1][1], parts[c][1])
            rh = self._land(got[2][0], got[2][1], parts[c][0]) if use_h else None
            if c + 1 < kg:
                inflight = send(c + 1)
            res = eng.arc_route(rs, rk, hint=rh) if use_h else eng.arc_route(rs, rk)
            if caps[c]:
                backs.append(self._a2a_into_regions(res, recv[c], parts[c][3], caps[c],
                                                    parts[c][2], dev, rnd[c]))
            else:
                backs.append(self._a2a(res, parts[c][3], recv[c], dev, rnd[c]) + (None,))
        for c in range(kg):
            back = self._land(backs[c][0], backs[c][1], parts[c][2])
            if backs[c][2] is not None:  # gloo: packed answers -> their regions
                cnt, cap = backs[c][2]
                full = torch.empty((G * cap,) + tuple(back.shape[1:]), dtype=back.dtype,
                                   device=back.device)
                for d, piece in enumerate(torch.split(back, list(cnt))):
                    full[d * cap: d * cap + cnt[d]] = piece
                back = full
            sl = slice(cut[c], cut[c + 1])
            eng.arc_deliver(back, parts[c][2], owner[sl], hops[sl],
                            status[sl] if status is not None else None)
            self.records_sent += int(sum(parts[c][3]))
        self.rounds = 2
        return 2

    def _comm_cuda(self):
        return self.comm_device is None or torch.device(self.comm_device).type == "cuda"

    def _gather_row(self, row):
        """all_gather of every rank's count row, landed on the host (RCCL: one
        pinned copy, one wait on the current stream)."""
        G = self.world
        if not self._comm_cuda():  # gloo (tests): through the host
            r = row.to(self.comm_device)
            mat = torch.empty((G, r.numel()), dtype=torch.int64, device=r.device)
            tdist.all_gather_into_tensor(mat.view(-1), r, group=self.group)
            return mat
        mat = torch.empty((G, row.numel()), dtype=torch.int64, device=row.device)
        tdist.all_gather_into_tensor(mat.view(-1), row, group=self.group)
        # one pinned landing buffer per row length (route and placement rows differ)
        pool = self.__dict__.setdefault("_pinned", {})
        host = pool.get(row.numel())
        if host is None:
            host = pool[row.numel()] = torch.empty(mat.shape, dtype=torch.int64, pin_memory=True)
        host.copy_(mat, non_blocking=True)
        torch.cuda.current_stream(mat.device).synchronize()
        return host

    def _a2a_views(self, outs, ins, rounds: int = 1):
        """all_to_all from the views `ins` (one per destination rank) into the
        views `outs` (one per source rank): RCCL's list all_to_all in
        `rounds` calls (_list_a2a), asynchronous (returns its work); gloo
        (tests): packed through host buffers on the current stream,
        synchronous (returns None)."""
        if self._comm_cuda():
            return self._list_a2a(outs, ins, rounds)
        dev = self.comm_device
        in_splits = [int(t.shape[0]) for t in ins]
        out_splits = [int(t.shape[0]) for t in outs]
        packed = torch.cat([t.to(dev) for t in ins])
        got = torch.empty((sum(out_splits),) + tuple(packed.shape[1:]), dtype=packed.dtype,
                          device=dev)
        tdist.all_to_all_single(got, packed, output_split_sizes=out_splits,
                                input_split_sizes=in_splits, group=self.group)
        for t, piece in zip(outs, torch.split(got, out_splits)):
            t.copy_(piece)
        return None

    def _agree(self, w0, proto: int):
        """The protocol (bit 21 of the gathered rows' first words: 1 = the
        exact layout) and self_exchange (bit 22) must be the same on every
        rank.  Every rank sees the same gathered words, so a disagreement
        raises on all of them instead of hanging the group in mismatched
        collectives."""
        words = {(int(w) >> 21) & 3 for w in w0}
        if len(words) != 1:
            raise RuntimeError("arc routing: ranks disagree on the protocol or self_exchange "
                               f"(bits 21-22 of the gathered rows: {sorted(words)})")
        if words.pop() != proto | (int(self.self_exchange) << 1):
            raise RuntimeError("arc routing: gathered protocol word does not match this rank's")

    def route_exact(self, src, keys, owner, hops, status, k, kmax) -> int:
        """route_soa on RCCL with the exact-layout partition (module docstring).

        Current stream: the count pass of every piece (arc_count_async into one
        device row; it also compacts the indices of the lookups of this rank's
        own arc), the all_gather of that row and its one host read, the walk of
        every piece's own lookups in place in ONE launch (arc_route_local:
        outputs straight into owner / hops / status; a walk launch below ~2^21
        lookups is latency-bound at ~0.17 ms, so G pieces' own lookups walked
        piece by piece would pay that G times), then per piece the walk of the
        lookups the other ranks sent, the answers' return exchange and the
        delivery of this rank's remote lookups.  Side stream (G > 1): the scatter of each piece's
        remote lookups (arc_scatter_async, reading the counts on the device,
        own lookups skipped), started as soon as the counts exist, and each
        piece's outgoing exchange, which waits on that scatter only.  A
        one-rank group has no remote lookups: no scatter, no all_to_all, no
        delivery -- unless self_exchange, which sends the rank's own lookups
        through the collectives like everyone else's (own walk skipped).

        The gathered row is 1 + kmax (G + 1) words, the length the region
        protocol gathers: word 0 = piece count | hints << 20 | 1 << 21 (exact)
        | self_exchange << 22, then kmax x G counts, then the kmax piece
        lengths; every rank checks every rank's counts against its lengths and
        the protocol bits, so a bad row raises on all ranks.  Returns 2."""
        eng, G, me = self.engine, self.world, self.rank
        sx = bool(self.self_exchange)
        dev = keys.device
        q = int(keys.shape[0])
        cut = [c * q // k for c in range(k + 1)]
        main = torch.cuda.current_stream(dev)
        if self._side is None or self._side.device != dev:
            self._side = torch.cuda.Stream(dev)
        side = self._side
        hints = bool(self.hints and getattr(eng, "arc_hints", False))
        LEN = 1 + kmax * G  # piece lengths start here
        # the row's host-known words (flags, piece lengths) in one pinned copy;
        # the landing buffer is free again: the previous call's row gather
        # waited on this stream after its copy
        pool = self.__dict__.setdefault("_rowh", {})
        rowh = pool.get(LEN + kmax)
        if rowh is None:
            rowh = pool[LEN + kmax] = torch.empty(LEN + kmax, dtype=torch.int64, pin_memory=True)
        rowh.zero_()
        rowh[0] = k | (int(hints) << 20) | (1 << 21) | (int(sx) << 22)
        for c in range(k):
            rowh[LEN + c] = cut[c + 1] - cut[c]
        row = rowh.to(dev, non_blocking=True)
        own_idx = torch.empty(max(q, 1), dtype=torch.int32, device=dev)
        wsw = eng.arc_own_ws_words(max(cut[c + 1] - cut[c] for c in range(k)))
        own_ws = torch.empty(k * wsw, dtype=torch.int32, device=dev)
        for c in range(k):
            eng.arc_count_async(G, keys[cut[c]:cut[c + 1]], row[1 + c * G: 1 + (c + 1) * G], me,
                                own_idx[cut[c]:], own_ws[c * wsw: (c + 1) * wsw])
        parts, ready = [], []
        scatter = G > 1 or sx
        if scatter:
            cursors = torch.empty(k * G, dtype=torch.int32, device=dev)
            side.wait_stream(main)  # the counts (and the caller's inputs) are written
            with torch.cuda.stream(side):
                for c in range(k):
                    sl = slice(cut[c], cut[c + 1])
                    part = eng.arc_scatter_async(G, src[sl], keys[sl],
                                                 row[1 + c * G: 1 + (c + 1) * G],
                                                 cursors[c * G: (c + 1) * G], hints=hints,
                                                 skip=-1 if sx else me)
                    parts.append(part if hints else part + (None,))
                    ev = torch.cuda.Event()
                    ev.record(side)
                    ready.append(ev)
        mat = self._gather_row(row)
        self._agree(mat[:, 0], 1)
        kg = int((mat[:, 0] & 0xFFFFF).max())  # pieces every rank runs
        use_h = bool(int((mat[:, 0] >> 20).min() & 1))  # every rank's pieces carry hints
        for r in range(G):  # every rank checks every row: a bad one raises everywhere
            for c in range(kmax):
                if sum(int(x) for x in mat[r, 1 + c * G: 1 + (c + 1) * G]) != int(mat[r, LEN + c]):
                    raise RuntimeError(f"arc count pass and partition disagree (rank {r}, "
                                       f"piece {c})")
        if scatter and kg > k:  # this rank's extra pieces are empty
            e = (keys[:0], src[:0], torch.empty(0, dtype=torch.int32, device=dev),
                 torch.empty(0, dtype=torch.int64, device=dev))
            parts += [e] * (kg - k)
            ready += [None] * (kg - k)
        cut += [q] * (kg - k)

        def crosses(r, d):  # lookups of rank r for rank d travel through the collective
            return r != d or sx
        cnt = [[int(mat[me, 1 + c * G + d]) for d in range(G)] for c in range(kg)]
        recv = [[int(mat[r, 1 + c * G + me]) if crosses(r, me) else 0 for r in range(G)]
                for c in range(kg)]
        offs = []  # travelling regions only (the own lookups take no slot)
        for c in range(kg):
            o, acc = [], 0
            for d in range(G):
                o.append(acc)
                acc += cnt[c][d] if crosses(me, d) else 0
            offs.append(o)
        # calls per exchange of piece c: its largest travelling per-peer view on
        # any rank, 16-B keys being the widest row (the same on every rank)
        rnd = [self._rounds(max([int(mat[r, 1 + c * G + d]) for r in range(G) for d in range(G)
                                 if crosses(r, d)] + [0]), 16) for c in range(kg)]
        # lookups that cross ranks anywhere (the same answer on every rank):
        # without any, no rank issues an all_to_all
        remote = any(int(mat[r, 1 + c * G + d]) for r in range(G) for d in range(G)
                     if crosses(r, d) for c in range(kg))

        def region(t, c, d):
            return t[offs[c][d]: offs[c][d] + cnt[c][d]] if crosses(me, d) else t[:0]

        def send(c):
            """Issued on the side stream: waits for piece c's scatter only.
            Returns ([(received, work)], event after the issue on the side
            stream)."""
            sk, ss, _, sh = parts[c]
            out = []
            with torch.cuda.stream(side):
                for t in ((sk, ss, sh) if use_h else (sk, ss)):
                    o = torch.empty((sum(recv[c]),) + tuple(t.shape[1:]), dtype=t.dtype,
                                    device=dev)
                    w = self._a2a_views(list(torch.split(o, recv[c])),
                                        [region(t, c, d) for d in range(G)], rnd[c])
                    out.append((o, w))
                ev = torch.cuda.Event()
                ev.record(side)
            return out, ev

        inflight = send(0) if remote else None
        # this rank's own lookups, every piece at once: walked in place, outputs
        # written (the count pass left each piece's indices piece-relative at
        # own_idx[cut[c]:])
        n_own = [0 if sx else cnt[c][me] for c in range(kg)]
        walk_own = eng.arc_route_local
        if sum(n_own):
            if sum(1 for x in n_own if x) == 1:
                c = next(c for c in range(kg) if n_own[c])
                sl = slice(cut[c], cut[c + 1])
                walk_own(src[sl], keys[sl], own_idx[cut[c]: cut[c] + n_own[c]],
                         owner[sl], hops[sl], status[sl] if status is not None else None)
            else:
                idx_all = torch.empty(sum(n_own), dtype=torch.int32, device=dev)
                at = 0
                for c in range(kg):
                    if n_own[c]:
                        torch.add(own_idx[cut[c]: cut[c] + n_own[c]], cut[c],
                                  out=idx_all[at: at + n_own[c]])
                        at += n_own[c]
                walk_own(src, keys, idx_all, owner, hops, status)
        backs = []
        for c in range(kg):
            got = inflight
            if remote and c + 1 < kg:
                inflight = send(c + 1)
            back, work = None, None
            if remote:
                n_rem = sum(cnt[c]) - n_own[c]
                # the piece's length (perm names slots < n_rem; arc_deliver
                # takes a result buffer at least as long as perm)
                back = torch.empty(cut[c + 1] - cut[c], dtype=torch.int64, device=dev)
                arrived, ev = got
                main.wait_event(ev)
                for t, w in arrived:
                    if w is not None:
                        w.wait()
                    # allocated on the side stream, read by this stream's walk:
                    # the allocator must not hand the block to a later side-
                    # stream allocation before that walk is done
                    t.record_stream(main)
                rk, rs_ = arrived[0][0], arrived[1][0]
                rh = arrived[2][0] if use_h else None
                res = eng.arc_route(rs_, rk, hint=rh) if use_h else eng.arc_route(rs_, rk)
                work = self._a2a_views([region(back, c, d) for d in range(G)],
                                       list(torch.split(res, recv[c])), rnd[c])
                self.records_sent += n_rem
            backs.append((back, work))
        if scatter:
            for c in range(kg):
                back, work = backs[c]
                if ready[c] is not None:
                    main.wait_event(ready[c])  # perm is written (no remote: nothing else)
                if work is not None:
                    work.wait()
                if back is None:
                    continue
                sl = slice(cut[c], cut[c + 1])
                parts[c][2].record_stream(main)  # perm: a side-stream block read here
                eng.arc_deliver(back, parts[c][2], owner[sl], hops[sl],
                                status[sl] if status is not None else None)
        self.rounds = 2
        return 2

    def successor(self, keys, owner) -> int:
        """Exact-successor mode of the arc layout: this rank's
        keys are bucketed by the arc that holds their owner (the arc
        splitters of cx_arc_build, as the walk's partition), sent there with
        one all_to_all-v, searched on that rank against its own arc of the
        ring only (StoredLocally's converged answer, abstract_chord_peer.cpp:
        720-725, over the arc's IDs), and the owners come back with the
        splits swapped; owner[i] = the global peer index.  Collective over the
        group; returns the number of exchange rounds (2; 0 on a single rank
        without exchange_always, which searches in place)."""
        eng = self.engine
        if self.world == 1 and not self.exchange_always:
            # the one arc is the whole ring: the engine's own search (no second
            # ring holding the same IDs)
            owner.copy_(eng.successor(keys).to(owner.dtype))
            return 0
        # one piece: the collectives cut themselves into calls of <= view_cap
        # bytes per view (_rounds)
        self._succ_piece(keys, owner, self._exact_piece(keys))
        return 2

    def _exact_piece(self, keys) -> bool:
        """The exact-layout piece protocol (device engine, device keys);
        self_exchange needs it."""
        exact = hasattr(self.engine, "arc_count_async") and keys.is_cuda
        if self.self_exchange and not exact:
            raise ValueError("self_exchange needs the exact protocol (a device engine)")
        return exact

    def _succ_piece(self, keys, owner, exact):
        if exact:
            return self._succ_piece_exact(keys, owner)
        eng, G = self.engine, self.world
        zero = self._zeros_src(keys)
        sk, _, perm, counts = eng.arc_partition(G, zero, keys)[:4]
        dev = self.comm_device if self.comm_device is not None else sk.device
        # the counts and, last, the protocol word (bits 21-22, _agree)
        mine = torch.tensor(list(counts) + [int(self.self_exchange) << 22], dtype=torch.int64,
                            device=dev)
        mat = torch.empty((G, G + 1), dtype=torch.int64, device=dev)
        tdist.all_gather_into_tensor(mat.view(-1), mine, group=self.group)
        m = mat.cpu() if mat.is_cuda else mat
        self._agree(m[:, G], 0)
        recv = [int(m[r, self.rank]) for r in range(G)]
        nr = self._rounds(max(int(x) for x in m[:, :G].flatten()), 16)
        rk, work = self._a2a(sk, recv, list(counts), dev, nr)
        rk = self._land(rk, work, sk)
        if rk.shape[0]:
            got = self._arc_ring().successor(rk)  # index in this rank's arc
            got = (got.to(torch.int64) + self.lo).to(torch.int32)
        else:  # nothing for this arc (or an empty arc: n < world)
            got = torch.empty(0, dtype=torch.int32, device=rk.device)
        back, work = self._a2a(got, list(counts), recv, dev, nr)
        back = self._land(back, work, perm)
        owner.copy_(back.to(owner.device)[perm.long()].to(owner.dtype))
        self.records_sent += int(sum(counts))

    def _succ_piece_exact(self, keys, owner):
        """One piece on a device engine: the count pass (device counts, this
        rank's own keys' indices) and one all_gather; own keys are searched in
        place on the arc's ring, the others go to their owner's rank in the
        exact layout (own skipped) and their owners come back through perm."""
        eng, G, me = self.engine, self.world, self.rank
        q = int(keys.shape[0])
        dev = keys.device
        mat, row, own_idx = self._count_gather(keys)
        sx = bool(self.self_exchange)
        c_me = 0 if sx else int(mat[me, me])

        def search(k):  # global owner indices of keys owned in this arc
            return (self._arc_ring().successor(k).to(torch.int64) + self.lo).to(torch.int32)
        if c_me == q and q:
            owner.copy_(search(keys).to(owner.dtype))
        elif c_me:
            oi = own_idx[:c_me].long()
            owner[oi] = search(keys[oi]).to(owner.dtype)
        remote = any(int(mat[r, d]) for r in range(G) for d in range(G) if r != d or sx)
        if not remote:
            return
        send = [int(mat[me, d]) if d != me or sx else 0 for d in range(G)]
        recv = [int(mat[r, me]) if r != me or sx else 0 for r in range(G)]
        nr = self._rounds(self._max_crossing(mat, sx), 16)
        cursor = torch.empty(G, dtype=torch.int32, device=dev)
        sk, _, perm = eng.arc_scatter_async(G, self._zeros_src(keys), keys, row, cursor,
                                            skip=-1 if sx else me)
        cdev = self.comm_device if self.comm_device is not None else dev
        rk, work = self._a2a(sk[:sum(send)], recv, send, cdev, nr)
        rk = self._land(rk, work, sk)
        got = search(rk) if rk.shape[0] else torch.empty(0, dtype=torch.int32, device=dev)
        back, work = self._a2a(got, send, recv, cdev, nr)
        back = self._land(back, work, perm).to(owner.device)
        pm = perm.long()
        sel = pm >= 0
        owner[sel] = back[pm[sel]].to(owner.dtype)
        self.records_sent += sum(send)

    def halo_ring(self, h: int):
        """This rank's arc plus the h peers after it as a ring of its own
        (SURVEY 8e's DHash halo: a 14-window from an owner in the arc reaches
        13 peers past it), and the map from its indices to global ones:
        (ring, wrap) -- local index j is global j when j < wrap (the halo
        wrapped past the ring's end to peers 0 .. wrap - 1, the smallest IDs),
        else lo + j - wrap.  Built once per h."""
        cache = getattr(self, "_halo", None)
        if cache is not None and cache[0] == h:
            return cache[1], cache[2]
        eng, n = self.engine, self.n
        ids = eng.ids_device()
        end = self.hi + h
        wrap = max(0, min(end - n, self.lo))  # never onto the arc itself (one rank: none)
        parts = [ids[self.lo:min(end, n)]]
        if wrap:
            parts.insert(0, ids[:wrap])
        sub = type(eng)(torch.cat(parts).contiguous(), device=eng.device)
        self._halo = (h, sub, wrap)
        return sub, wrap

    def nsucc(self, keys, n_list: int, lists, count) -> int:
        """DHash placement lists in the arc layout ("a 14-window may
        straddle an arc, so use a 13-peer halo"): this rank's keys go to the
        rank whose arc holds their owner (the exact-successor partition), that
        rank reads each key's n-successor window (GetNSuccessors on a
        converged ring, abstract_chord_peer.cpp:345-373) from its arc plus the
        n - 1 peers after it (halo_ring), and the windows come back as global
        peer indices with the splits swapped: lists[i, :] / count[i] as
        cx_nsucc on the whole ring.  Collective over the group; returns the
        number of exchange rounds (2; 0 on a single rank without
        exchange_always, or on a ring too small for disjoint halos, where the
        replicated ring answers in place)."""
        eng, G = self.engine, self.world
        h = n_list - 1
        if (G == 1 and not self.exchange_always) or self.n < G * (n_list + 1):
            lo_, co_ = eng.nsucc(keys, n_list)
            lists.copy_(lo_.to(lists.dtype))
            count.copy_(co_.to(count.dtype))
            return 0
        # one piece: the collectives cut themselves into calls of <= view_cap
        # bytes per view (_rounds; the 60-B rows back of a 2^25-key batch are
        # 2,013,265,920 B, which one RCCL call delivers only half of)
        if not self._exact_piece(keys):
            raise ValueError("ArcRouter.nsucc needs a device engine and device keys")
        self._nsucc_piece(keys, n_list, lists, count)
        return 2

    def _count_gather(self, keys):
        """The exact layout's count pass and its one all_gather: (gathered
        (G, G + 1) host matrix -- counts, then the protocol word --, the
        device counts row, own_idx).  Every rank checks the protocol words."""
        eng, G, me = self.engine, self.world, self.rank
        q = int(keys.shape[0])
        dev = keys.device
        row = torch.zeros(G + 1, dtype=torch.int64, device=dev)
        row[G] = (1 | (int(self.self_exchange) << 1)) << 21
        own_idx = torch.empty(max(q, 1), dtype=torch.int32, device=dev)
        ws = torch.empty(eng.arc_own_ws_words(q), dtype=torch.int32, device=dev)
        eng.arc_count_async(G, keys, row[:G], me, own_idx, ws)
        mat = self._gather_row(row)  # mat[r, d] = rank r's keys for rank d
        self._agree(mat[:, G], 1)
        return mat, row[:G], own_idx

    @staticmethod
    def _max_crossing(mat, sx):
        """Largest count any rank sends any rank through the collectives."""
        G = mat.shape[0]
        return max([int(mat[r, d]) for r in range(G) for d in range(G) if r != d or sx] + [0])

    def _windows(self, k, n_list, out=None):
        """The n-windows of keys k (owners in this rank's arc) as global peer
        indices, and their counts (halo_ring): (lists int32 (m, n), count
        uint8 (m,)), written into out when given."""
        m = int(k.shape[0])
        if out is None:
            out = (torch.empty((m, n_list), dtype=torch.int32, device=k.device),
                   torch.empty(m, dtype=torch.uint8, device=k.device))
        if m == 0:
            return out
        sub, wrap = self.halo_ring(n_list - 1)
        ll, lc = sub.nsucc(k, n_list, out=out)
        if self.lo != wrap:  # local index j >= wrap is global lo + j - wrap
            ll.add_((ll >= wrap).to(ll.dtype) * (self.lo - wrap))
        return ll, lc

    def _nsucc_piece(self, keys, n_list, lists, count):
        """One piece: the count pass (device counts, this rank's own lookups'
        indices) and one all_gather; the own lookups' windows are read in place
        and written straight into the outputs, the others go out in the exact
        layout (own skipped), their windows come back and land through perm."""
        eng, G, me = self.engine, self.world, self.rank
        q = int(keys.shape[0])
        dev = keys.device
        mat, row, own_idx = self._count_gather(keys)
        sx = bool(self.self_exchange)
        c_me = 0 if sx else int(mat[me, me])
        direct = (lists.dtype == torch.int32 and count.dtype == torch.uint8 and lists.is_cuda
                  and lists.is_contiguous() and count.is_contiguous())
        if c_me == q and q and direct:  # every lookup is this rank's: straight into the outputs
            self._windows(keys, n_list, out=(lists, count))
        elif c_me == q and q:
            wl, wc = self._windows(keys, n_list)
            lists.copy_(wl.to(lists.dtype))
            count.copy_(wc.to(count.dtype))
        elif c_me:
            oi = own_idx[:c_me].long()
            wl, wc = self._windows(keys[oi], n_list)
            lists[oi] = wl.to(lists.dtype)
            count[oi] = wc.to(count.dtype)
        remote = any(int(mat[r, d]) for r in range(G) for d in range(G) if r != d or sx)
        if not remote:  # every rank sees the same matrix: all exchange or none do
            return
        send = [int(mat[me, d]) if d != me or sx else 0 for d in range(G)]
        recv = [int(mat[r, me]) if r != me or sx else 0 for r in range(G)]
        nr = self._rounds(self._max_crossing(mat, sx), max(16, 4 * (n_list + 1)))
        cursor = torch.empty(G, dtype=torch.int32, device=dev)
        sk, _, perm = eng.arc_scatter_async(G, self._zeros_src(keys), keys, row, cursor,
                                            skip=-1 if sx else me)
        cdev = self.comm_device if self.comm_device is not None else dev
        rk, work = self._a2a(sk[:sum(send)], recv, send, cdev, nr)
        rk = self._land(rk, work, sk)
        gl, gc = self._windows(rk, n_list)
        got = torch.cat([gl, gc.to(torch.int32).view(-1, 1)], dim=1)  # one exchange
        back, work = self._a2a(got.contiguous(), send, recv, cdev, nr)
        back = self._land(back, work, perm).to(lists.device)
        pm = perm.long()
        sel = pm >= 0
        rows = back[pm[sel]]
        lists[sel] = rows[:, :n_list].to(lists.dtype)
        count[sel] = rows[:, n_list].to(count.dtype)
        self.records_sent += sum(send)

    def _zeros_src(self, keys):
        z = getattr(self, "_zsrc", None)
        if z is None or z.shape[0] < keys.shape[0] or z.device != keys.device:
            z = torch.zeros(keys.shape[0], dtype=torch.int32, device=keys.device)
            self._zsrc = z
        return z[:keys.shape[0]]

    def _arc_ring(self):
        """This rank's arc of the ring as its own searchable ring (built once):
        the exact-successor mode holds only these IDs."""
        if getattr(self, "_arc", None) is None:
            self._arc = self.engine.arc_local_ring(self.lo, self.hi)
        return self._arc

    def route(self, src, keys, owner, hops, status=None, key_first=None, protocol=None) -> int:
        """Routes this rank's lookups (issued at peers src[i]); collective over
        the group.  Writes owner/hops/status at the lookups' indices and
        returns the number of rounds taken.

        key_first (default self.key_first): the origin does not walk; every
        NEW lookup goes straight to the rank whose arc holds its key's owner,
        which walks it from its source over the replicated top planes and its
        own lower planes (a walk that needs a lower level is within 2^Lh of its
        key, i.e. in that arc or its halo).  Otherwise the origin walks the top
        levels first (cx_arc_start) and forwards a WALK record."""
        if protocol is None:
            protocol = "soa" if (hasattr(self.engine, "arc_partition") and
                                 (key_first is None or key_first)) else "records"
        if protocol == "soa":
            return self.route_soa(src, keys, owner, hops, status)
        if protocol != "records":
            raise ValueError("protocol must be 'soa' or 'records'")
        kf = self.key_first if key_first is None else key_first
        start = getattr(self.engine, "arc_start", None)
        ahead = getattr(self.engine, "arc_send_ahead", None)
        recs = None if (start and not kf) or (kf and ahead) else \
            self.engine.arc_seed(self.rank, src, keys)
        for rnd in range(1, MAX_ROUNDS + 1):
            if kf and rnd == 1:  # send the lookups ahead by key
                if ahead:
                    send, counts = ahead(self.world, self.rank, src, keys)
                else:
                    send, counts = self.engine.arc_bucket(self.world, recs)
            else:
                if recs is None:  # first step straight from the lookups
                    out = start(self.rank, src, keys, owner, hops, status)
                else:
                    out = self.engine.arc_step(self.rank, recs, owner, hops, status)
                send, counts = self.engine.arc_bucket(self.world, out)
            self.records_sent += int(sum(counts))
            recs, inflight = self._exchange(send, counts)
            if inflight == 0:
                self.rounds = rnd
                return rnd
        raise RuntimeError("arc routing did not drain within MAX_ROUNDS rounds")
