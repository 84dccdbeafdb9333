"""Diagnostic (round 6): what made the single-piece 2^25-key
return exchange of ArcRouter.nsucc come back half empty on a one-rank RCCL
group (commit 9ac284c).

Part A -- RCCL alone: list all_to_all (one view per rank, as ArcRouter._a2a),
all_to_all_single, and a 2-D (rows, 15) int32 buffer (the placement rows),
around and above 2^31 bytes; each output starts at a sentinel and is compared
in full with the input after work.wait().
Part B -- the 9ac284c _nsucc_piece path restated (partition -> exchange ->
halo-ring windows -> 60-B rows -> return exchange -> perm), at 2^24 and 2^25
keys, with and without a device synchronisation before each collective.
One JSON line per case on stdout."""
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + "/p2p-dhts_amd"]
import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(0)
import chordx  # noqa: E402
from chordx import dist  # noqa: E402

assert dist.init_single("nccl", dev)
part = sys.argv[1] if len(sys.argv) > 1 else "AB"


def emit(**kw):
    print(json.dumps(kw), flush=True)


def check(out, src, sentinel):
    torch.cuda.synchronize()
    ne = out != src
    bad = int(ne.sum())
    first = int(torch.nonzero(ne.flatten())[0]) if bad else -1
    untouched = int((out == sentinel).sum())
    return bad, first, untouched


MB = 1 << 20
SIZES = {"A": (1 << 30, 2013265920, (1 << 31) - 4 * MB, 1 << 31, (1 << 31) + 4 * MB,
               3 << 30, (1 << 32) + 4 * MB),
         # the threshold between 2^30 (whole) and 2013265920 (half)
         "S": (1 << 30, (1 << 30) + 4, (1 << 30) + 64 * 1024, (1 << 30) + 4 * MB)
         + tuple((1 << 30) + k * 64 * MB for k in range(1, 16))}
for P in ("A", "S"):
    if P not in part:
        continue
    for nbytes in SIZES[P]:
        n = nbytes // 4
        src = (torch.arange(n, dtype=torch.int64, device=dev) * 2654435761 % 2147483629).to(torch.int32)
        for kind in ("list", "single", "rows15"):
            if kind == "rows15" and n % 15:
                continue
            out = torch.full_like(src, -7)
            t0 = time.time()
            if kind == "list":
                w = tdist.all_to_all([out], [src], async_op=True)
            elif kind == "single":
                w = tdist.all_to_all_single(out, src, output_split_sizes=[n],
                                            input_split_sizes=[n], async_op=True)
            else:
                s2, o2 = src.view(-1, 15), out.view(-1, 15)
                w = tdist.all_to_all(list(torch.split(o2, [o2.shape[0]])),
                                     list(torch.split(s2, [s2.shape[0]])), async_op=True)
            try:
                w.wait()
                bad, first, untouched = check(out, src, -7)
                emit(part=P, kind=kind, nbytes=nbytes, elems=n, mismatched=bad,
                     first_bad=first, untouched=untouched, s=round(time.time() - t0, 3))
            except Exception as e:  # report and go on to the next size
                emit(part=P, kind=kind, nbytes=nbytes, error=repr(e)[:300])
            del out
        del src
        torch.cuda.empty_cache()

if "B" in part:
    lg = 24
    ids = torch.empty((1 << lg, 2), dtype=torch.int64, device=dev)
    chordx.fill_splitmix(ids, 0x5EED0005)
    ring = chordx.Ring(ids)
    ring.build_fingers()
    ring.arc_build(1, 0)  # the one-rank arc layout arc_partition reads
    sub = chordx.Ring(ring.ids_device().clone())  # the halo ring of a one-rank group: the whole ring
    for lq in (24, 25):
        keys = torch.empty((1 << lq, 2), dtype=torch.int64, device=dev)
        chordx.fill_splitmix(keys, 0x5EED0006)
        q = keys.shape[0]
        wl, wc = ring.nsucc(keys, 14)
        for sync in (False, True):
            zero = torch.zeros(q, dtype=torch.int32, device=dev)
            sk, _, perm, counts = ring.arc_partition(1, zero, keys)[:4]
            if sync:
                torch.cuda.synchronize()
            rk = torch.empty_like(sk)
            w = tdist.all_to_all(list(torch.split(rk, [q])), list(torch.split(sk, [q])),
                                 async_op=True)
            w.wait()
            ll, lc = sub.nsucc(rk, 14)
            got = torch.cat([ll.to(torch.int32), lc.to(torch.int32).view(-1, 1)], dim=1).contiguous()
            if sync:
                torch.cuda.synchronize()
            back = torch.empty_like(got)
            w = tdist.all_to_all(list(torch.split(back, [q])), list(torch.split(got, [q])),
                                 async_op=True)
            w.wait()
            rows_equal = int((back == got).all(dim=1).sum())
            res = back[perm.long()]
            ok_keys = int(((res[:, :14] == wl.to(torch.int32)).all(dim=1) &
                           (res[:, 14] == wc.to(torch.int32))).sum())
            torch.cuda.synchronize()
            emit(part="B", keys=q, ret_bytes=int(got.numel() * 4), sync=sync,
                 return_rows_equal=rows_equal, keys_equal_cx_nsucc=ok_keys,
                 forward_equal=bool((rk == sk).all()))
            del got, back, res, rk, ll, lc
            torch.cuda.empty_cache()
        del keys, wl, wc
tdist.destroy_process_group()
