"""Diagnostic: ArcRouter.nsucc (one-rank RCCL group, exchange_always) against
the ring's own cx_nsucc on the bench's C4 ring and keys; prints mismatches."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + "/p2p-dhts_amd"]
import torch  # noqa: E402
import chordx  # noqa: E402
from chordx import dist  # noqa: E402
from chordx.arc import ArcRouter  # noqa: E402

lg, lq = int(sys.argv[1]), int(sys.argv[2])
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
assert dist.init_single("nccl", dev)
ids = torch.empty((1 << lg, 2), dtype=torch.int64, device=dev)
chordx.fill_splitmix(ids, 0x5EED0005)
ring = chordx.Ring(ids)
ring.build_fingers()
keys = torch.empty((1 << lq, 2), dtype=torch.int64, device=dev)
chordx.fill_splitmix(keys, 0x5EED0006)
router = ArcRouter(ring, ring.n, 0, 1, exchange_always=True)
Q = keys.shape[0]
lists = torch.full((Q, 14), -1, dtype=torch.int32, device=dev)
cnt = torch.zeros(Q, dtype=torch.uint8, device=dev)
router.nsucc(keys, 14, lists, cnt)
torch.cuda.synchronize()
wl, wc = ring.nsucc(keys, 14)
torch.cuda.synchronize()
bad = (lists != wl.to(torch.int32)).any(dim=1) | (cnt != wc)
print("n", ring.n, "Q", Q, "mismatched keys", int(bad.sum()))
if int(bad.sum()):
    i = torch.nonzero(bad).flatten()[:4]
    for j in i.tolist():
        print(j, lists[j].tolist(), wl[j].tolist(), int(cnt[j]), int(wc[j]))
sub, wrap = router.halo_ring(13)
print("halo n", sub.n, "wrap", wrap)
s1 = sub.successor(keys)
s0 = ring.successor(keys)
print("successor mismatch on halo ring", int((s1 != s0).sum()))
l2, c2 = sub.nsucc(keys, 14)
print("nsucc mismatch on halo ring, direct", int(((l2 != wl).any(dim=1) | (c2 != wc)).sum()))
torch.distributed.destroy_process_group()
