#!/usr/bin/env python3
"""IDA encode/decode on 1 GiB (4 KiB blocks), for rocprofv3 kernel traces/PMC."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "p2p-dhts_amd"))
import torch  # noqa: E402

from chordx import ida  # noqa: E402

nb, bl = 1 << 18, 4096
g = torch.Generator(device="cuda").manual_seed(1)
data = torch.randint(0, 256, (nb * bl,), dtype=torch.uint8, device="cuda", generator=g)
offs = torch.arange(0, nb * bl + 1, bl, dtype=torch.int64, device="cuda")
frags, seg = ida.encode_flat(data, offs)
S = (bl + 9) // 10
keep = torch.tensor([0, 2, 3, 5, 6, 8, 9, 11, 12, 13], device="cuda")
rows = frags.view(nb, 14, S)[:, keep, :].contiguous().view(-1)
idx = (keep + 1).to(torch.uint8).repeat(nb).contiguous()
dec = ida.decode_flat(rows, seg, idx)
for _ in range(int(os.environ.get("REPS", "5"))):
    ida.encode_flat(data, offs, seg_offsets=seg, out=frags)
    ida.decode_flat(rows, seg, idx, out=dec)
torch.cuda.synchronize()
print("ok")
