"""Ring-sort timing for rocprofv3 (round 6): 2^24 splitmix IDs (the bench
ring's seed), the default MSD sort and the 16-pass LSD sort, 3 runs each
(chordx.ring.sort_time); one JSON line."""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R + "/p2p-dhts_amd"]
import torch  # noqa: E402
import chordx  # noqa: E402
from chordx.ring import sort_time  # noqa: E402

lg = int(sys.argv[1]) if len(sys.argv) > 1 else 24
ids = torch.empty((1 << lg, 2), dtype=torch.int64, device="cuda")
chordx.fill_splitmix(ids, 0x5EED0005)
out = {}
for v in (0, 1):
    r = [sort_time(ids, v) for _ in range(3)]
    out[("msd", "lsd")[v]] = {"ms": [x[0] for x in r], "sorted": all(x[1] for x in r)}
print(json.dumps({"keys": 1 << lg, **out}), flush=True)
