"""Round-4 verdict item 2: no environment variable changes what the product
library computes.  The former A/B probe variables (CX_MISPLACED_PROBE,
CX_CZ2_MODE, CX_CZ2_WPE, CX_FINGERS_SEARCH, CX_FINGERS_ROWS, CX_JOIN_SORT,
CX_DIR_EXTRA, CX_CZ_CODES, CX_CZ_*, CX_IDA_*) were removed from libchordx.so;
a child process started with every one of them set computes the same route
table (route_table_hash), the same routes and the oracle's DHash maintenance
lists (dhash_peer.cpp:298-348) as this process without them.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

FORMER_PROBES = {
    "CX_MISPLACED_PROBE": "1", "CX_CZ2_MODE": "1", "CX_CZ2_WPE": "8", "CX_CZ2_NB": "16",
    "CX_FINGERS_SEARCH": "1", "CX_FINGERS_ROWS": "1", "CX_JOIN_SORT": "radix",
    "CX_DIR_EXTRA": "3", "CX_CZ_CODES": "hi", "CX_CZ_PAIR": "2", "CX_CZ_CHUNK": "8",
    "CX_CZ_STORE": "0", "CX_CZ_ROOTS_MODE": "1", "CX_CZ_ROOTS_SPLIT": "6",
    "CX_IDA_GENERIC": "1", "CX_IDA_ENC_D": "4", "CX_IDA_DEC_D": "1",
}

CHILD = r"""
import json, sys
import numpy as np
sys.path[:0] = [sys.argv[1] + "/p2p-dhts_amd", sys.argv[1] + "/oracle"]
import chordx, oracle as O
ids = O.splitmix_keys(0x5EED0A01, 1 << 18)
ring = chordx.Ring(ids)
ring.build_fingers()
keys = O.splitmix_keys(0x5EED0A02, 1 << 16)
src = (np.arange(1 << 16) * 7 % ring.n).astype(np.uint32)
owner, hops, status = ring.route(src, keys)
joins = O.splitmix_keys(0x5EED0A03, 2000)
leaves = O.ring_build(ids)[::131][:2000]
new, o2n = ring.churn(joins, leaves)
ol, oc, nl, nc, mask, tgt = ring.dhash_maintenance(new, o2n, keys, 14)
want_new, want_o2n = O.churn(O.ring_build(ids), joins, leaves)
wl, wc, wm, wt = O.misplaced(O.ring_build(ids), want_new, want_o2n, keys, 14)
ok = bool((o2n == want_o2n).all() and (nl == wl).all() and (nc == wc).all()
          and (mask == wm).all() and (tgt == wt).all())
print(json.dumps({"hash": ring.route_table_hash(), "escapes": ring.route_info()[1],
                  "owner_sum": int(owner.astype(np.uint64).sum()),
                  "hops_sum": int(hops.astype(np.uint64).sum()), "bad": int((status != 0).sum()),
                  "maintenance_equals_oracle": ok}))
"""


def run_child(env_extra):
    env = dict(os.environ)
    for k in FORMER_PROBES:
        env.pop(k, None)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_former_probe_variables_change_nothing():
    import chordx
    if chordx.device_count() == 0:
        pytest.fail("gpu test without a HIP device")
    plain = run_child({})
    probed = run_child(FORMER_PROBES)
    assert plain["maintenance_equals_oracle"] and probed["maintenance_equals_oracle"]
    assert plain["bad"] == 0
    assert probed == plain
