"""Regenerate the committed golden vectors under tests/golden/.

Run in the build container (where /root/reference exists):

    python tests/golden/make_golden.py

Two outputs:

* reference_vectors.json -- DATA extracted from the reference's own test
  fixtures (test/test_json/**) and the literal operands/expectations of
  test/key_test.cc.  Inputs and expected outputs only; no reference source is
  copied.  Each record cites the fixture/test it came from.
* c1_truth.json -- config C1 ground truth produced by our CPU oracle
  (oracle/chord_oracle.c): 8 peers 127.0.0.1:5000-5007, keys key0..key999, every
  key routed from every peer (pattern of chord_test.cpp:704-714).  Hop counts
  are not instrumented anywhere in the reference, so this file
  is pinned only by the oracle's literal restatement of chord_peer.cpp:185-211.
"""
from __future__ import annotations

import json
import os
import sys
import uuid

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
FIX = os.path.join(REF, "test", "test_json")


def uuid5_hex(name: str) -> str:
    return format(int.from_bytes(uuid.uuid5(uuid.NAMESPACE_DNS, name).bytes, "big"), "x")


def load(rel):
    with open(os.path.join(FIX, rel)) as f:
        return json.load(f)


def peer_name(p):
    return f"{p.get('IP', p.get('IP_ADDR'))}:{p['PORT']}"


def collect_ids():
    """Every (ip:port, ID) pair in the fixtures.  The reference builds peers
    from ip:port (abstract_chord_peer.cpp:21), so a fixture ID equal to
    UUIDv5(ip:port) is a hashing vector; the rest are hand-written synthetic IDs
    (e.g. fff...f successors, the stale NO_CHANGES_NEEDED block)."""
    derived, synthetic = [], []

    def walk(o, path, f):
        if isinstance(o, dict):
            if "ID" in o and "PORT" in o:
                rec = {"name": peer_name(o), "id": o["ID"], "fixture": f"{f}:{path}"}
                (derived if uuid5_hex(rec["name"]) == o["ID"] else synthetic).append(rec)
            for k, v in o.items():
                walk(v, f"{path}/{k}", f)
        elif isinstance(o, list):
            for i, v in enumerate(o):
                walk(v, f"{path}[{i}]", f)

    for dirpath, _, files in sorted(os.walk(FIX)):
        for fn in sorted(files):
            rel = os.path.relpath(os.path.join(dirpath, fn), FIX)
            walk(load(rel), "", "test/test_json/" + rel)
    return derived, synthetic


def key_test_vectors():
    """Operands and expectations of test/key_test.cc (transcribed as data).
    `bits` = ring size in bits: EightBitKey = GenericKey<2, 8> (key_test.cc:5),
    ChordKey = GenericKey<16, 32> (key.h:355)."""
    ops = [
        # KeyOpTest.* (key_test.cc:10-40): key op key == expected
        {"test": "KeyOpTest.AdditionNoModulo", "bits": 8, "op": "+", "a": 16, "b": 15, "expect": 31},
        {"test": "KeyOpTest.AdditionWithModulo", "bits": 8, "op": "+", "a": 128, "b": 128, "expect": 0},
        {"test": "KeyOpTest.SubstractionNoModulo", "bits": 8, "op": "-", "a": 16, "b": 15, "expect": 1},
        {"test": "KeyOpTest.SubstractionWithModulo", "bits": 8, "op": "-", "a": 0, "b": 1, "expect": 255},
    ]
    h = lambda s: int(s, 16)  # noqa: E731
    inb = [
        # KeyInBetweenTest.* (key_test.cc:44-87): key.InBetween(lb, ub, incl) == expect
        {"test": "KeyInBetweenTest.ExclusiveNoModulo", "v": 75, "lb": 0, "ub": 99, "incl": False, "expect": True},
        {"test": "KeyInBetweenTest.ExclusiveNoModulo", "v": 99, "lb": 0, "ub": 99, "incl": False, "expect": False},
        {"test": "KeyInBetweenTest.ExclusiveWithModulo", "v": 1, "lb": 75, "ub": 25, "incl": False, "expect": True},
        {"test": "KeyInBetweenTest.ExclusiveWithModulo", "v": 25, "lb": 75, "ub": 25, "incl": False, "expect": False},
        {"test": "KeyInBetweenTest.InclusiveNoModulo", "v": 75, "lb": 0, "ub": 99, "incl": True, "expect": True},
        {"test": "KeyInBetweenTest.InclusiveNoModulo", "v": 99, "lb": 0, "ub": 99, "incl": True, "expect": True},
        {"test": "KeyInBetweenTest.InclusiveWithModulo", "v": 1, "lb": 75, "ub": 25, "incl": True, "expect": True},
        {"test": "KeyInBetweenTest.InclusiveWithModulo", "v": 25, "lb": 75, "ub": 25, "incl": True, "expect": True},
        {"test": "KeyInBetweenTest.DifferingLengths", "v": h("f4ee136cb4059b2883450e7e93698be"),
         "lb": h("633bd46b5c515992a5ce553d0680bec9"), "ub": h("f4ee136cb4059b2883450e7e93698bd"),
         "incl": True, "expect": False},
    ]
    for r in inb:
        for k in ("v", "lb", "ub"):
            r[k] = format(r[k], "x")
    return ops, inb


def join_placement():
    """ChordIntegration.Join (chord_test.cpp:645-683): keys key0..key9 created
    from peer 0 land on the peer listed in EXPECTED_KV_PAIRS; each peer's
    EXPECTED_PREDECESSOR_ID is its ring predecessor."""
    d = load("chord_tests/ChordIntegrationJoinTest.json")
    value_to_plain = {v: k for k, v in d["KV_PAIRS"].items()}
    peers, keys = [], []
    for p in d["PEERS"]:
        peers.append({"name": peer_name(p), "id": uuid5_hex(peer_name(p)),
                      "expected_pred": p["EXPECTED_PREDECESSOR_ID"]})
        for hashed, val in p["EXPECTED_KV_PAIRS"].items():
            keys.append({"plain": value_to_plain[val], "hash": hashed,
                         "owner": uuid5_hex(peer_name(p))})
    return {"source": "chord_test.cpp:645-683 + ChordIntegrationJoinTest.json",
            "peers": peers, "keys": keys}


def stabilize_succs():
    """ChordIntegration.Stabilize (chord_test.cpp:722-742): each peer's first 3
    successors after one stabilize cycle."""
    d = load("chord_tests/ChordIntegrationStabilizeTest.json")
    return {"source": "chord_test.cpp:722-742 + ChordIntegrationStabilizeTest.json",
            "n": 3,
            "peers": [{"name": peer_name(p), "id": uuid5_hex(peer_name(p)),
                       "expected_succs": p["EXPECTED_SUCCS"]} for p in d["PEERS"]]}


def node_failure():
    """ChordIntegration.NodeFailure (chord_test.cpp:783-817): peers 0 and 1 fail;
    survivors' min_key, predecessor and 3 successors after re-stabilisation."""
    d = load("chord_tests/ChordIntegrationNodeFailureTest.json")
    out = {"source": "chord_test.cpp:783-817 + ChordIntegrationNodeFailureTest.json",
           "failed": [0, 1], "n": 3, "peers": []}
    for i, p in enumerate(d["PEERS"]):
        rec = {"name": peer_name(p), "id": uuid5_hex(peer_name(p))}
        if i >= 2:
            rec.update({"expected_min_key": p["EXPECTED_MINKEY"],
                        "expected_pred": p["EXPECTED_PREDECESSOR_ID"],
                        "expected_succs": p["EXPECTED_SUCCS"][:3]})
        out["peers"].append(rec)
    return out


def update_succ():
    """ChordUpdateSuccList.* (chord_test.cpp:389-483): peer 0's successor list
    (NUM_SUCCS entries) after JOINING_PEERS join.  NO_CHANGES_NEEDED is skipped:
    its fixture IDs are stale (not UUIDv5 of their ports), so the peers the test
    actually builds are not the ones it expects."""
    d = load("chord_tests/UpdateSuccTest.json")
    cases = []
    for name in ("SINGLE_NODE_BETWEEN_SUCCS", "MULTIPLE_NODES_BETWEEN_SUCCS",
                 "CLOCKWISE_EXPANSION_NEEDED"):
        c = d[name]
        cases.append({
            "case": name,
            "n": c["PEERS"][0]["NUM_SUCCS"],
            "initial": [uuid5_hex(peer_name(p)) for p in c["PEERS"]],
            "joining": [uuid5_hex(peer_name(p)) for p in c["JOINING_PEERS"]],
            "tested": uuid5_hex(peer_name(c["PEERS"][0])),
            "expected_succs": [e["ID"] for e in c["EXPECTED_SUCCS"]],
        })
    return {"source": "chord_test.cpp:389-483 + UpdateSuccTest.json", "cases": cases}


def get_succ():
    """ChordGetSucc.* (chord_test.cpp:18-123)."""
    d = load("chord_tests/GetSuccTest.json")
    loc = d["GET_SUCC_OF_LOCAL_KEY"]
    ft = d["GET_SUCC_FROM_FINGER_TABLE"]
    pr = d["GET_SUCC_FROM_PREDECESSOR"]
    fa = d["GET_SUCC_FAILING"]
    return {
        "source": "chord_test.cpp:18-123 + GetSuccTest.json",
        # LocalKey: a lone peer with min_key set to 0 owns [0, id]; the key is local.
        # (The fixture's min-key field is spelled MINKEY while the test reads
        # MIN_KEY, chord_test.cpp:27, so the test actually sets min_key = "" ->
        # uint256("0x") = 0; both readings give 0.)
        "local_key": {"peer": uuid5_hex(peer_name(loc["PEER"])), "min_key": "0",
                      "key": loc["KEY_TO_LOOKUP"], "expected": uuid5_hex(peer_name(loc["PEER"]))},
        # FromFingerTable: 2-peer ring, lookup from peer 0 resolves via its finger table.
        "from_finger_table": {"peers": [uuid5_hex(peer_name(p)) for p in ft["PEERS"]],
                              "src": uuid5_hex(peer_name(ft["PEERS"][0])),
                              "key": ft["KEY_TO_LOOKUP"], "expected": ft["EXPECTED_SUCC_ID"]},
        # FromPredecessor: every finger of peer 0 points at itself (AdjustFingers,
        # chord_test.cpp:80-83) -> ForwardRequest substitutes the predecessor.
        "from_predecessor": {"peers": [uuid5_hex(peer_name(p)) for p in pr["PEERS"]],
                             "src": uuid5_hex(peer_name(pr["PEERS"][0])),
                             "key": pr["KEY_TO_LOOKUP"]},
        # Failing (chord_test.cpp:101-123): a constructed (server running,
        # StartChord never called) peer whose predecessor_ and only successor
        # are a peer that does not answer (port 1); AdjustFingers(succ) runs on
        # an empty finger table.  EXPECT_ANY_THROW(GetSuccessor(key)).
        "failing": {"peer": uuid5_hex(peer_name(fa["PEER"])),
                    "num_succs": fa["PEER"]["NUM_SUCCS"],
                    "dead_succ": fa["PEER"]["SUCCESSOR"]["ID"],
                    "dead_succ_min_key": fa["PEER"]["SUCCESSOR"]["MIN_KEY"],
                    "dead_succ_port": fa["PEER"]["SUCCESSOR"]["PORT"],
                    "key": fa["KEY_TO_LOOKUP"]},
    }


def get_pred():
    """ChordGetPred.* (chord_test.cpp:131-227) on converged rings."""
    d = load("chord_tests/GetPredTest.json")
    sl = d["GET_PRED_IN_SUCC_LIST"]
    ft = d["GET_PRED_FROM_FINGER_TABLE"]
    return {
        "source": "chord_test.cpp:131-227 + GetPredTest.json",
        # FromSuccList: 3-peer ring, key just below a peer's ID
        "in_succ_list": {"peers": [uuid5_hex(peer_name(p)) for p in sl["PEERS"]],
                         "key": sl["KEY_TO_LOOKUP"], "expected": sl["EXPECTED_PRED_ID"]},
        # FromFingerTable: 2-peer ring, key just above a peer's ID (owner wraps)
        "from_finger_table": {"peers": [uuid5_hex(peer_name(p)) for p in ft["PEERS"]],
                              "key": ft["KEY_TO_LOOKUP"], "expected": ft["EXPECTED_PRED_ID"]},
    }


def global_maintenance():
    """DHashGlobalMaintenance.MisplacedKeys (dhash_test.cpp:123-149): n=2
    (SetIdaParams(2,1,257)); keys 0x50..00-08 inserted into TESTED_IND's db; after
    RunGlobalMaintenance its db is empty (hash "0") and CORRECT_SUCC_IND holds them."""
    d = load("dhash_tests/GlobalMaintenanceTest.json")["MISPLACED_KEYS"]
    return {"source": "dhash_test.cpp:123-149 + GlobalMaintenanceTest.json",
            "n": 2,
            "peers": [uuid5_hex(peer_name(p)) for p in d["PEERS"]],
            "fixture_ids": [p["ID"] for p in d["PEERS"]],
            "keys": list(d["KEYS_TO_INSERT"].keys()),
            "holder": d["PEERS"][d["TESTED_IND"]]["ID"],
            "expected_target": d["PEERS"][d["CORRECT_SUCC_IND"]]["ID"],
            "expected_holder_db_hash": d["EXPECTED_TESTED_HASH"]}


def dhash_create_read():
    """DHashIntegration.CreateAndRead (dhash_test.cpp:213-226): 28 peers, n=14,
    key "key1": ring + plaintext key for the replica-list test (expected list =
    14 successors, asserted by the oracle)."""
    d = load("dhash_tests/DHashIntegrationCreateAndReadTest.json")
    return {"source": "dhash_test.cpp:213-226 + DHashIntegrationCreateAndReadTest.json",
            "peers": [uuid5_hex(peer_name(p)) for p in d["PEERS"]],
            "n": d["PEERS"][0]["NUM_SUCCS"], "key": d["KEY"]}


def ida_values():
    """Data the reference's DHash tests store through IDA, with the (n, m, p)
    each test uses: DataBlock defaults (14, 10, 257) (data_block.h:33-34) in
    DHashIntegration.CreateAndRead and DHashExchangeNode; SetIdaParams(2, 1,
    257) in DHashGlobalMaintenance; (3, 2, 257) in DHashSynchronize
    (dhash_test.cpp:20-150,185-226).  Reading a key back must return it."""
    out = []
    d = load("dhash_tests/DHashIntegrationCreateAndReadTest.json")
    out.append({"source": "dhash_test.cpp:213-226", "nmp": [14, 10, 257], "values": [d["VAL"]]})
    d = load("dhash_tests/ExchangeNodeTest.json")
    out.append({"source": "dhash_test.cpp:185-205", "nmp": [14, 10, 257],
                "values": list(d["NON_EXISTENT_NODE"]["KEYS_TO_INSERT"].values())})
    d = load("dhash_tests/GlobalMaintenanceTest.json")
    out.append({"source": "dhash_test.cpp:123-149", "nmp": [2, 1, 257],
                "values": list(d["MISPLACED_KEYS"]["KEYS_TO_INSERT"].values())})
    d = load("dhash_tests/LocalMaintenanceTest.json")
    vals = [d["DEPTH_ONE_SINGLE_KEY"]["VAL_TO_INSERT"],
            d["SYNCHRONIZE_USES_GIVEN_RANGE"]["VAL_TO_INSERT"]]
    vals += list(d["HIGH_DEPTH"]["KEYS_TO_INSERT"].values())
    out.append({"source": "dhash_test.cpp:20-110", "nmp": [3, 2, 257], "values": vals})
    return out


def c1_truth():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O

    names = [f"127.0.0.1:{5000 + j}" for j in range(8)]
    ring = O.ring_build(O.keys_from_ints([O.uuid5_key(s) for s in names]))
    F = O.fingers(ring)
    P = O.Peers(ring, F)
    keys_plain = [f"key{i}" for i in range(1000)]
    kv = O.keys_from_ints([O.uuid5_key(s) for s in keys_plain])
    q = len(keys_plain) * len(ring)
    src = np.repeat(np.arange(len(ring), dtype=np.uint32), len(keys_plain))
    kk = np.tile(kv, (len(ring), 1))
    owner, hops, status = O.route(P, src, kk)
    assert status.max() == 0
    lists, count = O.nsucc(P, kv, 3)
    return {
        "source": "oracle/chord_oracle.c (or_route, or_nsucc); SURVEY 8(d) C1",
        "peers": names,
        "ring": [format(v, "x") for v in O.ints_from_keys(ring)],
        "keys": keys_plain,
        "n_lookups": q,
        "src_major": "lookup j = src (j // 1000), key (j % 1000)",
        "owner": owner.tolist(),
        "hops": hops.tolist(),
        "nsucc3": lists.tolist(),
        "mean_hops": float(hops.mean()),
    }


def main():
    derived, synthetic = collect_ids()
    ops, inb = key_test_vectors()
    vec = {
        "reference": "Patrick-McKeever/P2P-DHTs (test/test_json/**, test/key_test.cc)",
        "generator": "tests/golden/make_golden.py",
        "id_hash": derived,
        "id_synthetic": synthetic,
        "key_ops": ops,
        "in_between": inb,
        "join_placement": join_placement(),
        "stabilize_succs": stabilize_succs(),
        "node_failure": node_failure(),
        "update_succ": update_succ(),
        "get_succ": get_succ(),
        "get_pred": get_pred(),
        "global_maintenance": global_maintenance(),
        "dhash_create_read": dhash_create_read(),
        "ida_values": ida_values(),
    }
    with open(os.path.join(HERE, "reference_vectors.json"), "w") as f:
        json.dump(vec, f, indent=1)
    with open(os.path.join(HERE, "c1_truth.json"), "w") as f:
        json.dump(c1_truth(), f)
    print(f"id vectors: {len(derived)} derived, {len(synthetic)} synthetic")


if __name__ == "__main__":
    main()
