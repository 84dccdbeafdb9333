"""Pin the CPU oracle against the reference's own fixtures (CPU only).

Every vector here comes from tests/golden/reference_vectors.json, which
make_golden.py extracted from /root/reference/test/test_json/** and
test/key_test.cc.  The oracle is trusted as the GPU parity checker only
because these pass.
"""
import numpy as np
import pytest

H = lambda s: int(s, 16)  # noqa: E731


# ---------------------------------------------------------------- a1: IDs
def test_uuid5_ids_match_reference_fixtures(O, refvec):
    """103 ip:port -> ID pairs (abstract_chord_peer.cpp:21, key.h:29-33)."""
    assert len(refvec["id_hash"]) == 103
    for rec in refvec["id_hash"]:
        assert format(O.uuid5_key(rec["name"]), "x") == rec["id"], rec["fixture"]
        assert format(O.uuid5_int(rec["name"]), "x") == rec["id"]


def test_synthetic_fixture_ids_are_not_hashes(O, refvec):
    # the 10 hand-written IDs (fff..f, e000..0, stale block) are not UUIDv5 of their ports
    for rec in refvec["id_synthetic"]:
        assert format(O.uuid5_key(rec["name"]), "x") != rec["id"]


def test_key_hashes_join_fixture(O, refvec):
    for k in refvec["join_placement"]["keys"]:
        assert format(O.uuid5_key(k["plain"]), "x") == k["hash"]


# ---------------------------------------------------------------- a2/a3
def test_key_ops_key_test_cc(O, refvec):
    """KeyOpTest.* (key_test.cc:10-40) on GenericKey<2, 8>."""
    for r in refvec["key_ops"]:
        a = O.GenericKey(r["a"], 2, r["bits"])
        b = O.GenericKey(r["b"], 2, r["bits"])
        got = a + b if r["op"] == "+" else a - b
        assert got.value == r["expect"], r["test"]


def test_in_between_key_test_cc(O, refvec):
    """KeyInBetweenTest.* (key_test.cc:44-87): C oracle and Python twin."""
    for r in refvec["in_between"]:
        v, lb, ub = H(r["v"]), H(r["lb"]), H(r["ub"])
        assert O.in_between(v, lb, ub, r["incl"]) == r["expect"], r["test"]
        assert O.GenericKey(v).in_between(lb, ub, r["incl"]) == r["expect"], r["test"]


def test_in_between_quirks_c_vs_python(O):
    """Raw-bound compare (key.h:121) and equal-bound point test (key.h:108-113)."""
    rng = np.random.default_rng(7)
    special = [0, 1, 2, (1 << 128) - 1, 1 << 128, (1 << 128) + 1, (1 << 256) - 1, 1 << 127]
    vals = special + [int(x) for x in rng.integers(0, 1 << 62, 20)] + \
        [int.from_bytes(rng.bytes(16), "big") for _ in range(20)]
    for v in vals[:16]:
        for lb in vals[::3]:
            for ub in vals[1::3]:
                for inc in (True, False):
                    assert O.in_between(v, lb, ub, inc) == O.GenericKey(v).in_between(lb, ub, inc)


def test_sub_quirks():
    """operator- (key.h:242-270): 1-1 -> 2^128 (non-canonical); 0-1 wraps in uint256."""
    import oracle as O
    assert (O.GenericKey(1) - 1).value == 1 << 128
    assert (O.GenericKey(0) - 1).value == (1 << 256) - 1
    assert (O.GenericKey(5) - O.GenericKey(5)).value == 1 << 128
    assert ((O.GenericKey(0) - 1) + 1).value == 0


# ---------------------------------------------------------------- a4/a5
def test_finger_index_equals_msb(O):
    """FingerTable::Lookup's linear first match == floor(log2((key - id) mod 2^128))."""
    rng = np.random.default_rng(3)
    for _ in range(400):
        pid = int.from_bytes(rng.bytes(16), "big")
        d = int.from_bytes(rng.bytes(16), "big") >> int(rng.integers(0, 128))
        if d == 0:
            d = 1
        key = (pid + d) % (1 << 128)
        assert O.finger_index(pid, key) == d.bit_length() - 1
    assert O.finger_index(5, 5) == -1  # key == id: "ChordKey not found"
    assert O.finger_index((1 << 128) - 2, (1 << 128) - 1) == 0
    assert O.finger_index((1 << 128) - 1, 0) == 0


def test_nth_range_wrap_bound():
    """GetNthRange upper bound: ((id + 2^128) mod 2^128) - 1 -> 2^256-1 raw when 0."""
    import oracle as O
    lb, ub = O.nth_range(0, 127)
    assert lb == 1 << 127 and ub == (1 << 256) - 1
    lb, ub = O.nth_range(3, 0)
    assert lb == ub == 4


# ---------------------------------------------------------------- placement
def _ring(O, ids):
    return O.ring_build(O.keys_from_ints(ids))


def test_join_placement(O, refvec):
    """ChordIntegration.Join: 10 keys land on the expected peers (lower_bound+wrap),
    and each peer's predecessor is its ring predecessor."""
    jp = refvec["join_placement"]
    ring = _ring(O, [H(p["id"]) for p in jp["peers"]])
    ids = [format(v, "x") for v in O.ints_from_keys(ring)]
    keys = O.keys_from_ints([H(k["hash"]) for k in jp["keys"]])
    owner = O.successor(ring, keys)
    assert [ids[o] for o in owner] == [k["owner"] for k in jp["keys"]]
    # routed from peer 0 (the test creates from peers[0]) with converged fingers
    P = O.Peers(ring, O.fingers(ring))
    src0 = ids.index(jp["peers"][0]["id"])
    o2, _, st = O.route(P, np.full(len(keys), src0, np.uint32), keys)
    assert (o2 == owner).all() and (st == 0).all()
    for p in jp["peers"]:
        i = ids.index(p["id"])
        assert ids[(i - 1) % len(ids)] == p["expected_pred"]


def test_stabilize_successor_lists(O, refvec):
    st = refvec["stabilize_succs"]
    ring = _ring(O, [H(p["id"]) for p in st["peers"]])
    ids = [format(v, "x") for v in O.ints_from_keys(ring)]
    P = O.Peers(ring, O.fingers(ring))
    for p in st["peers"]:
        # the successor list of peer id = GetNSuccessors(id + 1, n)
        key = O.keys_from_ints([(H(p["id"]) + 1) % (1 << 128)])
        lists, cnt = O.nsucc(P, key, st["n"], src=[ids.index(p["id"])])
        assert [ids[x] for x in lists[0][: cnt[0]]] == p["expected_succs"]


def test_node_failure_churn_leave(O, refvec):
    nf = refvec["node_failure"]
    all_ids = [H(p["id"]) for p in nf["peers"]]
    ring = _ring(O, all_ids)
    leaves = O.keys_from_ints([all_ids[i] for i in nf["failed"]])
    new_ring, o2n = O.churn(ring, O.keys_from_ints([]), leaves)
    assert len(new_ring) == len(all_ids) - len(nf["failed"])
    ids = [format(v, "x") for v in O.ints_from_keys(new_ring)]
    P = O.Peers(new_ring, O.fingers(new_ring))
    for p in nf["peers"][2:]:
        i = ids.index(p["id"])
        pred = ids[(i - 1) % len(ids)]
        assert pred == p["expected_pred"]
        assert format((H(pred) + 1) % (1 << 128), "x") == p["expected_min_key"]
        lists, cnt = O.nsucc(P, O.keys_from_ints([(H(p["id"]) + 1) % (1 << 128)]), nf["n"],
                             src=[i])
        assert [ids[x] for x in lists[0][: cnt[0]]] == p["expected_succs"]


def test_update_succ_churn_join(O, refvec):
    for c in refvec["update_succ"]["cases"]:
        ring = _ring(O, [H(x) for x in c["initial"]])
        new_ring, o2n = O.churn(ring, O.keys_from_ints([H(x) for x in c["joining"]]),
                                O.keys_from_ints([]))
        ids = [format(v, "x") for v in O.ints_from_keys(new_ring)]
        i = ids.index(c["tested"])
        P = O.Peers(new_ring, O.fingers(new_ring))
        lists, cnt = O.nsucc(P, O.keys_from_ints([(H(c["tested"]) + 1) % (1 << 128)]), c["n"],
                             src=[i])
        assert [ids[x] for x in lists[0][: cnt[0]]] == c["expected_succs"], c["case"]
        # surviving old peers keep their identity under old_to_new
        old_ids = [format(v, "x") for v in O.ints_from_keys(ring)]
        for p, q in enumerate(o2n):
            assert ids[q] == old_ids[p]


# ---------------------------------------------------------------- routing
def test_get_succ_local_key(O, refvec):
    g = refvec["get_succ"]["local_key"]
    ring = _ring(O, [H(g["peer"])])
    P = O.Peers(ring, O.fingers(ring), min_keys=O.keys_from_ints([H(g["min_key"])]))
    owner, hops, st = O.route(P, [0], O.keys_from_ints([H(g["key"])]))
    assert owner[0] == 0 and hops[0] == 0 and st[0] == 0


def test_get_succ_from_finger_table(O, refvec):
    g = refvec["get_succ"]["from_finger_table"]
    ring = _ring(O, [H(x) for x in g["peers"]])
    ids = [format(v, "x") for v in O.ints_from_keys(ring)]
    P = O.Peers(ring, O.fingers(ring))
    owner, hops, st = O.route(P, [ids.index(g["src"])], O.keys_from_ints([H(g["key"])]))
    assert ids[owner[0]] == g["expected"] and hops[0] == 1


def test_get_succ_from_predecessor(O, refvec):
    """Every finger of the source points at itself -> ForwardRequest forwards to
    the predecessor (chord_peer.cpp:195-197); the key is found there."""
    g = refvec["get_succ"]["from_predecessor"]
    ring = _ring(O, [H(x) for x in g["peers"]])
    ids = [format(v, "x") for v in O.ints_from_keys(ring)]
    s = ids.index(g["src"])
    F = O.fingers(ring)
    F[s, :] = s
    P = O.Peers(ring, F)
    owner, hops, st = O.route(P, [s], O.keys_from_ints([H(g["key"])]))
    assert owner[0] == (s - 1) % len(ids) and hops[0] == 1 and st[0] == 0


def test_hop_cap_when_no_predecessor(O):
    """Fingers all self and no live predecessor: the reference forwards to itself
    forever; the oracle stops at 255 forwards with OR_Q_HOPCAP."""
    ring = O.ring_build(O.splitmix_keys(11, 4))
    F = O.fingers(ring)
    F[0, :] = 0
    preds = np.array([O.NONE, 0, 1, 2], np.uint32)
    P = O.Peers(ring, F, preds=preds)
    key = O.keys_from_ints([(O.ints_from_keys(ring)[2])])
    owner, hops, st = O.route(P, [0], key)
    assert st[0] == 1 and hops[0] == 255 and owner[0] == O.NONE


def test_c1_truth_reproduces(O, c1truth):
    """C1 ground truth: 8 peers, key0..key999 routed from every peer."""
    ring = O.ring_build(O.keys_from_ints([O.uuid5_key(n) for n in c1truth["peers"]]))
    assert [format(v, "x") for v in O.ints_from_keys(ring)] == c1truth["ring"]
    P = O.Peers(ring, O.fingers(ring))
    kv = O.keys_from_ints([O.uuid5_key(k) for k in c1truth["keys"]])
    src = np.repeat(np.arange(len(ring), dtype=np.uint32), len(kv))
    owner, hops, st = O.route(P, src, np.tile(kv, (len(ring), 1)))
    assert owner.tolist() == c1truth["owner"] and hops.tolist() == c1truth["hops"]
    assert (owner == np.tile(O.successor(ring, kv), len(ring))).all()


def test_route_owner_is_lower_bound(O):
    ring = O.ring_build(O.splitmix_keys(0x5EED0001, 3000))
    P = O.Peers(ring, O.fingers(ring))
    keys = O.splitmix_keys(0x5EED0002, 20000)
    src = (np.arange(20000) * 7919 % len(ring)).astype(np.uint32)
    owner, hops, st = O.route(P, src, keys)
    assert (owner == O.successor(ring, keys)).all() and (st == 0).all()
    assert hops.max() <= 12


# ---------------------------------------------------------------- DHash
def test_nsucc_window(O):
    for n_ring in (1, 2, 3, 13, 14, 15, 200):
        ring = O.ring_build(O.splitmix_keys(n_ring, n_ring))
        P = O.Peers(ring, O.fingers(ring))
        keys = O.splitmix_keys(99, 300)
        lists, cnt = O.nsucc(P, keys, 14, src=np.arange(300) % n_ring)
        s = O.successor(ring, keys)
        for q in range(300):
            k = min(14, n_ring)
            assert cnt[q] == k
            assert lists[q, :k].tolist() == [(s[q] + j) % n_ring for j in range(k)]


def test_dhash_create_read_replicas(O, refvec):
    """DHashIntegration.CreateAndRead: 28 peers, n=14: key1's fragment list is the
    14-peer window (asserted literally by GetNSuccessors from every peer)."""
    d = refvec["dhash_create_read"]
    ring = _ring(O, [H(x) for x in d["peers"]])
    assert len(ring) == 28
    P = O.Peers(ring, O.fingers(ring))
    key = O.keys_from_ints([O.uuid5_key(d["key"])])
    s = O.successor(ring, key)[0]
    for src in range(28):
        lists, cnt = O.nsucc(P, key, d["n"], src=[src])
        assert cnt[0] == 14 and lists[0].tolist() == [(s + j) % 28 for j in range(14)]


def test_global_maintenance_fixture(O, refvec):
    """DHashGlobalMaintenance.MisplacedKeys: every key held by 4c55.. is misplaced
    (n=2 list = [c7ac, cd0a]) and goes to CORRECT_SUCC_IND (c7ac); holder empties."""
    g = refvec["global_maintenance"]
    assert g["peers"] == g["fixture_ids"]
    ring = _ring(O, [H(x) for x in g["peers"]])
    ids = [format(v, "x") for v in O.ints_from_keys(ring)]
    keys = O.keys_from_ints([H(k) for k in g["keys"]])
    holders = np.full((len(keys), 1), ids.index(g["holder"]), np.uint32)
    lists, cnt, mask, target = O.misplaced_holders(ring, keys, holders, g["n"])
    assert (mask == 1).all()  # holder 0 misplaced for every key -> db emptied ("0" hash)
    for q in range(len(keys)):
        assert ids[lists[q, target[q, 0]]] == g["expected_target"]


def test_misplaced_churn_semantics(O):
    old = O.ring_build(O.splitmix_keys(5, 60))
    joins = O.splitmix_keys(6, 3)
    leaves = old[[3, 10, 11, 40]]
    new, o2n = O.churn(old, joins, leaves)
    assert len(new) == 60 - 4 + 3
    assert (o2n[[3, 10, 11, 40]] == O.NONE).all()
    keys = O.splitmix_keys(7, 2000)
    lists, cnt, mask, target = O.misplaced(old, new, o2n, keys, 14)
    s_old = O.successor(old, keys)
    s_new = O.successor(new, keys)
    for q in range(2000):
        newlist = [(s_new[q] + j) % len(new) for j in range(14)]
        assert lists[q].tolist() == newlist
        holders = [o2n[(s_old[q] + j) % 60] for j in range(14)]
        has = {h for h in holders if h in newlist}
        for j, h in enumerate(holders):
            mis = h != O.NONE and h not in newlist
            assert bool(mask[q] >> j & 1) == mis
            if mis:
                free = [r for r in range(14) if newlist[r] not in has]
                if free:
                    assert target[q, j] == free[0]
                    has.add(newlist[free[0]])
                else:
                    assert target[q, j] == 0xFF
            else:
                assert target[q, j] == 0xFF


def test_churn_rejects_duplicate_join(O):
    old = O.ring_build(O.splitmix_keys(8, 10))
    joins = np.concatenate([old[[2]], O.splitmix_keys(9, 2), O.splitmix_keys(9, 1)])
    new, o2n = O.churn(old, joins, O.keys_from_ints([]))
    assert len(new) == 12  # join equal to old[2] and the repeated join are rejected
    new_ids, old_ids = O.ints_from_keys(new), O.ints_from_keys(old)
    assert len(set(new_ids)) == 12 and new_ids == sorted(new_ids)
    assert all(new_ids[o2n[p]] == old_ids[p] for p in range(10))


# ---- a9: ForwardRequest's dead-finger branch (chord_peer.cpp:193-208,
# dhash_peer.cpp:505-526) --------------------------------------------------
def failing_state(O, g, fill_fingers, rule):
    """ChordGetSucc.Failing (chord_test.cpp:101-123) as peer state: peer P
    (127.0.0.1:7003) was constructed -- its server answers, min_key_ = id_
    (abstract_chord_peer.cpp:21-22) -- but never started a chord, so its finger
    table is empty; its predecessor_ and only successor are `succ` (port 1,
    never answers).  AdjustFingers(succ) walks the empty table and changes
    nothing.  fill_fingers=True is the state the test's comment intends (every
    finger = succ)."""
    p_id, s_id = H(g["peer"]), H(g["dead_succ"])
    ring = _ring(O, [p_id, s_id])
    ids = O.ints_from_keys(ring)
    p, sd = ids.index(p_id), ids.index(s_id)
    F = np.full((2, 128), O.NONE, np.uint32)
    if fill_fingers:
        F[p, :] = sd
    min_keys = [0, 0]
    min_keys[p], min_keys[sd] = p_id, H(g["dead_succ_min_key"])
    preds = np.full(2, O.NONE, np.uint32)
    preds[p] = sd
    alive = np.zeros(2, np.uint8)
    alive[p] = 1
    succs = np.full((2, g["num_succs"]), O.NONE, np.uint32)
    succs[p, 0] = sd
    return ring, p, dict(F=F, min_keys=O.keys_from_ints(min_keys), preds=preds, alive=alive,
                         succs=succs, rule=rule)


@pytest.mark.parametrize("rule", [0, 1])
def test_get_succ_failing_literal(O, refvec, rule):
    """The literal test state: GetSuccessor throws -- from FingerTable::Lookup
    over the empty table ("ChordKey not found", finger_table.h:129)."""
    g = refvec["get_succ"]["failing"]
    ring, p, st = failing_state(O, g, False, rule)
    P = O.Peers(ring, **st)
    owner, hops, status = O.route(P, [p], O.keys_from_ints([H(g["key"])]))
    assert status[0] == O.Q_NOT_FOUND and owner[0] == O.NONE and hops[0] == 0


@pytest.mark.parametrize("rule", [0, 1])
def test_get_succ_failing_dead_finger(O, refvec, rule):
    """Every finger = the dead succ: not self -> IsAlive fails -> Chord:
    successors_.Lookup(0) finds succ (the wrapped range (id_P, succ]) dead;
    DHash: LookupLiving gives none, successors_[0] is dead -> "Lookup failed"."""
    g = refvec["get_succ"]["failing"]
    ring, p, st = failing_state(O, g, True, rule)
    P = O.Peers(ring, **st)
    owner, hops, status = O.route(P, [p], O.keys_from_ints([H(g["key"])]))
    assert status[0] == O.Q_FAILED and owner[0] == O.NONE and hops[0] == 0


def _five_peer(O, dead, rule):
    ring = O.keys_from_ints([k << 124 for k in range(1, 6)])
    alive = np.ones(5, np.uint8)
    alive[list(dead)] = 0
    return O.Peers(ring, O.fingers(ring), alive=alive, ns=3, rule=rule)


@pytest.mark.parametrize("dead,rule,want", [
    # key in (id2, id3]; from peer 0 the walk is 0 -> 2 -> 3 when all answer
    ((), 0, (3, 1 + 1, 0)),
    ((2,), 0, (3, 1, 0)),        # finger 2 dead: successors_.Lookup -> 3 (alive)
    ((2,), 1, (3, 1, 0)),        # LookupLiving -> 3
    ((3,), 0, (None, 1, 3)),     # at 2: finger 3 dead, list lookup 3 dead -> failed
    ((3,), 1, (None, 1, 3)),     # LookupLiving none, successors_[0] = 3 dead
    ((2, 3), 0, (None, 0, 3)),   # Chord: list lookup gives dead 3 at the source
    ((2, 3), 1, (None, 1, 3)),   # DHash: successors_[0] = 1 alive -> at 1 both dead
])
def test_dead_finger_fallback_hand_derived(O, dead, rule, want):
    P = _five_peer(O, dead, rule)
    owner, hops, status = O.route(P, [0], O.keys_from_ints([0x38 << 120]))
    w_owner, w_hops, w_st = want
    assert status[0] == w_st and hops[0] == w_hops
    assert owner[0] == (O.NONE if w_owner is None else w_owner)


def test_lookup_living_scan_never_runs(O):
    """RemotePeerList::LookupLiving's scan for a later living entry has a
    condition that is false on entry (remote_peer_list.cpp:123): with the found
    entry dead and a live one after it, DHash still falls back to
    successors_[0] rather than the later living entry."""
    ring = O.keys_from_ints([k << 124 for k in range(1, 6)])
    F = O.fingers(ring)
    alive = np.array([1, 1, 0, 0, 1], np.uint8)
    succs = np.array([[2, 3, 4], [2, 3, 4], [3, 4, 0], [4, 0, 1], [0, 1, 2]], np.uint32)
    # peer 0's list starts at a dead peer: successors_[0] dead too -> failed,
    # although entry 4 (alive) follows the dead 3 in the list
    P = O.Peers(ring, F, alive=alive, succs=succs, rule=1)
    owner, hops, status = O.route(P, [0], O.keys_from_ints([0x38 << 120]))
    assert status[0] == O.Q_FAILED and hops[0] == 0


@pytest.mark.parametrize("case", ["in_succ_list", "from_finger_table"])
def test_get_pred_fixture(O, refvec, case):
    """ChordGetPred.FromSuccList / FromFingerTable (chord_test.cpp:154-209):
    the converged ring's answer is the key owner's predecessor."""
    g = refvec["get_pred"][case]
    ring = _ring(O, [H(x) for x in g["peers"]])
    ids = [format(v, "x") for v in O.ints_from_keys(ring)]
    pred = O.predecessor(ring, O.keys_from_ints([H(g["key"])]))
    assert ids[pred[0]] == g["expected"]


def test_get_pred_lone_peer_is_itself(O):
    """A lone peer has no predecessor set and answers itself
    (abstract_chord_peer.cpp:383-385; ChordGetPred.LocalKey's one-peer ring)."""
    ring = _ring(O, [0xfffffffffffffffffffffffffffffff])
    assert (O.predecessor(ring, O.keys_from_ints([1 << 120, 0, 5])) == 0).all()


def test_maintenance_routed_equals_window_restatement(O):
    """C5's CPU baseline (or_maintenance_routed: placement and maintenance
    lists by routed GetNSuccessors, abstract_chord_peer.cpp:345-373, then
    RunGlobalMaintenance's check, dhash_peer.cpp:298-348) equals the
    converged-window restatement the GPU parity tests use (or_misplaced,
    or_nsucc) on a churned ring."""
    old = O.ring_build(O.splitmix_keys(0xC5A0, 3000))
    joins, leaves = O.splitmix_keys(0xC5A1, 60), old[::50][:60]
    new, o2n = O.churn(old, joins, leaves)
    keys = O.splitmix_keys(0xC5A2, 4000)
    Po, Pn = O.Peers(old, O.fingers(old)), O.Peers(new, O.fingers(new))
    ol, oc, nl, nc, mask, tg = O.maintenance_routed(Po, Pn, o2n, keys, 14)
    wl, wc, wm, wt = O.misplaced(old, new, o2n, keys, 14)
    xl, xc = O.nsucc(Po, keys, 14)
    assert (nl == wl).all() and (nc == wc).all() and (mask == wm).all() and (tg == wt).all()
    assert (ol == xl).all() and (oc == xc).all()
    assert int((mask != 0).sum()) > 0
