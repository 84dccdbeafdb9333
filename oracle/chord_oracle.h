/*
 * chord_oracle.h -- CPU restatement of the reference's Chord/DHash lookup path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the HIP
 * engine in p2p-dhts_amd/.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product path never calls it.
 *
 * Every function restates one piece of Patrick-McKeever/P2P-DHTs (read-only at
 * /root/reference) and cites the file:line it follows.  The reference itself
 * cannot be compiled here (needs Boost.Multiprecision/UUID, jsoncpp, googletest
 * fetched over the network: src/CMakeLists.txt:4-14,38), so parity is pinned by
 * the reference's own JSON fixtures and key_test.cc vectors (tests/golden/).
 *
 * Arithmetic: ring values are unsigned 128-bit (GenericKey<16,32>, key.h:355).
 * InBetween's raw bound compare (key.h:121) and operator-'s uint256 wrap
 * (key.h:242-250) can produce non-canonical values, so the quirk-faithful
 * primitives take 256-bit operands (or_u256).
 */
#ifndef CHORD_ORACLE_H
#define CHORD_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef unsigned __int128 or_u128;
/* Little-endian 64-bit limbs: value = w[3]*2^192 + w[2]*2^128 + w[1]*2^64 + w[0]. */
typedef struct { uint64_t w[4]; } or_u256;
/* Same layout as the engine's cx_u128: value = hi*2^64 + lo. */
typedef struct { uint64_t lo, hi; } or_key;

#define OR_NONE 0xFFFFFFFFu
#define OR_FINGERS 128 /* ChordKey::BinaryLen() = log2(16)*32, key.h:152-155 */

/* Per-query route status (mirrors cx_status in include/chordx.h). */
#define OR_Q_OK 0
#define OR_Q_HOPCAP 1
#define OR_Q_NOT_FOUND 4 /* "ChordKey not found" (finger_table.h:129): no finger
                          for the key's range (OR_NONE entry = never added) */
#define OR_Q_FAILED 3 /* "Lookup failed" (chord_peer.cpp:206, dhash_peer.cpp:524) */
#define OR_FWD_CHORD 0 /* ChordPeer::ForwardRequest, chord_peer.cpp:185-211 */
#define OR_FWD_DHASH 1 /* DHashPeer::ForwardRequest, dhash_peer.cpp:500-529 */
#define OR_HOP_CAP 255

/* ---- a1: identifiers ------------------------------------------------- */
/* RFC-4122 UUIDv5 in the DNS namespace read as a big-endian 128-bit integer:
 * GenerateSha1Hash (key.h:29-33) + uint256_t(uuid) (key.h:77-78). */
or_key or_uuid5_dns(const char *name, size_t len);
void or_sha1(const uint8_t *msg, size_t len, uint8_t out[20]);

/* ---- a2/a3: ring arithmetic (256-bit raw operands) ------------------- */
/* GenericKey::InBetween, key.h:103-131, raw-bound semantics. */
int or_in_between(or_u256 v, or_u256 lb, or_u256 ub, int inclusive);
/* operator+(key, T) key.h:236-240: (v + t) mod 2^256 (uint256 add) then mod 2^128. */
or_u256 or_add_num(or_u256 v, uint64_t t);
/* operator-(key, T) key.h:242-250: diff = v - t in uint256 (wraps); diff>0 ? diff : 2^128+diff. */
or_u256 or_sub_num(or_u256 v, uint64_t t);
/* operator-(key, key) key.h:258-270: signed diff; diff>0 ? diff : 2^128+diff. */
or_u256 or_sub_key(or_u256 a, or_u256 b);
/* GetNthRange, finger_table.h:177-188: lb=(id+2^n) mod 2^128, ub=((id+2^(n+1)) mod 2^128)-1 in uint256. */
void or_nth_range(or_key id, int n, or_u256 *lb, or_u256 *ub);

/* ---- a13: ring order ------------------------------------------------- */
/* Sort ascending and drop equal IDs (RemotePeerList::Insert rejects equal IDs,
 * remote_peer_list.cpp:56-58).  Returns the unique count; out may alias ids. */
size_t or_ring_build(const or_key *ids, size_t n, or_key *out);

/* ---- a5/a7: converged successor -------------------------------------- */
/* succ(x) = first ring id >= x, wrapping to index 0 (converged StoredLocally,
 * abstract_chord_peer.cpp:720-725 with min_key = pred+1, chord_peer.cpp:275). */
uint32_t or_successor(const or_key *ring, size_t n, or_key key);
void or_successor_batch(const or_key *ring, size_t n, const or_key *keys, size_t q,
                        uint32_t *owner, int nthreads);

/* ---- a4/a6: fingers -------------------------------------------------- */
/* Converged PopulateFingerTable (abstract_chord_peer.cpp:564-613):
 * F[p*128+i] = succ(GetNthRange(i).first) of peer p. */
void or_fingers_build(const or_key *ring, size_t n, uint32_t *F, int nthreads);
/* Same, for peers [p0, p1) only, written to F[(p-p0)*128+i]. */
void or_fingers_rows(const or_key *ring, size_t n, size_t p0, size_t p1, uint32_t *F,
                     int nthreads);
/* FingerTable::Lookup (finger_table.h:115-130): first finger whose
 * [lb_i, ub_i] contains key under InBetween(..., true).  Returns the finger
 * index, or -1 ("ChordKey not found"). */
int or_finger_index(or_key id, or_key key);

/* GetPredecessor (abstract_chord_peer.cpp:380-421) on the converged ring. */
void or_predecessor_batch(const or_key *ring, size_t n, const or_key *keys, size_t q,
                          uint32_t *pred, int nthreads);

/* ---- a7-a9: routed lookup -------------------------------------------- */
/* Per-peer state a ChordPeer carries into GetSuccessor/ForwardRequest.
 * min_keys == NULL -> converged min_key = ring[p-1]+1 (ring[p]+1 when n==1,
 *                     StartChord abstract_chord_peer.cpp:69)
 * preds    == NULL -> converged predecessor ring[p-1] (OR_NONE when n==1).
 * alive    == NULL -> every peer's server answers (RemotePeer::IsAlive,
 *                     remote_peer.cpp:43-46); else alive[p] = 0/1.
 * succs    == NULL -> converged successors_ list: the next min(ns, n-1) peers
 *                     clockwise; else n*ns peer indices per list, OR_NONE-padded
 *                     (RemotePeerList, starting key = the peer's id, ctor
 *                     abstract_chord_peer.cpp:25).
 * rule: OR_FWD_CHORD / OR_FWD_DHASH -- which ForwardRequest's dead-finger
 *       branch applies. */
typedef struct {
    const or_key *ring;
    size_t n;
    const uint32_t *F;        /* n*128 finger successors (peer indices) */
    const or_key *min_keys;   /* optional */
    const uint32_t *preds;    /* optional; OR_NONE = no predecessor set */
    const uint8_t *alive;     /* optional */
    const uint32_t *succs;    /* optional */
    int ns;                   /* successor-list length (num_succs_) */
    int rule;
} or_peers;

/* GetSuccessor (abstract_chord_peer.cpp:318-330) recursing through
 * ChordPeer::ForwardRequest (chord_peer.cpp:185-211).  Hops = number of
 * GET_SUCC requests sent (0 when the source stores the key).  Returns OR_Q_*. */
int or_route(const or_peers *P, uint32_t src, or_key key, uint32_t *owner, uint8_t *hops);
void or_route_batch(const or_peers *P, const uint32_t *src, const or_key *keys, size_t q,
                    uint32_t *owner, uint8_t *hops, uint8_t *status, int nthreads);
/* or_route on the raw uint256 key hi:lo (a wire key of 33-64 hex digits). */
void or_route_raw_batch(const or_peers *P, const uint32_t *src, const or_key *lo,
                        const or_key *hi, size_t q, uint32_t *owner, uint8_t *hops,
                        uint8_t *status);

/* ---- a10/a11: n successors ------------------------------------------- */
/* GetNSuccessors (abstract_chord_peer.cpp:345-373): n routed lookups from src,
 * stop at the first repeat.  Writes up to n peer indices, returns the count. */
int or_nsucc(const or_peers *P, uint32_t src, or_key key, int n, uint32_t *list);
void or_nsucc_batch(const or_peers *P, const uint32_t *src, const or_key *keys, size_t q,
                    int n, uint32_t *lists, uint8_t *count, int nthreads);

/* ---- a12: churn + misplaced scan ------------------------------------- */
/* New ring = sort/dedupe((old minus leaves) + joins).  old_to_new[p] = new index
 * of surviving old peer p, OR_NONE for a departed one.  Returns new size;
 * new_ring must hold n_old + nj entries. */
size_t or_churn(const or_key *old_ring, size_t n_old, const or_key *joins, size_t nj,
                const or_key *leaves, size_t nl, or_key *new_ring, uint32_t *old_to_new);
/* DHashPeer::RunGlobalMaintenance (dhash_peer.cpp:298-348) restated per key.
 * Holders = old window of key (its n successors on the old ring, the replica
 * set DHashPeer::Create placed, dhash_peer.cpp:103-129), surviving ones mapped
 * to the new ring.  For each holder rank j (old-list order): misplaced iff the
 * holder survived and is not in the new n-list; its target is the rank in the
 * new list of the first successor not already holding the key (0xFF if all
 * hold it: the reference then keeps the key, dhash_peer.cpp:331-338). */
void or_misplaced(const or_key *old_ring, size_t n_old, const or_key *new_ring, size_t n_new,
                  const uint32_t *old_to_new, const or_key *keys, size_t q, int n,
                  uint32_t *new_lists, uint8_t *count, uint16_t *mask, uint8_t *target,
                  int nthreads);

/* General form: explicit holders (q x nh ring indices, OR_NONE = empty), as in
 * DHashGlobalMaintenance.MisplacedKeys (dhash_test.cpp:123-149) where keys are
 * inserted straight into a non-owner's db.  nh <= 16 (mask is 16-bit). */
/* C5 CPU baseline: placement and maintenance lists by routed GetNSuccessors
 * on the old and new rings (lookups from peer q mod n), misplaced check. */
void or_maintenance_routed(const or_peers *P_old, const or_peers *P_new, const uint32_t *old_to_new,
                           const or_key *keys, size_t q, int n, uint32_t *old_lists,
                           uint8_t *old_count, uint32_t *new_lists, uint8_t *count,
                           uint16_t *mask, uint8_t *target, int nthreads);
void or_misplaced_holders(const or_key *ring, size_t n_ring, const or_key *keys, size_t q,
                          const uint32_t *holders, int nh, int n, uint32_t *new_lists,
                          uint8_t *count, uint16_t *mask, uint8_t *target, int nthreads);

/* Test helpers. */
void or_splitmix_keys(uint64_t seed, size_t offset, size_t count, or_key *out);
double or_now(void);

#ifdef __cplusplus
}
#endif
#endif
