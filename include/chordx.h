/*
 * chordx.h -- C ABI of the MI355X batched Chord/DHash lookup engine.
 *
 * Drop-in boundary for the lookup hot path of Patrick-McKeever/P2P-DHTs.
 * The reference has no FFI layer: the path sits behind C++ class interfaces
 * (FingerTable<PeerType>, ChordKey::InBetween, AbstractChordPeer::GetSuccessor /
 * GetNSuccessors, DHashPeer::RunGlobalMaintenance).  Each entry point below
 * names the reference interface it replaces (file:line under /root/reference).
 * INTEGRATION.md shows the binding a ChordPeer/DHashPeer maintainer would add.
 *
 * Conventions
 *  - 128-bit ring values are cx_u128 {lo, hi}: value = hi * 2^64 + lo
 *    (ChordKey = GenericKey<16,32>, key.h:355, ring size 16^32 = 2^128).
 *  - Peers are named by their index in the sorted ring (cx_ring_ids maps
 *    index -> ID); the reference names them by RemotePeer (id, ip, port).
 *  - Every call returns CX_OK (0) or a CX_E_* code; cx_last_error() gives a
 *    thread-local message.  Error texts reuse the reference's runtime_error
 *    messages where one exists ("Lookup failed", "Insufficient succs in list
 *    to complete request.", ...).
 *  - memkind CX_MEM_HOST: caller buffers are host memory; the engine stages
 *    them.  CX_MEM_DEVICE: caller buffers are device pointers on the ring's
 *    device and the call is asynchronous on the ring's stream (cx_ring_sync).
 *  - A ring handle is immutable once built (fingers/state uploads excepted,
 *    which are exclusive writes like the reference's WriteLock'ed
 *    FingerTable edits, finger_table.h:91-168).  Const queries from several
 *    host threads are safe if each thread uses its own handle stream.
 *  - No compute path exists on the host: without a HIP device every compute
 *    call fails with CX_E_HIP.
 */
#ifndef CHORDX_H
#define CHORDX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CHORDX_VERSION 1
#define CX_FINGERS 128u          /* ChordKey::BinaryLen(), key.h:152-155; finger_table.h:44 */
#define CX_NONE 0xFFFFFFFFu      /* "no peer" index */
#define CX_HOP_CAP 255u          /* max forwards recorded per lookup (uint8 hops) */
#define CX_MAX_NSUCC 16          /* n-successor list cap (uint16 misplaced mask) */

typedef struct { uint64_t lo, hi; } cx_u128;
typedef struct { uint64_t w[4]; } cx_u256; /* little-endian limbs, raw uint256_t values */
typedef struct cx_ring cx_ring;

enum cx_err {
    CX_OK = 0,
    CX_E_INVALID = 1,      /* bad argument */
    CX_E_NOT_FOUND = 2,    /* "ChordKey not found" (finger_table.h:129) */
    CX_E_LOOKUP_FAILED = 3,/* "Lookup failed" (chord_peer.cpp:206, dhash_peer.cpp:524) */
    CX_E_INSUFFICIENT = 4, /* "Insufficient succs in list to complete request." (dhash_peer.cpp:110) */
    CX_E_HIP = 5,          /* HIP runtime failure or no device */
    CX_E_RCCL = 6,
    CX_E_NOMEM = 7,
    CX_E_STATE = 8         /* operation needs state not built yet (e.g. fingers) */
};

enum cx_memkind { CX_MEM_HOST = 0, CX_MEM_DEVICE = 1 };

/* Per-query status of cx_route (the reference throws; a batch reports them
 * per lookup and does not fail as a whole). */
enum cx_qstatus {
    CX_Q_OK = 0,
    CX_Q_HOPCAP = 1,    /* more than CX_HOP_CAP forwards (the reference livelocks) */
    CX_Q_BADPEER = 2,   /* src >= ring size */
    CX_Q_FAILED = 3,    /* "Lookup failed" (chord_peer.cpp:206, dhash_peer.cpp:524) */
    CX_Q_NOT_FOUND = 4  /* "ChordKey not found": no finger for the key's range
                           (finger_table.h:129, table not populated) */
};

/* Which ForwardRequest's dead-finger fallback the literal walk applies. */
enum cx_fwd_rule {
    CX_FWD_CHORD = 0, /* ChordPeer::ForwardRequest, chord_peer.cpp:185-211 */
    CX_FWD_DHASH = 1  /* DHashPeer::ForwardRequest, dhash_peer.cpp:500-529 */
};

/* ---- library --------------------------------------------------------- */
int cx_version(void);
const char *cx_last_error(void);
/* Number of visible HIP devices (0 without a GPU; never fails). */
int cx_device_count(int *count);
/* Table pool: a destroyed ring's large tables (finger table, route tables,
 * arc planes, build and churn temporaries >= 64 KiB) are kept per process, up to
 * CX_POOL_CAP_GIB GiB (environment, default 96, 0 = off), for the next ring of
 * the same size -- a membership epoch reuses the previous epoch's HBM.  Any
 * allocation that fails releases the device's idle blocks and retries.
 * cx_pool_trim releases every idle block now (all devices), and the idle
 * device staging buffers of host-memory calls (one process-wide cache, at most
 * 64 MiB idle); cx_pool_info reports the idle table blocks and their bytes. */
int cx_pool_trim(void);
int cx_pool_info(uint64_t *blocks, uint64_t *bytes);

/* ---- ring lifecycle (a13) ---------------------------------------------
 * Replaces the converged RemotePeerList/successor ring that Join/Stabilize/
 * UpdateSuccList build over RPC (abstract_chord_peer.cpp:83-117,460-562;
 * remote_peer_list.cpp:31-84): LSD radix sort of the IDs on the GPU, equal
 * IDs dropped (remote_peer_list.cpp:56-58).  n >= 1. */
int cx_ring_create(const cx_u128 *ids, size_t n, int memkind, int device, cx_ring **out);
int cx_ring_destroy(cx_ring *ring);
int cx_ring_size(const cx_ring *ring, size_t *n);
/* Sorted unique IDs (index -> ID map), n entries. */
int cx_ring_ids(const cx_ring *ring, cx_u128 *out, int memkind);
/* Device pointer to the ring's sorted IDs (n x 16 B, read-only). */
int cx_ring_ids_device(const cx_ring *ring, const cx_u128 **ids);
/* Enqueue the handle's work on the caller's hipStream_t (NULL = the device's
 * null stream); cx_ring_use_own_stream restores the handle's private stream. */
int cx_ring_set_stream(cx_ring *ring, void *hip_stream);
int cx_ring_use_own_stream(cx_ring *ring);
int cx_ring_sync(const cx_ring *ring);

/* ---- a5/a7: exact successor --------------------------------------------
 * owner[i] = index of the peer whose StoredLocally(keys[i]) holds in the
 * converged ring (abstract_chord_peer.cpp:720-725, min_key = pred+1,
 * chord_peer.cpp:275): the first ID >= key, wrapping to 0.  Default search: a
 * bucket directory over the top ID bits (one gather answers most keys); A/B
 * alternatives: Eytzinger with LDS-staged top levels. */
int cx_successor(const cx_ring *ring, const cx_u128 *keys, size_t q, uint32_t *owner,
                 int memkind);

/* GetPredecessor(key) (abstract_chord_peer.cpp:380-421) on the converged
 * ring: the owner's predecessor, pred[i] = (owner(keys[i]) + n - 1) mod n --
 * what StoredLocally's predecessor_, the successor-list shortcut and the
 * forwarded GET_PRED all return there (a lone peer is its own predecessor). */
int cx_predecessor(const cx_ring *ring, const cx_u128 *keys, size_t q, uint32_t *pred,
                   int memkind);

/* ---- a4/a6: fingers ----------------------------------------------------
 * Converged PopulateFingerTable (abstract_chord_peer.cpp:564-613): row p,
 * entry i = succ(GetNthRange(i).first) = succ(id_p + 2^i mod 2^128)
 * (finger_table.h:177-188).  The table stays on the device for cx_route;
 * fingers_out (n x 128 uint32, may be NULL) receives a copy.  With
 * fingers_out NULL on a ring of 2^18 peers or more, the build hands the
 * default route table only the finger levels it reads and writes the
 * row-major table when it is first read (cx_fingers_device, fingers_out of a
 * later build, a literal or non-default walk, cx_arc_build): the same table,
 * 8 GiB fewer bytes on the churn -> route-ready path at 2^24. */
int cx_fingers_build(cx_ring *ring, uint32_t *fingers_out, int memkind);
/* Hand-edited / churned finger table (EditNthFinger, AdjustFingers,
 * ReplaceDeadPeer: finger_table.h:137-168), n x 128 peer indices; CX_NONE =
 * no finger added for that range (a table PopulateFingerTable never filled:
 * lookups through it report CX_Q_NOT_FOUND).  Validated before it replaces
 * the current table (a rejected upload changes nothing).  Switches cx_route
 * to the literal ForwardRequest walk. */
int cx_fingers_upload(cx_ring *ring, const uint32_t *fingers, int memkind);
/* Device pointer to the n x 128 finger table (NULL until built/uploaded);
 * a deferred table is written first (the call returns when it is complete). */
int cx_fingers_device(const cx_ring *ring, const uint32_t **fingers);
/* Per-peer min_key_ and predecessor_ (CX_NONE = predecessor not set, never
 * alive), as white-box tests set them (chord_test.cpp:18-123).  Either may be
 * NULL (= converged value: pred+1 / ring[p-1]).  Validated before it replaces
 * the current state.  Switches cx_route to the literal walk. */
int cx_peer_state_upload(cx_ring *ring, const cx_u128 *min_keys, const uint32_t *preds,
                         int memkind);
/* Peer liveness and successor lists for ForwardRequest's dead-finger branch
 * (chord_peer.cpp:193-208, dhash_peer.cpp:505-526).  alive: n bytes, 0 = the
 * peer's server does not answer (RemotePeer::IsAlive, remote_peer.cpp:43-46;
 * a Fail()ed peer, chord_peer.cpp:293-300), NULL = all alive.  succ_lists:
 * n x ns peer indices in list order, CX_NONE-padded (successors_, a
 * RemotePeerList whose starting key is the peer's id, abstract_chord_peer.cpp:
 * 25), NULL = the converged lists (next min(ns, n-1) peers clockwise).
 * forward_rule: cx_fwd_rule.  0 <= ns <= 64.  Validated before it replaces the
 * current state; switches cx_route to the literal walk.  alive == NULL and
 * succ_lists == NULL together reset the ring to "every peer alive, converged
 * lists": the literal walk is dropped again (unless cx_peer_state_upload or
 * cx_fingers_upload state remains) and the arc calls accept the ring. */
int cx_liveness_upload(cx_ring *ring, const uint8_t *alive, const uint32_t *succ_lists, int ns,
                       int forward_rule, int memkind);

/* ---- a7-a9: finger-routed lookup with hop counts -------------------------
 * GetSuccessor(key) issued at peer src[i] (abstract_chord_peer.cpp:318-330),
 * forwarded hop by hop through ChordPeer::ForwardRequest (chord_peer.cpp:
 * 185-211): FingerTable::Lookup's first matching finger (finger_table.h:
 * 115-130), self -> live predecessor substitution, dead finger -> successor
 * list (cx_liveness_upload).  hops[i] = GET_SUCC requests sent (0 if src
 * stores the key).  status[i] = cx_qstatus; owner = CX_NONE unless CX_Q_OK.
 * status may be NULL.  Needs fingers (cx_fingers_build or cx_fingers_upload). */
int cx_route(const cx_ring *ring, const uint32_t *src, const cx_u128 *keys, size_t q,
             uint32_t *owner, uint8_t *hops, uint8_t *status, int memkind);

/* ---- a10/a11: n-successor replica lists -----------------------------------
 * GetNSuccessors(key, n) (abstract_chord_peer.cpp:345-373) as used for DHash
 * fragment placement (dhash_peer.cpp:103-129): lists[i*n + j] = j-th
 * successor, count[i] = min(n, ring size), unused slots CX_NONE.  1 <= n <= 16. */
int cx_nsucc(const cx_ring *ring, const cx_u128 *keys, size_t q, int n, uint32_t *lists,
             uint8_t *count, int memkind);
/* DHashPeer::Create's precondition (dhash_peer.cpp:109-112): CX_E_INSUFFICIENT
 * when the ring has fewer than m peers (every key then gets < m successors). */
int cx_dhash_check(const cx_ring *ring, int n, int m);

/* ---- a12: churn + global-maintenance misplaced scan ------------------------
 * Batched join/leave: new ring = (old minus leaves) + joins, sorted, equal IDs
 * dropped (a join equal to a surviving ID is rejected).  Leaves not in the ring
 * are ignored.  old_to_new[p] = new index of old peer p or CX_NONE if it left
 * (may be NULL).  All buffers in memkind. */
int cx_churn(const cx_ring *old_ring, const cx_u128 *joins, size_t nj, const cx_u128 *leaves,
             size_t nl, int memkind, cx_ring **new_ring, uint32_t *old_to_new);
/* DHashPeer::RunGlobalMaintenance (dhash_peer.cpp:298-348) after churn, per
 * key.  Holders = the key's old n-window (DHashPeer::Create placed fragment j
 * on old list rank j), survivors mapped by old_to_new.  Outputs (q x n unless
 * noted): new_lists = new n-successor lists; count[q]; mask[q] bit j = old
 * holder j is misplaced (survived, not in its new list, dhash_peer.cpp:
 * 322-328); target[j] = rank in new_lists of the successor holder j's
 * CREATE_KEY goes to (first successor lacking the key, holders processed in
 * rank order), 0xFF if none (every successor already holds it).
 * old_to_new is in memkind and may come from cx_churn. */
int cx_misplaced(const cx_ring *old_ring, const cx_ring *new_ring, const uint32_t *old_to_new,
                 const cx_u128 *keys, size_t q, int n, uint32_t *new_lists, uint8_t *count,
                 uint16_t *mask, uint8_t *target, int memkind);
/* C5's step in one pass over the keys: cx_nsucc(old_ring, keys, n) into
 * old_lists / old_count (DHashPeer::Create's placement on the pre-churn ring,
 * dhash_peer.cpp:103-129) + cx_misplaced (RunGlobalMaintenance,
 * dhash_peer.cpp:298-348).  Outputs equal the two calls' outputs; the scan
 * already resolves each key's old successor, so the placement costs only its
 * list stores.  All buffers in memkind. */
int cx_dhash_maintenance(const cx_ring *old_ring, const cx_ring *new_ring,
                         const uint32_t *old_to_new, const cx_u128 *keys, size_t q, int n,
                         uint32_t *old_lists, uint8_t *old_count, uint32_t *new_lists,
                         uint8_t *count, uint16_t *mask, uint8_t *target, int memkind);
/* Same scan with explicit holders (q x nh ring indices, CX_NONE = empty), e.g.
 * keys inserted straight into a non-owner's db (dhash_test.cpp:123-149).
 * target is q x nh.  nh <= 16. */
int cx_misplaced_holders(const cx_ring *ring, const cx_u128 *keys, size_t q,
                         const uint32_t *holders, int nh, int n, uint32_t *new_lists,
                         uint8_t *count, uint16_t *mask, uint8_t *target, int memkind);

/* ---- a2: clockwise interval test ----------------------------------------
 * ChordKey::InBetween(lb, ub, inclusive) (key.h:103-131) on raw uint256
 * operands (its raw-bound compare and equal-bound point test included),
 * batched on the GPU: out[i] = 0/1. */
int cx_in_between(const cx_u256 *v, const cx_u256 *lb, const cx_u256 *ub, size_t q,
                  int inclusive, uint8_t *out, int memkind);

/* ---- a1: identifiers ------------------------------------------------------
 * out[i] = UUIDv5(DNS namespace, name_i) read as a big-endian 128-bit integer:
 * the ID a ChordPeer gets from "ip:port" (abstract_chord_peer.cpp:21) and a key
 * gets from ChordKey(plaintext, hashed = false) (key.h:29-33,76-79).  Names
 * are concatenated in `bytes`; name i = bytes[offsets[i] .. offsets[i+1]),
 * offsets has count + 1 entries.  SHA-1 runs on the GPU (one lane per name). */
int cx_uuid5_dns(const uint8_t *bytes, const uint64_t *offsets, size_t count, cx_u128 *out,
                 int memkind, int device);

/* ---- synthetic inputs (bench / tests) --------------------------------------
 * out[i] = {splitmix64(seed, 2(offset+i)), splitmix64(seed, 2(offset+i)+1)}
 * written on the device (SURVEY 8d generator). */
int cx_fill_splitmix(cx_u128 *out_device, size_t count, uint64_t seed, uint64_t offset,
                     int device, void *hip_stream);

/* ---- hex codec of keys on the wire ----------------------
 * cx_hex_parse: ChordKey(hex, hashed = true) = uint256("0x" + s) (key.h:73-75)
 * for each string bytes[offsets[i] .. offsets[i+1]); digits of either case, no
 * prefix.  out = value mod 2^128 (the engine's ring value); ok[i] = 1 for a
 * raw value < 2^128, 2 for a raw value >= 2^128 (33+ significant digits; the
 * raw uint256 wraps mod 2^256 like Boost's unchecked cpp_int -- over 64 digits
 * parity unpinned), 0 for an empty string or a non-hex character (where
 * boost's parse throws).  The raw value only matters to InBetween's point
 * test (key.h:108-113); cx_wire applies that corner (cx_wire.cpp wide_keys).
 * cx_hex_format: std::string(key) = IntToHexStr (key.h:41-47) -- lowercase,
 * no leading zeros, "0" for zero -- into out[32 i .. 32 i + len[i]), the rest of
 * each 32-byte slot zero.  Both run on the GPU. */
int cx_hex_parse(const uint8_t *bytes, const uint64_t *offsets, size_t count, cx_u128 *out,
                 uint8_t *ok, int memkind, int device);
int cx_hex_format(const cx_u128 *keys, size_t count, char *out, uint8_t *len, int memkind,
                  int device);

/* ---- Rabin IDA: DHash payload coding ---------------------
 * IDA(n, m, p) of src/ida/ida.cpp over a batch of ragged blocks (one datum
 * each): block b = data[offsets[b] .. offsets[b+1]), S_b = ceil(len_b / m)
 * segments, seg_offsets[b] = sum of S_c for c < b (cx_ida_segments, host).
 * cx_ida_encode: IDA::Encode (ida.cpp:59-73): fragment i (index i + 1,
 *   data_block.cpp:12-13) of block b is frags[n*seg_offsets[b] + i*S_b ..+ S_b).
 *   Host buffers are validated (seg_offsets must match offsets); with device
 *   buffers the call only enqueues kernels on the null stream (no sync).
 * cx_ida_decode: IDA::Decode (ida.cpp:120-162) from m fragment rows per block
 *   (frags[m*seg_offsets[b] + k*S_b ..]) with 1-based indices
 *   indices[b*m + k]: values (< p) at out[m*seg_offsets[b] ..], kept length
 *   out_len[b] (trailing zeros dropped as the reference does); out_len[b] =
 *   UINT64_MAX when the indices have no inverse ("N is not invertible",
 *   matrix_math.cpp:81-82).  Blocks sharing the previous block's index list
 *   share one inverse (one small device->host read per call to size them).
 *   The inverse follows matrix_math.cpp:103-168
 *   including its int arithmetic as compiled (wrap-around).
 * Limits: 1 <= m < n <= 32, n < p <= 46340.  DHash uses (14, 10, 257). */
int cx_ida_segments(const uint64_t *offsets, size_t blocks, int m, uint64_t *seg_offsets);
int cx_ida_encode(const uint8_t *data, const uint64_t *offsets, const uint64_t *seg_offsets,
                  size_t blocks, int n, int m, int p, uint16_t *frags, int memkind, int device);
int cx_ida_decode(const uint16_t *frags, const uint64_t *seg_offsets, const uint8_t *indices,
                  size_t blocks, int m, int p, uint16_t *out, uint64_t *out_len, int memkind,
                  int device);

/* ---- wire bridge: GET_SUCC over JSON ---------------------
 * A ring of peers named "ip:port" (IDs = UUIDv5 of the name,
 * abstract_chord_peer.cpp:21) answering the reference's request objects
 * (handler map chord_peer.cpp:15-40, server.h:194-210):
 *   {"COMMAND":"GET_SUCC","KEY":<hex>[,"SRC":"ip:port"]}
 *     -> {"ID","MIN_KEY","IP_ADDR","PORT","SUCCESS":true}  (remote_peer.cpp:83-91)
 *   {"COMMAND":"GET_SUCC_BATCH","KEYS":[<hex>...][,"SRC":"ip:port"|"SRCS":[...]]}
 *     -> {"RESULTS":[{"ID","MIN_KEY","IP_ADDR","PORT","HOPS"}...],"SUCCESS":true}
 * Failures answer {"SUCCESS":false,"ERRORS":<message>} as server.h:156-165
 * does.  SRC is the peer the request is issued at (default: ring index 0).
 * The response is malloc'd; release it with cx_wire_free. */
typedef struct cx_wire cx_wire;
int cx_wire_create(const char *const *addrs, size_t n, int device, cx_wire **out);
int cx_wire_destroy(cx_wire *wire);
int cx_wire_ring(const cx_wire *wire, const cx_ring **ring);
int cx_wire_handle(cx_wire *wire, const char *request, size_t len, char **response,
                   size_t *response_len);
void cx_wire_free(char *response);

/* ---- arc-sharded routing (multi-GPU layout 2) -------------------
 * Rank g of G owns the arc of peers [g n / G, (g+1) n / G).  Every rank keeps
 * the replicated sorted ring (and its finger table) and the pattern-keyed
 * route planes of the top levels [128 - T, 128) for ALL peers (T =
 * top_levels); the planes below them it keeps only for its own arc plus a
 * halo (the peers whose IDs lie within 2^(128 - T) before the arc).  A
 * lookup walks on its origin rank while it needs replicated rows; the first
 * time it needs a lower level it is within 2^(128 - T) of its key, so it
 * travels once, as a 32-B WALK record, to the rank whose arc holds the key's
 * owner -- the GET_SUCC request forwarded to the next peer
 * (ChordPeer::ForwardRequest, chord_peer.cpp:185-211) -- finishes there, and
 * its result travels home once (RESULT record).  Owners, hops and statuses
 * equal cx_route's on the replicated ring.  All arc buffers are device memory
 * (CX_MEM_DEVICE).  This record protocol (origin walk or key-first, three
 * rounds) is kept for A/B; the default exchange is the key-first structure-of-
 * arrays protocol at the end of this header (cx_arc_partition / route /
 * deliver: two all-to-alls, 20 B out and 8 B back per lookup). */
typedef struct cx_arc_rec {
    uint64_t w0, w1; /* key (lookups) / owner | status << 32 (results) */
    uint64_t qid;    /* origin rank << 40 | index at the origin */
    uint32_t cur;    /* peer the lookup continues at / owner (results) */
    uint32_t hk;     /* hops | kind << 8 */
} cx_arc_rec;
enum { CX_ARC_NEW = 0, CX_ARC_RESULT = 1, CX_ARC_WALK = 2, CX_ARC_NONE = 3 };
#define CX_ARC_MAX_RANKS 64
#define CX_ARC_TOP_LEVELS 6 /* default replicated top levels (top_levels = 0) */

/* Builds rank `rank`'s planes of a `world`-rank layout (and the converged
 * finger table if missing: the planes are derived from it, as the reference's
 * fingers are, abstract_chord_peer.cpp:564-613).  Arc routing walks the
 * converged ring: after cx_fingers_upload, cx_peer_state_upload or
 * cx_liveness_upload the arc calls fail with CX_E_STATE (cx_route honours
 * that state). */
int cx_arc_build(cx_ring *ring, int world, int rank, int top_levels);
/* Replicated top levels, local rows (arc + halo) and route-plane bytes. */
int cx_arc_info(const cx_ring *ring, int *top_levels, uint64_t *local_rows,
                uint64_t *table_bytes);

/* Records of q lookups issued at peers src[i] by rank `rank` (kind NEW). */
int cx_arc_seed(const cx_ring *ring, int rank, const uint32_t *src, const cx_u128 *keys,
                size_t q, cx_arc_rec *out);

/* One step on rank `rank`: every input record yields exactly one output record:
 * WALK (continue on the rank of the key's arc), RESULT (for a remote origin)
 * or NONE (result written to owner/hops/status at qid's index: results for
 * this rank's lookups, and RESULT records coming home). */
int cx_arc_step(const cx_ring *ring, int rank, const cx_arc_rec *in, size_t q, cx_arc_rec *out,
                uint32_t *owner, uint8_t *hops, uint8_t *status);

/* cx_arc_seed + the first cx_arc_step in one pass: the step reads the new
 * lookups straight from src / keys (out: one record per lookup). */
int cx_arc_start(const cx_ring *ring, int rank, const uint32_t *src, const cx_u128 *keys,
                 size_t q, cx_arc_rec *out, uint32_t *owner, uint8_t *hops, uint8_t *status);

/* Groups WALK/RESULT records (and NEW ones, by key) by destination rank into
 * `send` (NONE dropped); counts[world] (host) receives the per-destination
 * record counts. */
int cx_arc_bucket(const cx_ring *ring, int world, const cx_arc_rec *recs, size_t q,
                  cx_arc_rec *send, uint64_t *counts);
/* Lookups sent ahead by key (no origin walk): cx_arc_seed + cx_arc_bucket in
 * one pass, the NEW records built on the fly; the rank of the key's arc walks
 * them from their sources (cx_arc_step). */
int cx_arc_send_ahead(const cx_ring *ring, int world, int rank, const uint32_t *src,
                      const cx_u128 *keys, size_t q, cx_arc_rec *send, uint64_t *counts);

/* ---- key-first exchange, structure of arrays (the default arc protocol) -----
 * One batch = two all-to-all exchanges (ForwardRequest's GET_SUCC sent to the
 * key's arc, chord_peer.cpp:185-211, and its reply):
 *   1. cx_arc_partition on every rank: its lookups grouped by the rank of the
 *      key's arc -> send_keys / send_src (exchanged: 20 B per lookup), perm
 *      (kept: perm[i] = the send slot of lookup i), counts[world] (host);
 *   2. cx_arc_route on every rank over what it received (in receive order):
 *      res[j] = owner | hops << 32 | status << 40 | 1 << 63 for lookup j,
 *      walked from its source over the replicated top planes and the rank's
 *      own rows (a walk that needs a lower level is within 2^(128 - T) of its
 *      key: in the key's arc or its halo);
 *   3. res goes back with the splits swapped (8 B per lookup) and lands in
 *      send order (or in the partition's regions, cx_arc_partition_regions:
 *      perm then indexes world x cap slots); cx_arc_deliver writes owner /
 *      hops / status of lookup i
 *      from res[perm[i]] (perm == NULL: identity, the single-rank case).
 * Owners, hops and statuses equal cx_route's on the replicated ring.  Device
 * buffers; perm, send_* sized q. */
int cx_arc_partition(const cx_ring *ring, int world, const uint32_t *src, const cx_u128 *keys,
                     size_t q, cx_u128 *send_keys, uint32_t *send_src, uint32_t *perm,
                     uint64_t *counts);
/* Single-pass variant of cx_arc_partition: destination d's lookups go to the
 * region [d cap, (d + 1) cap) of send_keys / send_src (world x cap entries
 * each; counts[d] filled), perm[i] = the region slot of lookup i, so no count
 * pass precedes the scatter.  CX_E_STATE when some destination receives more
 * than cap lookups (nothing of it is written; use cx_arc_partition).
 * send_hint (world x cap, may be NULL): the origin resolves each lookup's
 * start at its source -- StoredLocally(key) at src (abstract_chord_peer.cpp:
 * 720-725) and d = (key - id_src) >> (116 - ceil(log2 n)) -- reading the
 * sources' (pred, self) IDs in lookup order, so the arc rank's walk
 * (cx_arc_route_hinted) needs no source IDs: 8 B more per lookup on the wire,
 * one random 32-B gather less per lookup at the arc. */
int cx_arc_partition_regions(const cx_ring *ring, int world, const uint32_t *src,
                             const cx_u128 *keys, size_t q, uint64_t cap, cx_u128 *send_keys,
                             uint32_t *send_src, uint64_t *send_hint, uint32_t *perm,
                             uint64_t *counts);
/* cx_arc_partition_regions without a host synchronisation: counts_dev
 * (device, world + 1 int64) receives counts[0..world) and, at [world], 1 if
 * some destination received more than cap lookups (then that destination's
 * region holds nothing and the caller re-partitions with cx_arc_partition).
 * Everything runs asynchronously on the ring's stream, so a caller can
 * partition several pieces and exchange all their counts in one collective. */
int cx_arc_partition_regions_async(const cx_ring *ring, int world, const uint32_t *src,
                                   const cx_u128 *keys, size_t q, uint64_t cap,
                                   cx_u128 *send_keys, uint32_t *send_src, uint64_t *send_hint,
                                   uint32_t *perm, int64_t *counts_dev);
/* Exact-layout partition in two asynchronous passes (no capacity, no
 * overflow, no host synchronisation): cx_arc_count_async writes the
 * per-destination counts of the lookups' keys into counts_dev (device,
 * world int64) and, with own_idx (device, q uint32) and own_ws (device
 * scratch of one uint32), writes the indices of the lookups of rank `me`'s
 * own arc into own_idx[0 .. counts[me]) for cx_arc_route_local (a permutation
 * of them: ascending within each block of up to 16 384 lookups, the blocks'
 * runs in completion order);
 * cx_arc_scatter_async, given those counts (still on the device), lays
 * destination d's lookups out at [sum_{j<d} counts[j], ...) of send_keys /
 * send_src / send_hint (q entries each; send_hint may be NULL) with perm[i] =
 * the slot of lookup i; skip_rank >= 0 leaves that destination's lookups out
 * (perm = 0xFFFFFFFF, their count taken as 0: the rank walks them in place).
 * cursor_dev: world uint32 of scratch (device) per concurrent scatter.  Both
 * run on the ring's stream, so a caller can count every piece, exchange the
 * counts in one collective, and scatter each piece on another stream while
 * earlier pieces are walked. */
int cx_arc_count_async(const cx_ring *ring, int world, const cx_u128 *keys, size_t q,
                       int64_t *counts_dev, int me, uint32_t *own_idx, uint32_t *own_ws);
int cx_arc_scatter_async(const cx_ring *ring, int world, const uint32_t *src,
                         const cx_u128 *keys, size_t q, const int64_t *counts_dev,
                         uint32_t *cursor_dev, cx_u128 *send_keys, uint32_t *send_src,
                         uint64_t *send_hint, uint32_t *perm, int skip_rank);
/* The lookups of this rank's own arc walked in place: keys[idx[j]] issued at
 * src[idx[j]] for j < q, over the arc planes (as cx_arc_route), started from
 * the sources' own IDs; owner / hops / status (status may be NULL) written at
 * idx[j] -- no exchange, no packed results, no delivery pass.  Every idx[j]
 * must index keys / src / owner / hops / status (device data: not checked). */
int cx_arc_route_local(const cx_ring *ring, const uint32_t *src, const cx_u128 *keys,
                       const uint32_t *idx, size_t q, uint32_t *owner, uint8_t *hops,
                       uint8_t *status);
int cx_arc_route(const cx_ring *ring, const uint32_t *src, const cx_u128 *keys, size_t q,
                 uint64_t *res);
/* cx_arc_route with the origins' source hints (cx_arc_partition_regions
 * send_hint, received alongside keys and sources): same results. */
int cx_arc_route_hinted(const cx_ring *ring, const uint32_t *src, const cx_u128 *keys,
                        const uint64_t *hint, size_t q, uint64_t *res);
int cx_arc_deliver(const cx_ring *ring, const uint64_t *res, const uint32_t *perm, size_t q,
                   uint32_t *owner, uint8_t *hops, uint8_t *status);

#ifdef __cplusplus
}
#endif
#endif /* CHORDX_H */
