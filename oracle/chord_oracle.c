/*
 * chord_oracle.c -- CPU restatement of the reference's lookup path.
 *
 * TEST INFRASTRUCTURE ONLY (see chord_oracle.h).  Plain C11 + pthreads; no
 * Boost.  Each function cites the reference file:line it restates.
 */
#define _GNU_SOURCE
#include "chord_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static const or_u128 ONE = 1;

static inline or_u128 k2u(or_key k) { return ((or_u128)k.hi << 64) | k.lo; }
static inline or_key u2k(or_u128 v) {
    or_key k;
    k.lo = (uint64_t)v;
    k.hi = (uint64_t)(v >> 64);
    return k;
}
static inline or_u256 u256_from128(or_u128 v) {
    or_u256 r = {{(uint64_t)v, (uint64_t)(v >> 64), 0, 0}};
    return r;
}
static inline or_u128 u256_low128(or_u256 a) { return ((or_u128)a.w[1] << 64) | a.w[0]; }
static int u256_cmp(or_u256 a, or_u256 b) {
    for (int i = 3; i >= 0; --i) {
        if (a.w[i] < b.w[i]) return -1;
        if (a.w[i] > b.w[i]) return 1;
    }
    return 0;
}
static or_u256 u256_add(or_u256 a, or_u256 b) {
    or_u256 r;
    unsigned carry = 0;
    for (int i = 0; i < 4; ++i) {
        or_u128 s = (or_u128)a.w[i] + b.w[i] + carry;
        r.w[i] = (uint64_t)s;
        carry = (unsigned)(s >> 64);
    }
    return r; /* mod 2^256, like unchecked uint256_t */
}
static or_u256 u256_sub(or_u256 a, or_u256 b) {
    or_u256 r;
    unsigned borrow = 0;
    for (int i = 0; i < 4; ++i) {
        or_u128 d = (or_u128)a.w[i] - b.w[i] - borrow;
        r.w[i] = (uint64_t)d;
        borrow = (unsigned)((d >> 64) & 1);
    }
    return r;
}
static int u256_is_zero(or_u256 a) { return !(a.w[0] | a.w[1] | a.w[2] | a.w[3]); }
static or_u256 u256_two128(void) {
    or_u256 r = {{0, 0, 1, 0}};
    return r;
}

/* ------------------------------------------------------------------------
 * SHA-1 (FIPS 180-4) and RFC-4122 name-based UUIDv5.
 * Restates boost::uuids::name_generator_sha1(ns::dns()) used by
 * GenerateSha1Hash, key.h:29-33; the uuid's 16 bytes become the integer value
 * big-endian (uint256_t(uuid), key.h:77-78).
 * ---------------------------------------------------------------------- */
static inline uint32_t rol(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

void or_sha1(const uint8_t *msg, size_t len, uint8_t out[20]) {
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    size_t total = ((len + 8) / 64 + 1) * 64;
    uint8_t *buf = (uint8_t *)calloc(total, 1);
    memcpy(buf, msg, len);
    buf[len] = 0x80;
    uint64_t bits = (uint64_t)len * 8;
    for (int i = 0; i < 8; ++i) buf[total - 1 - i] = (uint8_t)(bits >> (8 * i));
    for (size_t off = 0; off < total; off += 64) {
        uint32_t w[80];
        for (int i = 0; i < 16; ++i)
            w[i] = ((uint32_t)buf[off + 4 * i] << 24) | ((uint32_t)buf[off + 4 * i + 1] << 16) |
                   ((uint32_t)buf[off + 4 * i + 2] << 8) | buf[off + 4 * i + 3];
        for (int i = 16; i < 80; ++i) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
        for (int i = 0; i < 80; ++i) {
            uint32_t f, k;
            if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
            else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
            else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
            else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
            uint32_t t = rol(a, 5) + f + e + k + w[i];
            e = d; d = c; c = rol(b, 30); b = a; a = t;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
    }
    free(buf);
    for (int i = 0; i < 5; ++i) {
        out[4 * i] = (uint8_t)(h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8);
        out[4 * i + 3] = (uint8_t)h[i];
    }
}

or_key or_uuid5_dns(const char *name, size_t len) {
    /* RFC 4122 Appendix C: NameSpace_DNS 6ba7b810-9dad-11d1-80b4-00c04fd430c8 */
    static const uint8_t ns[16] = {0x6b, 0xa7, 0xb8, 0x10, 0x9d, 0xad, 0x11, 0xd1,
                                   0x80, 0xb4, 0x00, 0xc0, 0x4f, 0xd4, 0x30, 0xc8};
    uint8_t *m = (uint8_t *)malloc(16 + len + 1);
    memcpy(m, ns, 16);
    memcpy(m + 16, name, len);
    uint8_t dg[20];
    or_sha1(m, 16 + len, dg);
    free(m);
    dg[6] = (uint8_t)((dg[6] & 0x0F) | 0x50); /* version 5 */
    dg[8] = (uint8_t)((dg[8] & 0x3F) | 0x80); /* RFC 4122 variant */
    or_u128 v = 0;
    for (int i = 0; i < 16; ++i) v = (v << 8) | dg[i];
    return u2k(v);
}

/* ------------------------------------------------------------------------
 * a2: GenericKey::InBetween, key.h:103-131.
 * ---------------------------------------------------------------------- */
int or_in_between(or_u256 v, or_u256 lb, or_u256 ub, int inclusive) {
    /* key.h:108-113: equal bounds -> point test, regardless of `inclusive` */
    if (u256_cmp(lb, ub) == 0) return u256_cmp(v, ub) == 0;
    /* key.h:116-118: mod every operand by keys_in_ring_ = 16^32 = 2^128 */
    or_u256 mlb = u256_from128(u256_low128(lb));
    or_u256 mub = u256_from128(u256_low128(ub));
    or_u256 mv = u256_from128(u256_low128(v));
    if (u256_cmp(lb, ub) < 0) { /* key.h:121: RAW bounds compared */
        /* key.h:122-124: note the upper test uses the RAW upper bound */
        if (inclusive) return u256_cmp(mlb, mv) <= 0 && u256_cmp(mv, ub) <= 0;
        return u256_cmp(mlb, mv) < 0 && u256_cmp(mv, ub) < 0;
    }
    /* key.h:126-129 */
    if (inclusive) return !(u256_cmp(mub, mv) < 0 && u256_cmp(mv, mlb) < 0);
    return !(u256_cmp(mub, mv) <= 0 && u256_cmp(mv, mlb) <= 0);
}

/* a3: operator+(key, T), key.h:236-240. */
or_u256 or_add_num(or_u256 v, uint64_t t) {
    or_u256 tt = {{t, 0, 0, 0}};
    or_u256 s = u256_add(v, tt); /* uint256_t + T wraps mod 2^256 */
    return u256_from128(u256_low128(s));
}

/* a3: operator-(key, T), key.h:242-250.  `key.value_ - number` is evaluated in
 * uint256_t (wrapping), then tested `> 0` as cpp_int. */
or_u256 or_sub_num(or_u256 v, uint64_t t) {
    or_u256 tt = {{t, 0, 0, 0}};
    or_u256 d = u256_sub(v, tt);
    if (!u256_is_zero(d)) return d;
    return u256_two128(); /* keys_in_ring_ + 0 */
}

/* a3: operator-(key, key), key.h:258-270, signed cpp_int difference. */
or_u256 or_sub_key(or_u256 a, or_u256 b) {
    int c = u256_cmp(a, b);
    if (c > 0) return u256_sub(a, b);
    /* diff <= 0: keys_in_ring_ + diff = 2^128 - (b - a) (may be "negative"
     * only if b - a > 2^128, impossible for canonical keys) */
    or_u256 nd = u256_sub(b, a);
    return u256_sub(u256_two128(), nd);
}

/* a4: FingerTable::GetNthRange, finger_table.h:177-188. */
void or_nth_range(or_key id, int n, or_u256 *lb, or_u256 *ub) {
    or_u128 s = k2u(id);
    or_u128 l = s + (ONE << n); /* (start + 2^n) mod 2^128 */
    *lb = u256_from128(l);
    or_u128 u = (n + 1 == 128) ? s : s + (ONE << (n + 1)); /* 2^128 mod 2^128 = 0 */
    or_u256 um = u256_from128(u);
    or_u256 one = {{1, 0, 0, 0}};
    *ub = u256_sub(um, one); /* uint256_t(...) - 1: 0 -> 2^256-1 */
}

/* a5: FingerTable::Lookup, finger_table.h:115-130 -- linear first-match scan. */
static int finger_index_raw(or_key id, or_u256 v) {
    for (int i = 0; i < OR_FINGERS; ++i) {
        or_u256 lb, ub;
        or_nth_range(id, i, &lb, &ub);
        if (or_in_between(v, lb, ub, 1)) return i;
    }
    return -1; /* throw std::runtime_error("ChordKey not found") */
}
int or_finger_index(or_key id, or_key key) {
    return finger_index_raw(id, u256_from128(k2u(key)));
}

/* ------------------------------------------------------------------------
 * a13: ring build.
 * ---------------------------------------------------------------------- */
static int cmp_key(const void *a, const void *b) {
    or_u128 x = k2u(*(const or_key *)a), y = k2u(*(const or_key *)b);
    return x < y ? -1 : (x > y ? 1 : 0);
}

size_t or_ring_build(const or_key *ids, size_t n, or_key *out) {
    if (out != ids) memmove(out, ids, n * sizeof(or_key));
    qsort(out, n, sizeof(or_key), cmp_key);
    size_t m = 0;
    for (size_t i = 0; i < n; ++i)
        if (m == 0 || k2u(out[m - 1]) != k2u(out[i])) out[m++] = out[i];
    return m;
}

/* lower_bound with wrap: owner of key in the converged ring. */
uint32_t or_successor(const or_key *ring, size_t n, or_key key) {
    or_u128 x = k2u(key);
    size_t lo = 0, hi = n;
    while (lo < hi) {
        size_t mid = lo + (hi - lo) / 2;
        if (k2u(ring[mid]) < x) lo = mid + 1;
        else hi = mid;
    }
    return (uint32_t)(lo == n ? 0 : lo);
}

/* ------------------------------------------------------------------------
 * Thread pool helper: split [0, count) over nthreads.
 * ---------------------------------------------------------------------- */
typedef void (*range_fn)(void *ctx, size_t b, size_t e);
typedef struct { range_fn fn; void *ctx; size_t b, e; } job_t;
static void *job_run(void *p) {
    job_t *j = (job_t *)p;
    j->fn(j->ctx, j->b, j->e);
    return NULL;
}
static void parallel_for(size_t count, int nthreads, range_fn fn, void *ctx) {
    if (nthreads <= 1 || count < 2) { fn(ctx, 0, count); return; }
    if ((size_t)nthreads > count) nthreads = (int)count;
    pthread_t th[256];
    job_t jobs[256];
    if (nthreads > 256) nthreads = 256;
    size_t chunk = (count + nthreads - 1) / nthreads;
    int t = 0;
    for (; t < nthreads; ++t) {
        size_t b = t * chunk, e = b + chunk > count ? count : b + chunk;
        if (b >= e) break;
        jobs[t].fn = fn; jobs[t].ctx = ctx; jobs[t].b = b; jobs[t].e = e;
        pthread_create(&th[t], NULL, job_run, &jobs[t]);
    }
    for (int i = 0; i < t; ++i) pthread_join(th[i], NULL);
}

typedef struct { const or_key *ring; size_t n; const or_key *keys; uint32_t *owner; } succ_ctx;
static void succ_range(void *c, size_t b, size_t e) {
    succ_ctx *s = (succ_ctx *)c;
    for (size_t i = b; i < e; ++i) s->owner[i] = or_successor(s->ring, s->n, s->keys[i]);
}
void or_successor_batch(const or_key *ring, size_t n, const or_key *keys, size_t q,
                        uint32_t *owner, int nthreads) {
    succ_ctx c = {ring, n, keys, owner};
    parallel_for(q, nthreads, succ_range, &c);
}

/* GetPredecessor, abstract_chord_peer.cpp:380-421, on the converged ring:
 * predecessor_ of the key's owner (StoredLocally at the owner returns it,
 * :388-390; the successor-list shortcut checks InBetween(pred_of_succ, succ),
 * :394-401; a forwarded GET_PRED ends at the owner, :405-412); a lone peer
 * has no predecessor set and returns itself (:383-385). */
typedef struct { const or_key *ring; size_t n; const or_key *keys; uint32_t *out; } pred_ctx;
static void pred_range(void *c, size_t b, size_t e) {
    pred_ctx *s = (pred_ctx *)c;
    for (size_t i = b; i < e; ++i) {
        uint32_t o = or_successor(s->ring, s->n, s->keys[i]);
        s->out[i] = s->n == 1 ? o : (o == 0 ? (uint32_t)(s->n - 1) : o - 1);
    }
}
void or_predecessor_batch(const or_key *ring, size_t n, const or_key *keys, size_t q,
                          uint32_t *pred, int nthreads) {
    pred_ctx c = {ring, n, keys, pred};
    parallel_for(q, nthreads, pred_range, &c);
}

/* ------------------------------------------------------------------------
 * a6: converged PopulateFingerTable, abstract_chord_peer.cpp:564-613.
 * Entry i of peer p = successor of GetNthRange(i).first.
 * ---------------------------------------------------------------------- */
typedef struct { const or_key *ring; size_t n, p0; uint32_t *F; } fing_ctx;
static void fing_range(void *c, size_t b, size_t e) {
    fing_ctx *f = (fing_ctx *)c;
    for (size_t r = b; r < e; ++r) {
        size_t p = f->p0 + r;
        for (int i = 0; i < OR_FINGERS; ++i) {
            or_u256 lb, ub;
            or_nth_range(f->ring[p], i, &lb, &ub);
            f->F[r * OR_FINGERS + i] = or_successor(f->ring, f->n, u2k(u256_low128(lb)));
        }
    }
}
void or_fingers_rows(const or_key *ring, size_t n, size_t p0, size_t p1, uint32_t *F,
                     int nthreads) {
    fing_ctx c = {ring, n, p0, F};
    parallel_for(p1 - p0, nthreads, fing_range, &c);
}
void or_fingers_build(const or_key *ring, size_t n, uint32_t *F, int nthreads) {
    or_fingers_rows(ring, n, 0, n, F, nthreads);
}

/* ------------------------------------------------------------------------
 * a7-a9: routed lookup.
 * ---------------------------------------------------------------------- */
static or_u256 peer_min_key(const or_peers *P, uint32_t p) {
    if (P->min_keys) return u256_from128(k2u(P->min_keys[p]));
    /* min_key_ = predecessor id + 1: chord_peer.cpp:275 / abstract_chord_peer.cpp:96;
     * single peer: id_ + 1 (StartChord, abstract_chord_peer.cpp:69). */
    uint32_t pr = P->n == 1 ? p : (p == 0 ? (uint32_t)(P->n - 1) : p - 1);
    return or_add_num(u256_from128(k2u(P->ring[pr])), 1);
}
static uint32_t peer_pred(const or_peers *P, uint32_t p) {
    if (P->preds) return P->preds[p];
    if (P->n == 1) return OR_NONE;
    return p == 0 ? (uint32_t)(P->n - 1) : p - 1;
}
/* RemotePeer::IsAlive (remote_peer.cpp:43-46): a TCP connect to the peer's
 * server; an unset peer (OR_NONE, port 0) never answers. */
static int peer_alive(const or_peers *P, uint32_t p) {
    if (p == OR_NONE || p >= P->n) return 0;
    return P->alive ? P->alive[p] != 0 : 1;
}
/* Entry j of peer p's successors_ list, OR_NONE past its end. */
static uint32_t succ_entry(const or_peers *P, uint32_t p, int j) {
    if (j >= P->ns) return OR_NONE;
    if (P->succs) return P->succs[(size_t)p * P->ns + j];
    if ((size_t)j >= P->n - 1) return OR_NONE; /* converged: n-1 other peers */
    return (uint32_t)((p + 1 + (uint32_t)j) % P->n);
}
static int succ_list_size(const or_peers *P, uint32_t p) {
    int k = 0;
    while (k < P->ns && succ_entry(P, p, k) != OR_NONE) ++k;
    return k;
}
/* RemotePeerList::Lookup(key, succ = true), remote_peer_list.cpp:86-110:
 * first entry i with key in [previous, id_i] (InBetween inclusive, previous
 * starting at the list's starting key = the owner's id), else none. */
static uint32_t succ_list_lookup(const or_peers *P, uint32_t p, or_u256 v) {
    or_u256 prev = u256_from128(k2u(P->ring[p]));
    const int sz = succ_list_size(P, p);
    for (int i = 0; i < sz; ++i) {
        uint32_t e = succ_entry(P, p, i);
        or_u256 id = u256_from128(k2u(P->ring[e]));
        if (or_in_between(v, prev, id, 1)) return e;
        prev = id;
    }
    return OR_NONE;
}
/* RemotePeerList::LookupLiving, remote_peer_list.cpp:112-132, as written: the
 * found entry if alive; the scan for a later living entry runs
 * `for (i = succ_ind; i % size < succ_ind; ++i)`, whose condition is false on
 * entry (succ_ind < size), so it never executes. */
static uint32_t succ_list_lookup_living(const or_peers *P, uint32_t p, or_u256 key) {
    uint32_t s = succ_list_lookup(P, p, key);
    if (s == OR_NONE) return OR_NONE;
    if (peer_alive(P, s)) return s;
    const int sz = succ_list_size(P, p);
    int succ_ind = 0;
    while (succ_ind < sz && succ_entry(P, p, succ_ind) != s) ++succ_ind; /* GetIndex */
    for (int i = succ_ind; (size_t)i % (size_t)sz < (size_t)succ_ind; ++i) {
        uint32_t e = succ_entry(P, p, i % sz);
        if (peer_alive(P, e)) return e;
    }
    return OR_NONE;
}
/* StoredLocally, abstract_chord_peer.cpp:720-725. */
static int stored_locally(const or_peers *P, uint32_t p, or_u256 key) {
    return or_in_between(key, peer_min_key(P, p),
                         u256_from128(k2u(P->ring[p])), 1);
}

/* The walk on the key's raw uint256 value: GenericKey keeps uint256("0x"+s)
 * unreduced (key.h:73-75), so a wire key of 33+ significant hex digits fails
 * every InBetween point test (key.h:108-113) while the ranged tests reduce it
 * mod 2^128 (key.h:116-118). */
static int route_raw(const or_peers *P, uint32_t src, or_u256 key, uint32_t *owner,
                     uint8_t *hops) {
    uint32_t cur = src;
    unsigned h = 0;
    for (;;) {
        /* GetSuccessor: abstract_chord_peer.cpp:320-323 */
        if (stored_locally(P, cur, key)) {
            *owner = cur;
            *hops = (uint8_t)h;
            return OR_Q_OK;
        }
        /* ChordPeer::ForwardRequest, chord_peer.cpp:185-211 */
        int fi = finger_index_raw(P->ring[cur], key);
        if (fi < 0) { /* no range holds key == id (or, raw, id + 1): Lookup
                       * throws "ChordKey not found" (finger_table.h:129);
                       * unreachable for a key < 2^128, which its own id stores */
            *owner = OR_NONE;
            *hops = (uint8_t)h;
            return OR_Q_NOT_FOUND;
        }
        uint32_t nxt = P->F[(size_t)cur * OR_FINGERS + fi];
        if (nxt == OR_NONE) { /* the matching finger was never added: Lookup
                               * scans table_ and throws (finger_table.h:119-129) */
            *owner = OR_NONE;
            *hops = (uint8_t)h;
            return OR_Q_NOT_FOUND;
        }
        uint32_t pr = peer_pred(P, cur);
        /* chord_peer.cpp:195-197 / dhash_peer.cpp:508-510: finger points at
         * self and the predecessor is alive */
        if (nxt == cur && peer_alive(P, pr)) {
            nxt = pr;
        } else if (!peer_alive(P, nxt)) {
            if (P->rule == OR_FWD_DHASH) {
                /* dhash_peer.cpp:516-526: LookupLiving, else successors_[0]
                 * if alive, else throw.  (An empty list makes the reference's
                 * GetNthEntry(0) dereference end(); treated as the throw.) */
                uint32_t s = succ_list_lookup_living(P, cur, key);
                uint32_t s0 = succ_entry(P, cur, 0);
                if (s != OR_NONE) nxt = s;
                else if (peer_alive(P, s0)) nxt = s0;
                else nxt = OR_NONE;
            } else {
                /* chord_peer.cpp:201-208: successors_.Lookup, used if alive */
                uint32_t s = succ_list_lookup(P, cur, key);
                nxt = (s != OR_NONE && peer_alive(P, s)) ? s : OR_NONE;
            }
            if (nxt == OR_NONE) { /* throw std::runtime_error("Lookup failed") */
                *owner = OR_NONE;
                *hops = (uint8_t)h;
                return OR_Q_FAILED;
            }
        }
        /* chord_peer.cpp:210 SendRequest = one hop; the receiver's
         * GetSuccHandler (abstract_chord_peer.cpp:332-337) recurses. */
        if (h == OR_HOP_CAP) {
            *owner = OR_NONE;
            *hops = OR_HOP_CAP;
            return OR_Q_HOPCAP;
        }
        ++h;
        cur = nxt;
    }
}
int or_route(const or_peers *P, uint32_t src, or_key key, uint32_t *owner, uint8_t *hops) {
    return route_raw(P, src, u256_from128(k2u(key)), owner, hops);
}

typedef struct {
    const or_peers *P; const uint32_t *src; const or_key *keys;
    uint32_t *owner; uint8_t *hops; uint8_t *status;
} route_ctx;
static void route_range(void *c, size_t b, size_t e) {
    route_ctx *r = (route_ctx *)c;
    for (size_t i = b; i < e; ++i) {
        uint32_t o; uint8_t h;
        int st = or_route(r->P, r->src[i], r->keys[i], &o, &h);
        r->owner[i] = o;
        r->hops[i] = h;
        if (r->status) r->status[i] = (uint8_t)st;
    }
}
void or_route_batch(const or_peers *P, const uint32_t *src, const or_key *keys, size_t q,
                    uint32_t *owner, uint8_t *hops, uint8_t *status, int nthreads) {
    route_ctx c = {P, src, keys, owner, hops, status};
    parallel_for(q, nthreads, route_range, &c);
}

/* Raw-value walk: key i = hi[i]:lo[i] (bits 255..128 : 127..0). */
void or_route_raw_batch(const or_peers *P, const uint32_t *src, const or_key *lo,
                        const or_key *hi, size_t q, uint32_t *owner, uint8_t *hops,
                        uint8_t *status) {
    for (size_t i = 0; i < q; ++i) {
        or_u256 v = {{lo[i].lo, lo[i].hi, hi[i].lo, hi[i].hi}};
        status[i] = (uint8_t)route_raw(P, src[i], v, &owner[i], &hops[i]);
    }
}

/* a10: GetNSuccessors, abstract_chord_peer.cpp:345-373. */
int or_nsucc(const or_peers *P, uint32_t src, or_key key, int n, uint32_t *list) {
    /* ChordKey previous_peer_id = key - 1;  (key.h:242-250 quirks) */
    or_u256 prev = or_sub_num(u256_from128(k2u(key)), 1);
    int cnt = 0;
    for (int i = 0; i < n; ++i) {
        or_u256 q = or_add_num(prev, 1); /* previous_peer_id + 1, canonical */
        uint32_t s;
        uint8_t h;
        if (or_route(P, src, u2k(u256_low128(q)), &s, &h) != OR_Q_OK) break;
        int seen = 0;
        for (int j = 0; j < cnt; ++j) seen |= (list[j] == s);
        if (seen) break; /* abstract_chord_peer.cpp:362-365 */
        list[cnt++] = s;
        prev = u256_from128(k2u(P->ring[s]));
    }
    return cnt;
}

typedef struct {
    const or_peers *P; const uint32_t *src; const or_key *keys; int n;
    uint32_t *lists; uint8_t *count;
} nsucc_ctx;
static void nsucc_range(void *c, size_t b, size_t e) {
    nsucc_ctx *x = (nsucc_ctx *)c;
    for (size_t i = b; i < e; ++i) {
        uint32_t *l = x->lists + i * (size_t)x->n;
        int k = or_nsucc(x->P, x->src ? x->src[i] : 0, x->keys[i], x->n, l);
        for (int j = k; j < x->n; ++j) l[j] = OR_NONE;
        x->count[i] = (uint8_t)k;
    }
}
void or_nsucc_batch(const or_peers *P, const uint32_t *src, const or_key *keys, size_t q,
                    int n, uint32_t *lists, uint8_t *count, int nthreads) {
    nsucc_ctx c = {P, src, keys, n, lists, count};
    parallel_for(q, nthreads, nsucc_range, &c);
}

/* ------------------------------------------------------------------------
 * a12: churn + global-maintenance misplaced scan.
 * ---------------------------------------------------------------------- */
typedef struct { or_key id; uint32_t tag; } tagged;
static int cmp_tagged(const void *a, const void *b) {
    or_u128 x = k2u(((const tagged *)a)->id), y = k2u(((const tagged *)b)->id);
    if (x != y) return x < y ? -1 : 1;
    uint32_t s = ((const tagged *)a)->tag, t = ((const tagged *)b)->tag;
    return s < t ? -1 : (s > t ? 1 : 0);
}
size_t or_churn(const or_key *old_ring, size_t n_old, const or_key *joins, size_t nj,
                const or_key *leaves, size_t nl, or_key *new_ring, uint32_t *old_to_new) {
    uint8_t *gone = (uint8_t *)calloc(n_old ? n_old : 1, 1);
    for (size_t i = 0; i < nl; ++i) {
        uint32_t s = or_successor(old_ring, n_old, leaves[i]);
        if (n_old && k2u(old_ring[s]) == k2u(leaves[i])) gone[s] = 1;
    }
    tagged *all = (tagged *)malloc((n_old + nj + 1) * sizeof(tagged));
    size_t m = 0;
    for (size_t p = 0; p < n_old; ++p) {
        old_to_new[p] = OR_NONE;
        if (!gone[p]) { all[m].id = old_ring[p]; all[m].tag = (uint32_t)p; ++m; }
    }
    for (size_t i = 0; i < nj; ++i) { all[m].id = joins[i]; all[m].tag = OR_NONE; ++m; }
    /* Survivor tags sort before OR_NONE, so on an ID collision the surviving
     * peer is kept and the duplicate join is rejected (remote_peer_list.cpp:56-58). */
    qsort(all, m, sizeof(tagged), cmp_tagged);
    size_t k = 0;
    for (size_t i = 0; i < m; ++i) {
        if (k && k2u(new_ring[k - 1]) == k2u(all[i].id)) continue;
        new_ring[k] = all[i].id;
        if (all[i].tag != OR_NONE) old_to_new[all[i].tag] = (uint32_t)k;
        ++k;
    }
    free(all);
    free(gone);
    return k;
}

/* Misplaced holders of one key given its new successor list nl[0..nn)
 * (dhash_peer.cpp:298-348).  holder[0..nh) are ring indices (OR_NONE =
 * departed / empty slot).
 *
 * ORDERING ASSUMPTION (parity-unpinned): when several holders of a key are
 * misplaced, they are applied in list order -- holder j's pass runs after
 * holders 0..j-1 have handed the key over, so has[] already records the
 * successors they filled.  In the reference every holder runs its own 5-s
 * maintenance thread (DHashPeer::MaintenanceLoop, dhash_peer.cpp:271-296);
 * which holder hands the key to which lacking successor first depends on
 * thread timing there.  The reference's own test pins only the single-holder
 * case (DHashGlobalMaintenance.MisplacedKeys, dhash_test.cpp:123-149); the
 * multi-holder target assignment is this restatement's contract
 * (tests/test_gpu_parity.py::test_misplaced_multi_holder_order). */
static void misplaced_from_list(const uint32_t *nl, int nn, const uint32_t *holder, int nh,
                                uint16_t *mask, uint8_t *tg) {
    for (int j = 0; j < nh; ++j) tg[j] = 0xFF;
    uint8_t has[256];
    for (int r = 0; r < nn; ++r) {
        has[r] = 0;
        for (int j = 0; j < nh; ++j) has[r] |= (holder[j] == nl[r]);
    }
    uint16_t m = 0;
    for (int j = 0; j < nh; ++j) {
        if (holder[j] == OR_NONE) continue; /* departed peer: holds nothing */
        int in_list = 0;
        for (int r = 0; r < nn; ++r) in_list |= (nl[r] == holder[j]);
        if (in_list) continue; /* dhash_peer.cpp:322-328: id_ found in succs */
        m |= (uint16_t)(1u << j);
        /* dhash_peer.cpp:330-340: walk succs in list order; READ_RANGE shows
         * which lack the key; CREATE_KEY to the first lacking one, then
         * db_.Delete, so later succs are not offered it by this holder. */
        for (int r = 0; r < nn; ++r)
            if (!has[r]) { has[r] = 1; tg[j] = (uint8_t)r; break; }
    }
    *mask = m;
}

/* Core of the scan for one key on the converged ring: the new list is the
 * n-window of the key's successor (GetNSuccessors, a10). */
static void misplaced_one(const or_key *ring, size_t n_ring, or_key key, const uint32_t *holder,
                          int nh, int n, uint32_t *nl, uint8_t *count, uint16_t *mask,
                          uint8_t *tg) {
    int nn = (int)(n_ring < (size_t)n ? n_ring : (size_t)n);
    uint32_t sn = n_ring ? or_successor(ring, n_ring, key) : 0;
    for (int j = 0; j < n; ++j) nl[j] = j < nn ? (uint32_t)((sn + j) % n_ring) : OR_NONE;
    *count = (uint8_t)nn;
    misplaced_from_list(nl, nn, holder, nh, mask, tg);
}

typedef struct {
    const or_key *ring; size_t n_ring; const or_key *keys; const uint32_t *holders; int nh; int n;
    const or_key *old_ring; size_t n_old; const uint32_t *o2n; /* churn form when old_ring */
    uint32_t *new_lists; uint8_t *count; uint16_t *mask; uint8_t *target;
} mis_ctx;
static void mis_range(void *c, size_t b, size_t e) {
    mis_ctx *x = (mis_ctx *)c;
    uint32_t hb[256];
    for (size_t q = b; q < e; ++q) {
        const uint32_t *h;
        int nh = x->nh;
        if (x->old_ring) {
            /* holders = old n-window: DHashPeer::Create put fragment j on old
             * list rank j (dhash_peer.cpp:114-122); survivors mapped to the
             * new ring, departed peers -> OR_NONE */
            int no = (int)(x->n_old < (size_t)x->n ? x->n_old : (size_t)x->n);
            uint32_t so = x->n_old ? or_successor(x->old_ring, x->n_old, x->keys[q]) : 0;
            for (int j = 0; j < x->n; ++j)
                hb[j] = j < no ? x->o2n[(so + j) % x->n_old] : OR_NONE;
            h = hb;
            nh = x->n;
        } else {
            h = x->holders + q * (size_t)x->nh;
        }
        misplaced_one(x->ring, x->n_ring, x->keys[q], h, nh, x->n,
                      x->new_lists + q * (size_t)x->n, x->count + q, x->mask + q,
                      x->target + q * (size_t)nh);
    }
}
void or_misplaced_holders(const or_key *ring, size_t n_ring, const or_key *keys, size_t q,
                          const uint32_t *holders, int nh, int n, uint32_t *new_lists,
                          uint8_t *count, uint16_t *mask, uint8_t *target, int nthreads) {
    mis_ctx c = {ring, n_ring, keys, holders, nh, n, NULL, 0, NULL,
                 new_lists, count, mask, target};
    parallel_for(q, nthreads, mis_range, &c);
}
void or_misplaced(const or_key *old_ring, size_t n_old, const or_key *new_ring, size_t n_new,
                  const uint32_t *old_to_new, const or_key *keys, size_t q, int n,
                  uint32_t *new_lists, uint8_t *count, uint16_t *mask, uint8_t *target,
                  int nthreads) {
    mis_ctx c = {new_ring, n_new, keys, NULL, n, n, old_ring, n_old, old_to_new,
                 new_lists, count, mask, target};
    parallel_for(q, nthreads, mis_range, &c);
}

/* C5's CPU baseline: DHash maintenance computed as the
 * reference computes it, by routed lookups.  Per key: the placement list on
 * the old ring, GetNSuccessors(key, n) = n routed GetSuccessor lookups
 * (or_nsucc, abstract_chord_peer.cpp:345-373; DHashPeer::Create,
 * dhash_peer.cpp:103-129); its holders mapped to the new ring (old_to_new,
 * departed -> OR_NONE); the new list by the same routed GetNSuccessors on the
 * new ring; and the misplaced check of RunGlobalMaintenance
 * (dhash_peer.cpp:298-348) against it.  Lookups start at peer q mod n of each
 * ring.  Outputs as or_misplaced's plus the old lists and counts. */
typedef struct {
    const or_peers *Po, *Pn; const uint32_t *o2n; const or_key *keys; int n;
    uint32_t *old_lists; uint8_t *old_count; uint32_t *new_lists; uint8_t *count;
    uint16_t *mask; uint8_t *target;
} mroute_ctx;
static void mroute_range(void *c, size_t b, size_t e) {
    mroute_ctx *x = (mroute_ctx *)c;
    uint32_t hb[256];
    for (size_t q = b; q < e; ++q) {
        uint32_t *ol = x->old_lists + q * (size_t)x->n, *nl = x->new_lists + q * (size_t)x->n;
        int no = or_nsucc(x->Po, (uint32_t)(q % x->Po->n), x->keys[q], x->n, ol);
        for (int j = no; j < x->n; ++j) ol[j] = OR_NONE;
        x->old_count[q] = (uint8_t)no;
        for (int j = 0; j < x->n; ++j) hb[j] = j < no ? x->o2n[ol[j]] : OR_NONE;
        int nn = or_nsucc(x->Pn, (uint32_t)(q % x->Pn->n), x->keys[q], x->n, nl);
        for (int j = nn; j < x->n; ++j) nl[j] = OR_NONE;
        x->count[q] = (uint8_t)nn;
        misplaced_from_list(nl, nn, hb, x->n, x->mask + q, x->target + q * (size_t)x->n);
    }
}
void or_maintenance_routed(const or_peers *P_old, const or_peers *P_new, const uint32_t *old_to_new,
                           const or_key *keys, size_t q, int n, uint32_t *old_lists,
                           uint8_t *old_count, uint32_t *new_lists, uint8_t *count,
                           uint16_t *mask, uint8_t *target, int nthreads) {
    mroute_ctx c = {P_old, P_new, old_to_new, keys, n, old_lists, old_count, new_lists, count,
                    mask, target};
    parallel_for(q, nthreads, mroute_range, &c);
}

/* ------------------------------------------------------------------------
 * Synthetic inputs: splitmix64(seed, 2i) -> lo, (seed, 2i+1) -> hi.
 * ---------------------------------------------------------------------- */
static inline uint64_t splitmix64(uint64_t seed, uint64_t ctr) {
    uint64_t z = seed + (ctr + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
void or_splitmix_keys(uint64_t seed, size_t offset, size_t count, or_key *out) {
    for (size_t i = 0; i < count; ++i) {
        uint64_t c = (uint64_t)(offset + i);
        out[i].lo = splitmix64(seed, 2 * c);
        out[i].hi = splitmix64(seed, 2 * c + 1);
    }
}

double or_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}
