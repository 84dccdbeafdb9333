// cx_kernels.hpp -- launchers of the gfx950 kernels (internal to libchordx).
#pragma once

#include "cx_common.hpp"

// Tags >= CX_TAG_JOIN mark joining peers during a churn sort; smaller tags
// are old ring indices.
#define CX_TAG_JOIN 0x80000000u

// In-flight record of the arc-sharded walk (32 B, the unit exchanged between
// ranks).  qid = origin rank << ARC_ORIGIN_SHIFT | index at the origin.
struct alignas(16) ArcRec {
    uint64_t w0, w1;  // key (queries) / owner | status << 32 (results)
    uint64_t qid;
    uint32_t cur;     // peer to continue at (queries) / owner (results)
    uint32_t hk;      // hops | kind << 8
};
static_assert(sizeof(ArcRec) == 32, "ArcRec is 32 B");
#define ARC_ORIGIN_SHIFT 40
// Last peer ID of a non-empty arc and its rank (WALK destinations).
struct ArcBound {
    uint64_t lo, hi;
    uint32_t rank, pad;
};
#define ARC_INDEX_MASK ((1ull << ARC_ORIGIN_SHIFT) - 1)
// source hints of the key-first exchange (d >> gs < 2^36, so these are free)
#define ARC_HINT_LOCAL 0xFFFFFFFFFFFFFFFFull  // StoredLocally at the source: 0 hops
#define ARC_HINT_BAD 0xFFFFFFFFFFFFFFFEull    // src not a ring index (BADPEER at the arc)
enum { ARC_NEW = 0, ARC_RESULT = 1, ARC_WALK = 2, ARC_NONE = 3 };

// Peer liveness and successors_ lists for the literal walk's dead-finger
// branch (cx_liveness_upload).
// Guard words written right after the decode's inverse table (cx_api.hip).
#define IDA_GUARD_WORD 0xA5C3A5C3u
#define IDA_GUARD_WORDS 64

struct LitState {
    const uint8_t *alive;   // n bytes, nullptr = all alive
    const uint32_t *succs;  // n x ns, CX_NONE-padded, nullptr = converged window
    int ns;                 // successor-list length
    int rule;               // CX_FWD_CHORD / CX_FWD_DHASH
};

namespace cxk {

size_t scan_workspace_words(size_t n);
hipError_t exclusive_scan(uint32_t *data, size_t n, uint32_t *ws, hipStream_t s);

// Gap-code shift of the pattern-keyed route table: codes are successor gaps in
// units of 2^(116 - ib), ib = ceil(log2 n).
__host__ __device__ __forceinline__ int cz_shift(int ib) { return 116 - ib; }

// First level the streaming finger build's tile holds (planes-only builds need
// every plane level at or above it).
constexpr int FINGERS_TILE_L0 = 88;

// f2 finger repair: the level planes [L, L + nl) (nl <= 128 - FINGERS_TILE_L0)
// of a churned ring from its parent's (Pold, n_old peers) and the churn's
// old_to_new map; n2o: n words of workspace; *nsearch (device, optional) +=
// the fingers searched exactly instead of remapped.
hipError_t planes_repair(const SearchView &sv, const cell128 *ring, size_t n, const uint32_t *Pold,
                         size_t n_old, const uint32_t *o2n, uint32_t *n2o, int L, int nl,
                         uint32_t *Pnew, uint32_t *nsearch, hipStream_t s);

size_t sort_workspace_words(size_t n);
// Small batches of uniformly distributed keys (a churn's joins): top-bit
// buckets + per-bucket insertion sort; *overflow (device) != 0 = a bucket was
// too full (clustered input) and out is not sorted: use radix_sort.
size_t bucket_sort_workspace_words(size_t n);
hipError_t bucket_sort(const cell128 *keys, size_t n, cell128 *out, uint32_t *ws,
                       uint32_t *overflow, hipStream_t s);
// (keys, tags) by (key, tag) into (k0, t0) -- the stable key order when the
// tags ascend in input order; MSD buckets + LDS bucket sort, LSD fallback for
// clustered keys (one host synchronisation).  ws: sort_workspace_words(n).
hipError_t radix_sort(cell128 *k0, uint32_t *t0, cell128 *k1, uint32_t *t1, size_t n,
                      uint32_t *ws, hipStream_t s);
// *bad (device) = 0 iff (k, t) ascend by (key, tag).
hipError_t check_sorted(const cell128 *k, const uint32_t *t, size_t n, uint32_t *bad,
                        hipStream_t s);
// The 16-pass LSD sort alone (stable by key), for A/B timing.
hipError_t radix_sort_lsd(cell128 *k0, uint32_t *t0, cell128 *k1, uint32_t *t1, size_t n,
                          uint32_t *ws, hipStream_t s);
hipError_t unique_sorted(const cell128 *keys, const uint32_t *tags, size_t n, uint32_t *pos,
                         uint32_t *scan_ws, cell128 *out, uint32_t *old_to_new,
                         uint32_t *d_count, hipStream_t s);
hipError_t compact_survivors(const cell128 *ring, const uint8_t *gone, size_t n, uint32_t *pos,
                             uint32_t *scan_ws, cell128 *out_keys, uint32_t *out_tags,
                             uint32_t *d_count, hipStream_t s);
hipError_t copy_tagged(const cell128 *src, size_t n, uint32_t tag_base, cell128 *dk,
                       uint32_t *dt, hipStream_t s);
hipError_t iota(uint32_t *t, size_t n, uint32_t base, hipStream_t s);
hipError_t fill_u32(uint32_t *t, size_t n, uint32_t v, hipStream_t s);

hipError_t eyt_build(const cell128 *sorted, size_t n, cell128 *E, hipStream_t s);
hipError_t dir_build(const cell128 *ring, size_t n, int k, uint32_t *lo_tmp, uint4 *dir,
                     hipStream_t s);
hipError_t successor(const SearchView &ev, const cell128 *keys, size_t q, uint32_t *owner,
                     hipStream_t s);
// Streaming build when ring_key (ID slices at finger_key_shift(n),
// ring_slice_build) and ws (fingers_workspace_bytes) are given and the ring
// has >= 2^18 peers, else one directory search per entry.
size_t fingers_workspace_bytes(size_t n);
int finger_key_shift(size_t n);
hipError_t predecessor(const SearchView &ev, const cell128 *keys, size_t q, uint32_t *pred,
                       hipStream_t s);
// LDS slice tables of rings that fit LDS (search variants 1 and 4): the
// table's bytes for n peers and b bucket bits, its build, and the search
// (steps = binary-search rounds covering the largest bucket).
constexpr size_t SLICE_TAB_MAX = 160 * 1024;
size_t slice_tab_bytes(size_t n, int b, bool dev16 = false);
hipError_t slice_tab_build(const cell128 *ring, size_t n, int b, void *tab, hipStream_t s);
hipError_t successor_lds(const void *tab, int b, bool dev16, int steps, const cell128 *ring,
                         size_t n, const cell128 *keys, size_t q, uint32_t *out, bool pred,
                         hipStream_t s);
hipError_t fingers_build(const SearchView &sv, const cell128 *ring, const uint32_t *ring_key,
                         void *ws, uint32_t *F, hipStream_t s, uint32_t *FT = nullptr,
                         int Lft = 0, bool *planes_done = nullptr);
hipError_t ring_slice_build(const cell128 *ring, size_t n, int kb, uint32_t *key, hipStream_t s);
hipError_t route(const cell128 *ring, size_t n, const uint32_t *F, const cell128 *min_keys,
                 const uint32_t *preds, const LitState &ls, bool literal, const uint32_t *src,
                 const cell128 *keys, size_t q, uint32_t *owner, uint8_t *hops, uint8_t *status,
                 hipStream_t s);
hipError_t ring_ext_build(const cell128 *ring, size_t n, cell128 *ring_ext, hipStream_t s);
hipError_t tree_build(const uint32_t *F, const cell128 *ring, size_t n, int l0, int R, int ib,
                      uint64_t *tree, hipStream_t s);
hipError_t route_tree(const cell128 *ring_ext, const cell128 *ring, size_t n,
                      const uint64_t *tree, int l0, int R, int ib, const uint32_t *F,
                      const uint32_t *src, const cell128 *keys, size_t q, uint32_t *owner,
                      uint8_t *hops, uint8_t *status, hipStream_t s);
// Finger access for the route-table builds: F[x][l] = F[x * sx + (l - L) * sl]
// for l in [L, L + nl): the row-major table (sx = 128, sl = 1, L = 0,
// nl = 128) or level planes from fingers_levels (sx = 1, sl = n).
struct FingerView {
    const uint32_t *F;
    size_t sx, sl;
    int L, nl;
    // planes only, optional: two-hop planes C2[(l - L - 1) * sl + x] =
    // F[F[x][l]][l - 1] for l in (L, L + nl) (fingers_pairs)
    const uint32_t *C2 = nullptr;
    // host-side build choice: 2 = root-centric windows in blocks sized by
    // distinct roots (k_cz_build_roots2: needs C2 and rs), 0 = one lane per
    // entry (k_cz_build)
    int roots = 0;
    // root-centric build, optional: 32-bit ID slices (ring_codes) for the gap
    // codes instead of the 64-bit high words; only when every ring gap is
    // below 2^(gs + 17)
    const uint32_t *rs = nullptr;
    __host__ __device__ uint32_t at(uint32_t x, int l) const {
        return F[(size_t)x * sx + (size_t)(l - L) * sl];
    }
    static FingerView rows(const uint32_t *F) {
        return FingerView{F, CX_FINGERS, 1, 0, CX_FINGERS, nullptr, 0};
    }
    static FingerView planes(const uint32_t *FT, size_t n, int L, int nl) {
        return FingerView{FT, 1, n, L, nl, nullptr, 0};
    }
};
// Order-sensitive 64-bit hash of `bytes` (multiple of 8) into *out (device).
hipError_t table_hash(const void *t, size_t bytes, unsigned long long *out, hipStream_t s);
// Search variant 2: static 16-ary S+-tree over the ring (k_successor_stree).
#define CX_STREE_MAX 10
struct STreeView {
    const cell128 *lv[CX_STREE_MAX];  // lv[0] = the ring; lv[l][j] = ring[j * 16^l]
    uint32_t sz[CX_STREE_MAX];
    int top;                          // sz[top] <= 16
    size_t words;                     // cells of levels 1..top (buffer size)
    int lds_from;                     // levels >= lds_from are staged in LDS
    uint32_t lds_off[CX_STREE_MAX];   // their offsets there (cells)
};
STreeView stree_plan(const cell128 *ring, size_t n, cell128 *buf);
hipError_t stree_build(const STreeView &v, hipStream_t s);
hipError_t successor_stree(const STreeView &st, const cell128 *keys, size_t q, uint32_t *owner,
                           bool pred, hipStream_t s);
// Search variant 3: sixteen lanes per query over the Eytzinger copy, four
// levels per step (ballot of the subtree's 15 compares).
hipError_t eyt_rank_build(size_t n, uint32_t *rank, hipStream_t s);
hipError_t successor_eyt16(const EytView &ev, const uint32_t *rank, const cell128 *keys, size_t q,
                           uint32_t *owner, bool pred, hipStream_t s);
hipError_t fingers_levels(const uint32_t *F, size_t n, int L, int nl, uint32_t *FT,
                          hipStream_t s);
// C2 planes (nl - 1 of them) from the level planes FT.
hipError_t fingers_pairs(const uint32_t *FT, size_t n, int nl, uint32_t *C2, hipStream_t s);
// rh = the IDs' high words (ring_hi); the build needs l0 >= 69 and ib <= 51.
// esc[0] += slots not representable; esc[1] |= 1 if a finger was out of range.
hipError_t ring_hi(const cell128 *ring, size_t n, uint64_t *hi, hipStream_t s);
// rs[p] = bits [gs - 15, gs + 17) of ring[p] (gs = 116 - ib); *wide (device)
// = 1 if a cyclic ring gap reaches 2^(gs + 17): rs serves the root-centric
// build when *wide == 0.
hipError_t ring_codes(const cell128 *ring, size_t n, int ib, uint32_t *rs, uint32_t *wide,
                      hipStream_t s);
// ws (optional, cz_build_ws_words words): the overflow list of the default
// root-centric build (fv.roots == 2); without it the build takes 256-row blocks
hipError_t cz_build(const FingerView &fv, const cell128 *ring, const uint64_t *rh, size_t n,
                    int l0, int R, int ib, uint64_t *cz, uint32_t *esc, hipStream_t s,
                    uint32_t *ws = nullptr);
size_t cz_build_ws_words(size_t n, int lvl_base, int nlev, uint32_t M);
// Distinct roots per block before the default build defers rows to an
// overflow launch (256; tests only: lower, to exercise that path).
uint32_t cz2_cap();
void cz2_set_cap(uint32_t cap);
// The default walk (cx_walk.hip): straight-line window steps over the same
// table; n < 2^30, gs = cz_shift(ib) >= 64.
hipError_t route_walk(const cell128 *ring_ext, const cell128 *ring, size_t n, const uint64_t *cz,
                      int l0, int ib, const SearchView &sv, const uint32_t *src,
                      const cell128 *keys, size_t q, uint32_t *owner, uint8_t *hops,
                      uint8_t *status, unsigned long long *stats, hipStream_t s);
// Dependent random gathers of 64-B entries (four lanes, one 16-B load each),
// the walk's access pattern, over `bytes` of `table` (read only): entries/s.
hipError_t gather_probe(const void *table, size_t bytes, int lanes, int hops, double *rate,
                        hipStream_t s);
hipError_t cz_build_part(const FingerView &fv, const cell128 *ring, const uint64_t *rh, size_t n,
                         int lvl_base, int nlev, uint32_t p_first, uint32_t M, int ib,
                         uint64_t *cz, uint32_t *esc, hipStream_t s, uint32_t *ws = nullptr);
hipError_t route_arc(const cell128 *ring_ext, const cell128 *ring, size_t n, const uint64_t *cz,
                     int l0, int R, int ib, const SearchView &sv, int Lh, uint32_t plo, uint32_t M,
                     int self, const ArcRec *in, const uint32_t *src, const cell128 *keys, size_t q,
                     ArcRec *out, uint32_t *owner, uint8_t *hops, uint8_t *status, hipStream_t s);
// Key-first SoA protocol (cx_arc_partition / cx_arc_route / cx_arc_deliver):
// the straight-line walk (cx_walk.hip) over the rank's arc table, packed
// results in input order; dh = the origin's source hints or null.
hipError_t route_walk_arc(const cell128 *ring_ext, const cell128 *ring, size_t n,
                          const uint64_t *arc_tree, int l0, int ib, const SearchView &sv, int Lh,
                          uint32_t plo, uint32_t M, const uint32_t *src, const cell128 *keys,
                          size_t q, const uint64_t *dh, uint64_t *res, hipStream_t s);
// The arc rank's own lookups in place: keys[idx[j]] from src[idx[j]], outputs
// at idx[j] (cx_arc_route_local).
hipError_t route_walk_arc_local(const cell128 *ring_ext, const cell128 *ring, size_t n,
                                const uint64_t *arc_tree, int l0, int ib, const SearchView &sv,
                                int Lh, uint32_t plo, uint32_t M, const uint32_t *src,
                                const cell128 *keys, const uint32_t *idx, size_t q,
                                uint32_t *owner, uint8_t *hops, uint8_t *status, hipStream_t s);
hipError_t arc_partition(const uint32_t *src, const cell128 *keys, size_t q,
                         const ArcBound *bounds, int nb, int G, uint32_t *counts_dev,
                         uint32_t *cursor_dev, cell128 *skeys, uint32_t *ssrc, uint32_t *perm,
                         hipStream_t s);
hipError_t arc_partition_regions(const uint32_t *src, const cell128 *keys, size_t q,
                                 const ArcBound *bounds, int nb, int G, uint32_t cap,
                                 uint32_t *cursor_dev, uint32_t *ovf, cell128 *skeys,
                                 uint32_t *ssrc, uint32_t *perm, uint64_t *sd,
                                 const cell128 *ring_ext, size_t n, int ib, hipStream_t s);
// Device-side region cursors / counts of the single-pass partition (G <= 64).
// Exact-layout partition (ArcRouter's device-count path): per-destination
// counts of the lookups' keys (int64, zeroed first), then the scatter that
// lays destination d's lookups out at the sum of the counts below d.
hipError_t arc_count_keys(const cell128 *keys, size_t q, const ArcBound *bounds, int nb, int G,
                          int64_t *counts, int me, uint32_t *own_idx, uint32_t *own_ws,
                          hipStream_t s);
hipError_t arc_scatter_exact(const uint32_t *src, const cell128 *keys, size_t q,
                             const ArcBound *bounds, int nb, int G, const int64_t *counts,
                             uint32_t *cursor, cell128 *skeys, uint32_t *ssrc, uint32_t *perm,
                             uint64_t *sd, const cell128 *ring_ext, size_t n, int ib, int skip,
                             hipStream_t s);
hipError_t arc_cursor_init(uint32_t *cursor, uint32_t *ovf, int G, uint32_t cap, hipStream_t s);
hipError_t arc_counts_out(const uint32_t *cursor, const uint32_t *ovf, int G, uint32_t cap,
                          int64_t *counts, hipStream_t s);
hipError_t arc_deliver(const uint64_t *res, const uint32_t *perm, size_t q, uint32_t *owner,
                       uint8_t *hops, uint8_t *status, hipStream_t s);
hipError_t arc_seed(const uint32_t *src, const cell128 *keys, size_t q, int self, ArcRec *out,
                    hipStream_t s);
hipError_t arc_bucket(const ArcRec *recs, size_t q, const ArcBound *bounds, int nb, int G,
                      uint32_t *counts_dev, uint32_t *cursor_dev, ArcRec *send, hipStream_t s,
                      bool scatter);
// arc_bucket of the NEW records arc_seed would write for (src, keys), without
// writing them (lookups sent ahead by key).
hipError_t arc_bucket_seed(const uint32_t *src, const cell128 *keys, int self, size_t q,
                           const ArcBound *bounds, int nb, int G, uint32_t *counts_dev,
                           uint32_t *cursor_dev, ArcRec *send, hipStream_t s, bool scatter);
hipError_t nsucc(const SearchView &ev, const cell128 *keys, size_t q, int n, uint32_t *lists,
                 uint8_t *count, hipStream_t s);
hipError_t mark_leaves(const SearchView &ev, const cell128 *ring, const cell128 *leaves, size_t nl,
                       uint8_t *gone, hipStream_t s);
hipError_t merge_mark(const SearchView &sv, const cell128 *ring, const cell128 *leaves,
                      size_t nl, uint32_t *gone, hipStream_t s);
hipError_t merge_join_pos(const SearchView &sv, const cell128 *ring, size_t n,
                          const uint32_t *gone, const cell128 *J, size_t nj, uint32_t *pos,
                          uint32_t *keep, uint32_t *A, hipStream_t s);
hipError_t merge_scatter(const cell128 *ring, size_t n, const uint32_t *SG, const uint32_t *SA,
                         const cell128 *J, size_t nj, const uint32_t *pos, const uint32_t *kidx,
                         cell128 *out, uint32_t *o2n, hipStream_t s);
// Churn directory of (old ring, new ring, cx_churn's old_to_new): 2^kb
// buckets x 32 B (k_misplaced's one-gather path).  ok: device flag, nonzero
// when the caller's old_to_new equals the one the directory was built from.
struct ChurnDirArgs {
    const uint4 *cd;
    int kb;
    const uint32_t *ok;
};
hipError_t misplaced_churn(const SearchView &ev_old, const SearchView &ev_new,
                           const uint32_t *old_to_new, const cell128 *keys, size_t q, int n,
                           uint32_t *lists, uint8_t *count, uint16_t *mask, uint8_t *target,
                           const ChurnDirArgs *cda, hipStream_t s, uint32_t *old_lists = nullptr,
                           uint8_t *old_count = nullptr);
size_t churn_dir_workspace_bytes(size_t n_old, size_t n_new);
// lo: 2^kb + 1 words; scan_ws: scan_workspace_words(max(n_old, n_new) + 1).
hipError_t churn_dir_build(const SearchView &sv_old, const SearchView &sv_new,
                           const uint32_t *o2n, int kb, void *ws, uint32_t *lo, uint4 *cd,
                           uint32_t *scan_ws, uint32_t *M_out, hipStream_t s);
hipError_t churn_dir_same(const uint32_t *a, const uint32_t *b, size_t n, uint32_t *ok,
                          hipStream_t s);
hipError_t misplaced_holders(const SearchView &ev, const uint32_t *holders, int nh,
                             const cell128 *keys, size_t q, int n, uint32_t *lists,
                             uint8_t *count, uint16_t *mask, uint8_t *target, hipStream_t s);
hipError_t in_between(const cx_u256 *v, const cx_u256 *lb, const cx_u256 *ub, size_t q,
                      int inclusive, uint8_t *out, hipStream_t s);
hipError_t fill_splitmix(cell128 *out, size_t count, uint64_t seed, uint64_t offset,
                         hipStream_t s);
hipError_t uuid5(const uint8_t *bytes, const uint64_t *offs, size_t count, cell128 *out,
                 hipStream_t s);
hipError_t hex_parse(const uint8_t *bytes, const uint64_t *offs, size_t count, cell128 *out,
                     uint8_t *ok, hipStream_t s);
hipError_t hex_format(const cell128 *keys, size_t count, char *out, uint8_t *len, hipStream_t s);
hipError_t ida_encode(const uint8_t *data, const uint64_t *offs, const uint64_t *seg,
                      size_t blocks, int n, int m, int p, uint16_t *frags, hipStream_t s);
hipError_t ida_runs(const uint8_t *idx, size_t blocks, int m, uint32_t *flag, hipStream_t s);
hipError_t ida_run_index(const uint32_t *flag_excl, const uint32_t *flag_raw, size_t blocks,
                         size_t runs, uint32_t *run_of, uint32_t *run_start, uint32_t *err,
                         hipStream_t s);
hipError_t ida_inverse(const uint8_t *idx, const uint32_t *run_start, size_t runs, size_t blocks,
                       int m, int p, int32_t *inv, uint8_t *okf, uint32_t *err, hipStream_t s);
hipError_t ida_decode(const uint16_t *frags, const uint64_t *seg, size_t blocks, int m, int p,
                      const int32_t *inv, const uint32_t *run_of, size_t runs, const uint8_t *okf,
                      uint16_t *out, uint64_t *out_len, uint32_t *err, hipStream_t s);
hipError_t ida_mark_failed(const uint32_t *run_of, const uint8_t *okf, size_t blocks, size_t runs,
                           uint64_t *out_len, uint32_t *err, hipStream_t s);
hipError_t ida_check_guard(const uint32_t *guard, int words, uint32_t *err, hipStream_t s);
hipError_t check_indices(const uint32_t *idx, size_t count, uint32_t limit, bool allow_none,
                         uint32_t *d_bad, hipStream_t s);

}  // namespace cxk
