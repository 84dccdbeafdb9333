// cx_walk.hip -- the default finger-routed walk with hop counts: cx_route on a
// converged ring of <= 2^24 peers over the pattern-keyed window table
// (DESIGN.md 4.1).  SURVEY 8(a) rows a5, a7, a8, a9 (converged, all alive):
//   AbstractChordPeer::GetSuccessor   abstract_chord_peer.cpp:318-337
//   StoredLocally                     abstract_chord_peer.cpp:720-725
//   ChordPeer::ForwardRequest         chord_peer.cpp:185-211 (one hop = one GET_SUCC)
//   FingerTable::Lookup               finger_table.h:115-130 (level = msb(key - id))
//
// One lane walks one lookup; a wave keeps 64 walks in flight and advances all
// of them by one memory round per loop iteration.  The table stores, per
// (level i, pattern bit b, peer p), 16 relative nodes: the root A = f(p, i) and
// the nodes reached from A (b = 0) or from A' = f(A, i - 1) (b = 1) by every
// subset of hops at levels i-2 .. i-5 (cx_kernels.hip, k_cz_build*).  After a
// gather the lane takes the root hop and then steps the window's levels
// i-1 .. i-5 in a fixed, fully unrolled order: a hop at level l is due iff
// d >= 2^l, and d < 2^(l+1) holds at every step (a hop at l leaves d < 2^l).
// All lanes run the same straight-line steps -- no data-dependent loop -- so a
// round costs the same VALU work whatever mix of hops the wave's lanes take.
//
// Distances are kept in units u = 2^gs as an interval [dmin, dmax] (the gap
// codes are floor(gap / u)): a decision the interval cannot take exactly
// fetches the exact IDs (M_FIX: id(cur); M_FIXT: id(cur), id(next)).  Levels
// below the table, below gs, and nodes the format could not represent take
// exact hops (M_EXACT: id(cur), id(cur + 1), the directory if the finger is
// not the next peer).
#include "cx_kernels.hpp"

namespace cxk {
namespace {

constexpr int WK_BLOCK = 256;
constexpr uint32_t WK_NONE = 0xFFFFFFFFu;
constexpr uint32_t WK_CZ_NONE = 0xFFFFFFFFu;  // a node the 4-B format cannot hold (CZ_NONE)
constexpr uint32_t CX_QI_ARC_MISS = 0xFE;     // key-first arc walk left the rank's rows

enum { M_NONE = 0, M_HOP = 1, M_FIX = 2, M_EXACT = 3, M_FIXT = 4 };
enum { B_EMPTY = 0, B_KEYS = 1, B_READY = 2, B_IDX = 3 };
enum { P_WALK = 0, P_LOCAL = 1, P_BAD = 2 };

struct WalkIO {
    const cell128 *ring_ext;  // [ring[n-1], ring[0..n-1]]: (pred, self) of p at p, p + 1
    const cell128 *ring;
    uint32_t n;
    const uint4 *cz;  // [R][2][n] entries of 64 B (level-major)
    int l0, gs;
    SearchView sv;
    const uint32_t *src;
    const cell128 *keys;
    size_t q, chunk;
    uint32_t *owner;
    uint8_t *hops, *status;
    // counting build: [0] table gathers, [1] exact 16-B ID gathers, [2] exact
    // hops through the directory (a directory entry + an ID each), [3] lookups
    unsigned long long *stats;
    // key-first arc walk (KF): the rank's arc table = the replicated planes of
    // levels [Lh, 128) for all n peers, then the planes of levels [l0, Lh) for
    // the M peers plo, plo + 1, ... (cyclic: the arc and its halo); lookups
    // start from the origin's hint dh; packed results in input order (res_out)
    int Lh;
    uint32_t plo, M;
    const uint64_t *dh;
    uint64_t *res_out;
    // IX: the lookups are keys[idx[j]], src[idx[j]] (j < q), their outputs
    // owner / hops / status at idx[j] (an arc rank's own lookups, walked in
    // place without leaving the origin's arrays)
    const uint32_t *idx;
};

// E(l) = round(n 2^(l - 128)), the expected index advance of a level-l finger
// (n < 2^30: 32-bit arithmetic is exact).
__device__ __forceinline__ uint32_t wk_expect(uint32_t n, int l) {
    const int sh = 128 - l;
    return sh >= 32 ? 0u : (n + (1u << (sh - 1))) >> sh;
}

// Node word -> peer index: cur + E(l) + advance (stored + 2^15); Etab[l] =
// E(l) - 2^15.  t lies in (-n/2, 2n): one of t, t + n, t - n is in [0, n),
// and as u32 it is the smallest of the three (n < 2^30).
__device__ __forceinline__ uint32_t wk_next(const uint32_t *Etab, uint32_t n, uint32_t cur, int l,
                                            uint32_t wd) {
    const uint32_t t = cur + Etab[l] + (wd & 0xFFFFu);
    return min(t, min(t + n, t - n));
}

// floor(x / 2^gs) for gs >= 64 (ib <= 24 -> gs >= 92).
__device__ __forceinline__ uint64_t wk_units(u128 x, int gs) {
    return (uint64_t)(x >> 64) >> (gs - 64);
}

__device__ __forceinline__ u128 wk_u128(const unsigned int __attribute__((ext_vector_type(4))) v) {
    return ((u128)(((uint64_t)v.w << 32) | v.z) << 64) | (((uint64_t)v.y << 32) | v.x);
}

__device__ __forceinline__ uint64_t wk_pack(uint32_t own, uint32_t h, uint32_t st) {
    return (1ull << 63) | ((uint64_t)st << 40) | ((uint64_t)(h & 0xFF) << 32) | own;
}

#ifdef CX_WALK_WPE
#define WK_ATTR __attribute__((amdgpu_waves_per_eu(CX_WALK_WPE)))
#else
#define WK_ATTR
#endif

template <bool STATS, bool KF, bool IX = false>
__global__ __launch_bounds__(WK_BLOCK) WK_ATTR void k_walk(WalkIO io) {
    constexpr bool PACK = KF && !IX;  // packed results in input order (res_out)
    // entries land by LDS-DMA: region k of a wave = the 16-B quarters its
    // lanes loaded in gather k, lane-linear; lane j's entry is 64 contiguous
    // bytes in region j & 3 at (j >> 2) * 64 (regions 4 dwords apart mod 32
    // banks: <= 4-way ds_read_b32 conflicts)
    constexpr int RG = 260;
    __shared__ uint32_t ent_all[WK_BLOCK / 64][4 * RG];
    __shared__ uint32_t Etab[CX_FINGERS];  // E(l) - 2^15 per level
    const uint32_t n = io.n;
    for (int l = threadIdx.x; l < (int)CX_FINGERS; l += WK_BLOCK) Etab[l] = wk_expect(n, l) - 32768u;
    __syncthreads();
    const int l0 = io.l0, gs = io.gs;
    const int lane = threadIdx.x & 63, qs = threadIdx.x & 3;
    uint32_t *ent_w = ent_all[threadIdx.x >> 6];
    const uint32_t *ent = ent_w + (lane & 3) * RG + (lane >> 2) * 16;
    // wave-uniform by construction; readfirstlane tells the compiler, so base
    // and every array pointer below live in SGPRs (6 VGPRs fewer)
    const size_t wave = __builtin_amdgcn_readfirstlane(
        (uint32_t)((blockIdx.x * (size_t)WK_BLOCK + threadIdx.x) >> 6));
    const size_t base = wave * io.chunk;
    if (base >= io.q) return;  // wave-uniform
    // lookups [base, base + cnt) of the batch, by offset from base (32-bit:
    // chunk < 2^32); results are stored as each lookup finishes (a wave's
    // lookups finish within a few hundred of each other, so its scattered
    // 4-B / 1-B stores fill the same few lines, merged in L2)
    const uint32_t cnt = (uint32_t)((base + io.chunk < io.q) ? io.chunk : io.q - base);
    // IX: lookup "offsets" are the indices idx[] names, relative to the arrays
    const size_t ab = IX ? 0 : base;
    uint32_t *const own_w = PACK ? nullptr : io.owner + ab;
    uint8_t *const hop_w = PACK ? nullptr : io.hops + ab;
    uint8_t *const st_w = PACK || !io.status ? nullptr : io.status + ab;
    uint64_t *const res_w = PACK ? io.res_out + base : nullptr;
    const cell128 *const key_r = io.keys + ab;
    const uint32_t *const src_r = io.src + ab;
    const uint64_t *const dh_r = PACK && io.dh ? io.dh + base : nullptr;
    const uint32_t *const idx_r = IX ? io.idx + base : nullptr;
    auto put = [&](uint32_t o, uint32_t ow, uint32_t hh, uint32_t st) {
        if (PACK) {
            res_w[o] = wk_pack(ow, hh, st);
        } else {
            own_w[o] = ow;
            hop_w[o] = (uint8_t)hh;
            if (st_w) st_w[o] = (uint8_t)st;
        }
    };
    uint32_t head = 0;

    // slot A: the lookup being walked
    int mode = M_NONE, lvl = 0, rb = 0;
    uint32_t cur = 0, h = 0, pn = 0;
    uint64_t dmin = 0, dmax = 0;
    u128 key = 0;
    uint32_t qi = 0;
    // slot B: the next lookup (key + source, then the source's ID pair)
    int bst = B_EMPTY, pst = P_WALK;
    uint32_t pq = 0;
    u128 pkey = 0;
    uint32_t psrc = 0;
    uint64_t pd = 0;
    uint32_t n_g64 = 0, n_r16 = 0, n_xc = 0, n_q = 0;
    const uint32_t arc_top = KF ? (uint32_t)(CX_FINGERS - io.Lh) * 2u * n : 0u;  // KF: local rows

    for (;;) {
        if (__ballot(mode != M_NONE || bst != B_EMPTY) == 0 && head >= cnt)
            break;  // wave-uniform: every lookup delivered

        // ---- memory round: every load of the round, one wait ----
        uint32_t eidx = WK_NONE;
        if (mode == M_HOP) {
            if (!KF)
                eidx = (uint32_t)((lvl - l0) * 2 + rb) * n + cur;
            else if (lvl >= io.Lh)  // replicated top planes, all peers
                eidx = (uint32_t)((lvl - io.Lh) * 2 + rb) * n + cur;
            else  // this rank's rows (checked local by the plan)
                eidx = arc_top + (uint32_t)((lvl - l0) * 2 + rb) * io.M +
                       (cur >= io.plo ? cur - io.plo : cur + n - io.plo);
        }
        if (STATS) {
            n_g64 += mode == M_HOP;
            n_r16 += mode == M_FIX ? 1u : (mode >= M_EXACT ? 2u : 0u);
        }
        // Load order: the source pairs of the lookups refilled last round
        // (their psrc is read before this round's refill loads overwrite it
        // for other lanes), the refill, the table entries, exact IDs.  The
        // pair and ID values are made opaque until every load is issued
        // (wk_opaque), so no early wait on them splits the round's loads.
        typedef unsigned int v4n __attribute__((ext_vector_type(4)));
        const bool pair_now = bst == B_KEYS;
        v4n pa4 = {0, 0, 0, 0}, pb4 = {0, 0, 0, 0};
        if ((!PACK || !io.dh) && pair_now && psrc < n) {  // the source's (pred, self) IDs: one 32-B pair
            pa4 = __builtin_nontemporal_load(reinterpret_cast<const v4n *>(io.ring_ext + psrc));
            pb4 = __builtin_nontemporal_load(reinterpret_cast<const v4n *>(io.ring_ext + psrc + 1));
        }
        if (IX && bst == B_IDX) {  // the index arrived last round: key and source
            pkey = ld128(key_r + pq);
            psrc = src_r[pq];
            bst = B_KEYS;
        }
        {  // refill slot B in lookup order
            const uint32_t avail = cnt - head;
            const uint64_t want = __ballot(bst == B_EMPTY);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
            if (bst == B_EMPTY && rank < avail) {
                if (IX) {  // the lookup's index first (one more round of the pipeline)
                    pq = idx_r[head + rank];
                    bst = B_IDX;
                } else {
                    pq = head + rank;
                    pkey = ld128(key_r + pq);
                    psrc = src_r[pq];
                    if (PACK && io.dh) pd = dh_r[pq];  // the origin's start: d >> gs, or LOCAL / BAD
                    bst = B_KEYS;
                }
            }
            const uint32_t took = (uint32_t)__popcll(want);
            head += took < avail ? took : avail;
        }
        // quad-cooperative 64-B gathers straight into LDS (LDS-DMA): lane qs of
        // each quad loads 16 B of the four entries its quad wants, one load
        // instruction = 16 lines (quad_perm broadcast of lane k: dpp k * 0x55)
        const uint32_t ek[4] = {(uint32_t)__builtin_amdgcn_mov_dpp((int)eidx, 0x00, 0xF, 0xF, false),
                                (uint32_t)__builtin_amdgcn_mov_dpp((int)eidx, 0x55, 0xF, 0xF, false),
                                (uint32_t)__builtin_amdgcn_mov_dpp((int)eidx, 0xAA, 0xF, 0xF, false),
                                (uint32_t)__builtin_amdgcn_mov_dpp((int)eidx, 0xFF, 0xF, 0xF, false)};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (ek[k] != WK_NONE)
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void *)(io.cz + (size_t)ek[k] * 4 + qs),
                    (__attribute__((address_space(3))) void *)(ent_w + k * RG), 16, 0, 2 /* nt */);
        v4n xa4 = {0, 0, 0, 0}, xb4 = {0, 0, 0, 0};
        if (mode >= M_FIX) {
            xa4 = *reinterpret_cast<const v4n *>(io.ring + cur);
            if (mode != M_FIX)
                xb4 = *reinterpret_cast<const v4n *>(io.ring + (mode == M_FIXT ? pn : (cur + 1 == n ? 0u : cur + 1)));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA landed
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        asm volatile("" : "+v"(pa4), "+v"(pb4), "+v"(xa4), "+v"(xb4));  // wk_opaque
        const u128 pa = wk_u128(pa4), pb = wk_u128(pb4), xa = wk_u128(xa4), xb = wk_u128(xb4);

        // ---- slot B: StoredLocally at the source, or the start distance ----
        if (PACK && io.dh && pair_now) {  // the origin resolved the start (k_arc_scatter_soa)
            pst = psrc >= n || pd == ARC_HINT_BAD ? P_BAD : (pd == ARC_HINT_LOCAL ? P_LOCAL : P_WALK);
            bst = B_READY;
        } else if (pair_now) {
            if (psrc >= n) {
                pst = P_BAD;
            } else if (n == 1 || (pkey - pa - 1) <= (pb - pa - 1)) {
                pst = P_LOCAL;  // key in (pred, src]: 0 hops
            } else {
                pst = P_WALK;
                pd = wk_units(pkey - pb, gs);
            }
            bst = B_READY;
        }

        uint32_t own = CX_NONE, st = CX_Q_OK;
        bool fin = false, plan = false;
        // ---- exact IDs arrived (rare) ----
        if (mode >= M_FIX) {
            const u128 d = key - xa;
            if (mode == M_FIX) {
                dmin = dmax = wk_units(d, gs);
                plan = true;
            } else if (mode == M_FIXT) {  // the undecided StoredLocally(pn), exactly
                if (d <= xb - xa) {
                    fin = true;
                    own = pn;
                } else {
                    cur = pn;
                    dmin = dmax = wk_units(key - xb, gs);
                    plan = true;
                }
            } else {  // M_EXACT: the exact finger at level msb(d) = succ(id + 2^i)
                const int i = msb128(d);
                const u128 step = pow2_128(i);
                uint32_t nxt;
                u128 idn;
                if (step <= xb - xa) {  // the next peer
                    nxt = cur + 1 == n ? 0u : cur + 1;
                    idn = xb;
                } else {
                    nxt = dir_successor(io.sv, xa + step);
                    idn = ld128(io.ring + nxt);
                    if (STATS) ++n_xc;
                }
                ++h;
                if (d <= idn - xa) {
                    fin = true;
                    own = nxt;
                } else {
                    cur = nxt;
                    dmin = dmax = wk_units(key - idn, gs);
                    plan = true;
                }
            }
        }

        // ---- table entry arrived: root hop, then the window's five levels ----
        // Straight-line, branch-free steps (selects): every lane runs the same
        // instructions whatever hops it takes.  No hop cap here: on a converged
        // ring each hop strictly lowers msb(d) (d' = d - (id_nxt - id_cur) <
        // 2^i), so a walk takes <= 128 < CX_HOP_CAP hops.
        int cs = -1, ri = 0;  // cs: window subset the lane stands on (16: root A of b = 1)
        if (mode == M_HOP) {
            const uint32_t wd = ent[rb ? 15 : 0];
            ri = lvl;
            if (wd == WK_CZ_NONE) {
                mode = M_EXACT;  // the root is not representable: exact finger next round
            } else {
                const uint64_t e = (1ull << (lvl - gs)) + (wd >> 16);
                const uint32_t nxt = wk_next(Etab, n, cur, lvl, wd);
                ++h;
                if (dmax < e) {
                    fin = true;
                    own = nxt;
                } else if (dmin <= e) {
                    mode = M_FIXT;
                    pn = nxt;
                } else {
                    cur = nxt;
                    dmin -= e + 1;
                    dmax -= e;
                    cs = rb ? 16 : 0;
                }
            }
        }
#pragma unroll
        for (int o = 1; o <= 5; ++o) {
            const int l = ri - o;
            const bool act = cs >= 0 && l >= gs;
            const uint64_t T = 1ull << ((l - gs) & 63);  // d >= 2^l <=> floor(d/u) >= T
            const bool need = act && dmax >= T;           // a hop at level l is due (or undecided)
            int v;
            bool vv;
            if (o == 1) {
                v = 0;
                vv = cs == 16;  // b = 1: A -> A' (slot 0)
            } else {
                v = (cs & 15) | (1 << (o - 2));
                vv = cs < 16 && !(rb && v == 15);  // slot 15 of a b = 1 entry is A
            }
            const uint32_t wd = ent[v];
            const bool ok = need && vv && dmin >= T && wd != WK_CZ_NONE;
            const uint64_t e = T + (wd >> 16);
            const uint32_t nxt = wk_next(Etab, n, cur, l, wd);
            const bool own_now = ok && dmax < e;
            const bool und = ok && !own_now && dmin <= e;
            const bool mv = ok && !own_now && !und;
            h += ok ? 1u : 0u;
            if (own_now) own = nxt;
            fin = fin || own_now;
            if (und) {
                pn = nxt;
                mode = M_FIXT;
            }
            cur = mv ? nxt : cur;
            dmin = mv ? dmin - e - 1 : dmin;
            dmax = mv ? dmax - e : dmax;
            cs = mv ? v : ((need || !act) ? -1 : cs);  // left the window unless moved / not due
        }
        if (mode == M_HOP && !fin) plan = true;

        // ---- deliver, promote slot B ----
        if (fin) {
            put(qi, own, h, st);
            mode = M_NONE;
        }
        if (!plan && mode == M_NONE && bst == B_READY) {
            bst = B_EMPTY;
            qi = pq;
            key = pkey;
            cur = psrc;
            h = 0;
            if (STATS) ++n_q;
            if (pst == P_WALK) {
                dmin = dmax = pd;
                plan = true;
            } else {
                put(qi, pst == P_LOCAL ? cur : CX_NONE, 0, pst == P_LOCAL ? CX_Q_OK : CX_Q_BADPEER);
            }
        }

        // ---- plan: the next level and what it needs ----
        if (plan) {
            if (dmin == 0) {
                mode = M_EXACT;  // d < 2^gs
            } else {
                const int ma = 63 - __builtin_clzll(dmin), mb = 63 - __builtin_clzll(dmax);
                if (ma != mb) {
                    mode = M_FIX;  // the level itself is undecided
                } else if (ma + gs >= l0) {
                    mode = M_HOP;
                    lvl = ma + gs;
                    rb = ma >= 1 ? (int)((dmax >> (ma - 1)) & 1) : 0;  // bit lvl-1 of d
                    if (KF && lvl < io.Lh && (cur >= io.plo ? cur - io.plo : cur + n - io.plo) >= io.M) {
                        // a row outside the rank's arc + halo: a layout bug (the
                        // lookup was sent to its key's arc), reported, never seen
                        mode = M_NONE;
                        put(qi, CX_NONE, h, CX_QI_ARC_MISS);
                    }
                } else {
                    mode = M_EXACT;  // below the table
                }
            }
        }
    }
    if (STATS) {
        uint64_t v[4] = {n_g64, n_r16, n_xc, n_q};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off, 64);
        }
        if (lane == 0)
#pragma unroll
            for (int k = 0; k < 4; ++k) atomicAdd(io.stats + k, (unsigned long long)v[k]);
    }
}

// Waves per SIMD the walk runs at (one 256-thread block = one wave per SIMD
// of a CU).  The register budget allows 8 (57 VGPRs) but 8 measured slower
// than 7 (3.43-3.45 vs 3.27 ms, profiles/r05/walk_ab/w8_vs_w7): past ~4.6 x
// 10^5 walks in flight the random-request latency grows faster than the
// requests.  Dynamic LDS holds a launch to CX_WALK_WAVES blocks per CU.
// Fewest lookups per wave of a launch (small batches): one per lane.  A walk
// is a chain of dependent gathers, so a batch below one resident round of
// waves is fastest spread over as many waves as it fills; at >= 1024 per wave
// (before round 5) a 2^16 / 2^18 / 2^20 / 2^22 batch took 159 / 167 / 175 /
// 443 us, at 64 per wave 24 / 39 / 123 / 417 us (profiles/r05/walk_q/minq/).
constexpr size_t WK_MIN_PER_WAVE = 64;
#ifndef CX_WALK_WAVES
#define CX_WALK_WAVES 7
#endif

template <class K>
size_t walk_lds_pad(K kernel) {
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(kernel)) != hipSuccess) return 0;
    const size_t lds = 160 * 1024, cap = lds / (CX_WALK_WAVES + 1) + 256;  // > 1/(w+1) of LDS
    return fa.sharedSizeBytes < cap ? cap - fa.sharedSizeBytes : 0;
}

template <class K>
unsigned walk_resident_grid(K kernel, size_t pad) {
    int dev = 0, cus = 256, per = 1;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, WK_BLOCK, pad) != hipSuccess ||
        per < 1)
        per = 1;
    return (unsigned)(per * cus);
}

}  // namespace

hipError_t route_walk(const cell128 *ring_ext, const cell128 *ring, size_t n, const uint64_t *cz,
                      int l0, int ib, const SearchView &sv, const uint32_t *src,
                      const cell128 *keys, size_t q, uint32_t *owner, uint8_t *hops,
                      uint8_t *status, unsigned long long *stats, hipStream_t s) {
    if (q == 0) return hipSuccess;
    const int gs = cz_shift(ib);
    // the walk's index and distance arithmetic: n < 2^30, u = 2^gs with gs >= 64,
    // 32-bit entry indices (l0 - 5 >= 0 levels x 2 x n < 2^32)
    if (n == 0 || n >= (1u << 30) || gs < 64 || l0 < 5 || (size_t)(128 - l0) * 2 * n >= WK_NONE)
        return hipErrorInvalidValue;
    WalkIO io = {};
    io.ring_ext = ring_ext;
    io.ring = ring;
    io.n = (uint32_t)n;
    io.cz = reinterpret_cast<const uint4 *>(cz);
    io.l0 = l0;
    io.gs = gs;
    io.sv = sv;
    io.src = src;
    io.keys = keys;
    io.q = q;
    io.owner = owner;
    io.hops = hops;
    io.status = status;
    io.stats = stats;
    // one resident round of waves (no second, partial round of blocks); small
    // batches: >= WK_MIN_PER_WAVE lookups per wave
    static const size_t pad = walk_lds_pad(k_walk<false, false>);
    static const unsigned resident = walk_resident_grid(k_walk<false, false>, pad);
    size_t waves = (size_t)resident * (WK_BLOCK / 64);
    const size_t small = (q + WK_MIN_PER_WAVE - 1) / WK_MIN_PER_WAVE;
    if (small < waves) waves = small ? small : 1;
    io.chunk = (q + waves - 1) / waves;
    if (io.chunk >= (1ull << 32)) return hipErrorInvalidValue;  // 32-bit lookup offsets
    waves = (q + io.chunk - 1) / io.chunk;
    const unsigned blocks = (unsigned)((waves * 64 + WK_BLOCK - 1) / WK_BLOCK);
    if (stats)
        k_walk<true, false><<<blocks, WK_BLOCK, pad, s>>>(io);
    else
        k_walk<false, false><<<blocks, WK_BLOCK, pad, s>>>(io);
    return hipGetLastError();
}

// Key-first arc walk (chordx.arc.ArcRouter's default protocol): the
// lookups this rank received for its arc, walked from their sources over the
// replicated top planes [Lh, 128) and its own rows below, started from the
// origin's hints (dh: d >> gs, ARC_HINT_LOCAL, ARC_HINT_BAD; or, without
// dh, from the source's (pred, self) IDs like the replicated walk); one packed
// result (owner | hops << 32 | status << 40 | 1 << 63) per lookup in input
// order.
hipError_t route_walk_arc(const cell128 *ring_ext, const cell128 *ring, size_t n,
                          const uint64_t *arc_tree, int l0, int ib, const SearchView &sv, int Lh,
                          uint32_t plo, uint32_t M, const uint32_t *src, const cell128 *keys,
                          size_t q, const uint64_t *dh, uint64_t *res, hipStream_t s) {
    if (q == 0) return hipSuccess;
    const int gs = cz_shift(ib);
    if (n == 0 || n >= (1u << 30) || gs < 64 || l0 < 5 || Lh < l0 || Lh > (int)CX_FINGERS ||
        M > n || (size_t)(CX_FINGERS - Lh) * 2 * n + (size_t)(Lh - l0) * 2 * M >= WK_NONE)
        return hipErrorInvalidValue;
    WalkIO io = {};
    io.ring_ext = ring_ext;
    io.ring = ring;
    io.n = (uint32_t)n;
    io.cz = reinterpret_cast<const uint4 *>(arc_tree);
    io.l0 = l0;
    io.gs = gs;
    io.sv = sv;
    io.src = src;
    io.keys = keys;
    io.q = q;
    io.Lh = Lh;
    io.plo = plo;
    io.M = M;
    io.dh = dh;
    io.res_out = res;
    static const size_t pad = walk_lds_pad(k_walk<false, true>);
    static const unsigned resident = walk_resident_grid(k_walk<false, true>, pad);
    size_t waves = (size_t)resident * (WK_BLOCK / 64);
    const size_t small = (q + WK_MIN_PER_WAVE - 1) / WK_MIN_PER_WAVE;
    if (small < waves) waves = small ? small : 1;
    io.chunk = (q + waves - 1) / waves;
    if (io.chunk >= (1ull << 32)) return hipErrorInvalidValue;  // 32-bit lookup offsets
    waves = (q + io.chunk - 1) / io.chunk;
    const unsigned blocks = (unsigned)((waves * 64 + WK_BLOCK - 1) / WK_BLOCK);
    k_walk<false, true><<<blocks, WK_BLOCK, pad, s>>>(io);
    return hipGetLastError();
}

// An arc rank's own lookups in place (ArcRouter.route_exact): the key-first
// arc walk over keys[idx[j]] from src[idx[j]] (started from the source's
// (pred, self) IDs, no hints), owner / hops / status written at idx[j].
hipError_t route_walk_arc_local(const cell128 *ring_ext, const cell128 *ring, size_t n,
                                const uint64_t *arc_tree, int l0, int ib, const SearchView &sv,
                                int Lh, uint32_t plo, uint32_t M, const uint32_t *src,
                                const cell128 *keys, const uint32_t *idx, size_t q,
                                uint32_t *owner, uint8_t *hops, uint8_t *status, hipStream_t s) {
    if (q == 0) return hipSuccess;
    const int gs = cz_shift(ib);
    if (n == 0 || n >= (1u << 30) || gs < 64 || l0 < 5 || Lh < l0 || Lh > (int)CX_FINGERS ||
        M > n || (size_t)(CX_FINGERS - Lh) * 2 * n + (size_t)(Lh - l0) * 2 * M >= WK_NONE)
        return hipErrorInvalidValue;
    WalkIO io = {};
    io.ring_ext = ring_ext;
    io.ring = ring;
    io.n = (uint32_t)n;
    io.cz = reinterpret_cast<const uint4 *>(arc_tree);
    io.l0 = l0;
    io.gs = gs;
    io.sv = sv;
    io.src = src;
    io.keys = keys;
    io.q = q;
    io.owner = owner;
    io.hops = hops;
    io.status = status;
    io.Lh = Lh;
    io.plo = plo;
    io.M = M;
    io.idx = idx;
    static const size_t pad = walk_lds_pad(k_walk<false, true, true>);
    static const unsigned resident = walk_resident_grid(k_walk<false, true, true>, pad);
    size_t waves = (size_t)resident * (WK_BLOCK / 64);
    const size_t small = (q + WK_MIN_PER_WAVE - 1) / WK_MIN_PER_WAVE;
    if (small < waves) waves = small ? small : 1;
    io.chunk = (q + waves - 1) / waves;
    if (io.chunk >= (1ull << 32)) return hipErrorInvalidValue;  // 32-bit lookup offsets
    waves = (q + io.chunk - 1) / io.chunk;
    const unsigned blocks = (unsigned)((waves * 64 + WK_BLOCK - 1) / WK_BLOCK);
    k_walk<false, true, true><<<blocks, WK_BLOCK, pad, s>>>(io);
    return hipGetLastError();
}

}  // namespace cxk
