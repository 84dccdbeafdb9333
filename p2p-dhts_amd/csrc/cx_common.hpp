// cx_common.hpp -- shared device/host definitions for the chordx HIP engine.
//
// Ring values are unsigned 128-bit (ChordKey = GenericKey<16,32>, key.h:355).
// In HBM a value is one 16-byte cell {lo, hi} (cx_u128); in registers it is an
// unsigned __int128, which hipcc lowers to 64-bit VALU pairs on gfx950.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/chordx.h"

typedef unsigned __int128 u128;

struct alignas(16) cell128 {
    uint64_t lo, hi;
};
static_assert(sizeof(cell128) == 16, "cell128 must be 16 B");
static_assert(sizeof(cx_u128) == 16, "cx_u128 must be 16 B");

__host__ __device__ __forceinline__ u128 to_u128(cell128 c) {
    return ((u128)c.hi << 64) | c.lo;
}
__host__ __device__ __forceinline__ cell128 to_cell(u128 v) {
    cell128 c;
    c.lo = (uint64_t)v;
    c.hi = (uint64_t)(v >> 64);
    return c;
}

// One 16-byte load (global_load_dwordx4) of a ring cell.
__device__ __forceinline__ u128 ld128(const cell128 *p) {
    const uint4 v = *reinterpret_cast<const uint4 *>(p);
    return ((u128)(((uint64_t)v.w << 32) | v.z) << 64) | (((uint64_t)v.y << 32) | v.x);
}
// ... non-temporal (read once, nothing to keep in L2 for)
__device__ __forceinline__ u128 ld128_nt(const cell128 *p) {
    typedef unsigned int v4n __attribute__((ext_vector_type(4)));
    const v4n v = __builtin_nontemporal_load(reinterpret_cast<const v4n *>(p));
    return ((u128)(((uint64_t)v.w << 32) | v.z) << 64) | (((uint64_t)v.y << 32) | v.x);
}
__device__ __forceinline__ void st128(cell128 *p, u128 x) {
    uint4 v;
    v.x = (uint32_t)x;
    v.y = (uint32_t)(x >> 32);
    v.z = (uint32_t)(x >> 64);
    v.w = (uint32_t)(x >> 96);
    *reinterpret_cast<uint4 *>(p) = v;
}

// Variable shifts of 128-bit ring values, spelled in 64-bit halves.  Round 6
// (profiles/r06/u128/): the compiled level-plane route-table
// build with the round-5 gap code -- a u128 `>> gs` in a lane-divergent
// branch -- wrote nondeterministic words, only in lanes 48-63 of a wave and
// only in its slot-8 encode, with its inputs built on the host and no race
// in the kernel; the same encode in the row-major build, standalone, and the
// i128 shift itself (every amount, VGPR / SGPR amounts, divergent) were
// exact.  Instruction padding cut the rate 8x without removing it.  No device
// code shifts a u128 by a variable amount any more; these helpers take every
// such shift (amounts in [0, 128); a uniform amount keeps them scalar).
__host__ __device__ __forceinline__ u128 make128(uint64_t hi, uint64_t lo) {
    return ((u128)hi << 64) | lo;
}
__host__ __device__ __forceinline__ uint64_t hi64(u128 v) { return (uint64_t)(v >> 64); }
__host__ __device__ __forceinline__ uint64_t lo64(u128 v) { return (uint64_t)v; }
// 2^s
__host__ __device__ __forceinline__ u128 pow2_128(int s) {
    const uint64_t b = 1ull << (s & 63);
    return s < 64 ? make128(0, b) : make128(b, 0);
}
// v >> s
__host__ __device__ __forceinline__ u128 shr128(u128 v, int s) {
    const uint64_t hi = hi64(v), lo = lo64(v);
    if (s == 0) return v;
    if (s < 64) return make128(hi >> s, (lo >> s) | (hi << (64 - s)));
    return make128(0, hi >> (s - 64));
}
// v << s
__host__ __device__ __forceinline__ u128 shl128(u128 v, int s) {
    const uint64_t hi = hi64(v), lo = lo64(v);
    if (s == 0) return v;
    if (s < 64) return make128((hi << s) | (lo >> (64 - s)), lo << s);
    return make128(lo << (s - 64), 0);
}
// the 64 bits of v from bit s up: (uint64_t)(v >> s)
__host__ __device__ __forceinline__ uint64_t bits64(u128 v, int s) { return lo64(shr128(v, s)); }
// the top k bits, v >> (128 - k), for 0 <= k <= 64 (directory buckets)
__host__ __device__ __forceinline__ uint64_t top_bits(u128 v, int k) {
    return k >= 64 ? hi64(v) : (k <= 0 ? 0 : hi64(v) >> (64 - k));
}
// (uint64_t)(v >> (64 - k)) for 0 <= k <= 63: ID bits [64 - k, 128 - k)
__host__ __device__ __forceinline__ uint64_t mid_bits(u128 v, int k) {
    return k == 0 ? lo64(v) : (hi64(v) << k) | (lo64(v) >> (64 - k));
}

// floor(log2(d)) for d != 0: the finger index FingerTable::Lookup's first-match
// scan selects (finger ranges [id+2^i, id+2^(i+1)-1] partition (id, id-1],
// finger_table.h:177-188).
__device__ __forceinline__ int msb128(u128 d) {
    const uint64_t hi = (uint64_t)(d >> 64);
    const uint64_t lo = (uint64_t)d;
    return hi ? 127 - __clzll((long long)hi) : 63 - __clzll((long long)lo);
}

// Counter-based synthetic generator of SURVEY 8(d).
__host__ __device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t ctr) {
    uint64_t z = seed + (ctr + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ---------------------------------------------------------------------------
// Eytzinger (BFS) layout of the sorted ring.  Node k (1-based) of a heap-shaped
// tree with n nodes; tree height h = floor(log2 n).  The first `lds_levels`
// levels are staged in LDS by every search workgroup.
// ---------------------------------------------------------------------------
struct EytView {
    const cell128 *E;   // E[1..n]
    uint32_t n;
    int h;              // floor(log2 n)
};

// Number of nodes in the subtree rooted at j (depth dj), 0 if j > n.
__host__ __device__ __forceinline__ uint32_t eyt_subtree(uint64_t j, int dj, uint32_t n, int h) {
    if (j > n) return 0;
    const int t = h - dj;                    // levels below j down to level h
    const uint32_t full = (1u << t) - 1u;    // complete levels dj .. h-1
    const uint64_t first_last = j << t;      // leftmost level-h node under j
    uint64_t last = 0;
    if ((uint64_t)n >= first_last) {
        last = (uint64_t)n - first_last + 1;
        if (last > (1ull << t)) last = 1ull << t;
    }
    return full + (uint32_t)last;
}

#define CX_LDS_LEVELS 12                     // 4095 nodes x 16 B = 64 KiB of LDS
#define CX_LDS_NODES ((1u << CX_LDS_LEVELS) - 1u)

// Sorted index of succ(x) (first id >= x, wrapping to 0).  `lds` holds nodes
// 1..min(n, CX_LDS_NODES) at lds[k-1].  Tracks the count of ids < x along the
// descent: going right past node k passes its left subtree and k itself.
__device__ __forceinline__ uint32_t eyt_successor(const EytView &ev, const u128 *lds, u128 x) {
    uint64_t k = 1;
    uint32_t less = 0;
    int d = 0;
    const uint32_t n = ev.n;
    while (k <= n) {
        const u128 e = (k <= CX_LDS_NODES) ? lds[k - 1] : ld128(ev.E + k);
        const bool lt = e < x;
        if (lt) less += eyt_subtree(2 * k, d + 1, n, ev.h) + 1u;
        k = 2 * k + (lt ? 1 : 0);
        ++d;
    }
    return less == n ? 0u : less;
}

__device__ __forceinline__ void eyt_stage_lds(const EytView &ev, u128 *lds) {
    const uint32_t m = ev.n < CX_LDS_NODES ? ev.n : CX_LDS_NODES;
    for (uint32_t k = threadIdx.x; k < m; k += blockDim.x) lds[k] = ld128(ev.E + 1 + k);
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Bucket directory of the ring (uniform hash IDs): k = ceil(log2 n) top bits
// pick bucket b; entry b (16 B) = {lo, hi, frac}: [lo, hi) are the ring
// indices whose IDs fall in bucket b (lo = first index >= b << (128-k)), frac
// = the 64 ID bits of ring[lo] just below the bucket bits.  One gather answers
// an empty bucket, a key below the bucket's first ID, or a one-entry bucket;
// otherwise an exact binary search over the bucket's IDs finishes it.
// ---------------------------------------------------------------------------
struct SearchView {
    EytView ev;          // Eytzinger copy (always built)
    const uint4 *dir;    // [2^k] directory entries, or nullptr (use Eytzinger)
    int k;
    const cell128 *ring;
};

// Number of ring IDs < x (the unwrapped successor index, n if x is past the
// last ID).
__device__ __forceinline__ uint32_t dir_lower_bound(const SearchView &sv, u128 x) {
    const int k = sv.k;
    const uint4 e = sv.dir[(size_t)top_bits(x, k)];
    const uint32_t lo = e.x, hi = e.y;
    if (lo == hi) return hi;
    const uint64_t frac = ((uint64_t)e.w << 32) | e.z;
    const uint64_t xf = mid_bits(x, k);  // ID bits [64-k, 128-k)
    if (xf < frac) return lo;
    if (xf > frac && hi - lo == 1) return hi;
    uint32_t a = (xf > frac) ? lo + 1 : lo, z = hi;
    while (a < z) {
        const uint32_t m = a + (z - a) / 2;
        if (ld128(sv.ring + m) < x) a = m + 1;
        else z = m;
    }
    return a;
}

__device__ __forceinline__ uint32_t dir_successor(const SearchView &sv, u128 x) {
    const uint32_t n = sv.ev.n;
    const int k = sv.k;
    const uint4 e = sv.dir[(size_t)top_bits(x, k)];
    const uint32_t lo = e.x, hi = e.y;
    uint32_t ans;
    if (lo == hi) {
        ans = hi;
    } else {
        const uint64_t frac = ((uint64_t)e.w << 32) | e.z;
        const uint64_t xf = mid_bits(x, k);  // ID bits [64-k, 128-k)
        if (xf < frac) {
            ans = lo;
        } else if (xf > frac && hi - lo == 1) {
            ans = hi;
        } else {
            uint32_t a = (xf > frac) ? lo + 1 : lo, z = hi;
            while (a < z) {
                const uint32_t m = a + (z - a) / 2;
                if (ld128(sv.ring + m) < x) a = m + 1;
                else z = m;
            }
            ans = a;
        }
    }
    return ans == n ? 0u : ans;
}

// Compile-time choice of the successor search inside a kernel.
template <bool DIR>
struct Searcher;
template <>
struct Searcher<false> {
    static constexpr unsigned LDS = CX_LDS_NODES;
    __device__ static void stage(const SearchView &sv, u128 *lds) { eyt_stage_lds(sv.ev, lds); }
    __device__ static uint32_t find(const SearchView &sv, const u128 *lds, u128 x) {
        return eyt_successor(sv.ev, lds, x);
    }
};
template <>
struct Searcher<true> {
    static constexpr unsigned LDS = 1;
    __device__ static void stage(const SearchView &, u128 *) {}
    __device__ static uint32_t find(const SearchView &sv, const u128 *, u128 x) {
        return dir_successor(sv, x);
    }
};

// ---------------------------------------------------------------------------
// Host-side launch helpers.
// ---------------------------------------------------------------------------
static inline unsigned cx_grid(size_t work, unsigned block, unsigned cap = 8192) {
    size_t g = (work + block - 1) / block;
    if (g == 0) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}
