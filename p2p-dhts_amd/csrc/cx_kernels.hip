// cx_kernels.hip -- gfx950 kernels of the chordx engine and their launchers.
//
// Every kernel is HBM/latency bound integer work: no MFMA.  Layout
// in HBM: ring IDs as 16-B cells (AoS, one dwordx4 per ID), finger table as
// row-major uint32 [peer][128], Eytzinger copy of the ring for searches.
#include <atomic>
#include <initializer_list>
#include <cmath>
#include <type_traits>

#include "cx_kernels.hpp"

namespace cxk {

// ===========================================================================
// Device-wide exclusive scan of uint32 (radix offsets, compaction indices).
// ===========================================================================
constexpr int SCAN_BLOCK = 256;
constexpr int SCAN_ITEMS = 16;
constexpr int SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(v, off, 64);
        if (lane >= off) v += t;
    }
    return v;
}

// Block-wide exclusive scan of one value per thread; returns the block total
// through *total.  Block = SCAN_BLOCK threads (4 waves).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *total) {
    __shared__ uint32_t wsum[SCAN_BLOCK / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v, lane);
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < SCAN_BLOCK / 64; ++w) {
        wbase += (w < wave) ? wsum[w] : 0u;
        tot += wsum[w];
    }
    __syncthreads();
    *total = tot;
    return wbase + inc - v;
}

// In-place exclusive scan inside each SCAN_TILE tile; tile totals -> sums.
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_tiles(uint32_t *data, size_t n,
                                                           uint32_t *sums) {
    __shared__ uint32_t tile[SCAN_TILE + SCAN_TILE / 32];  // +1 pad per 32 words
    const size_t base = (size_t)blockIdx.x * SCAN_TILE;
    const int t = threadIdx.x;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const int li = j * SCAN_BLOCK + t;
        const size_t gi = base + li;
        tile[li + (li >> 5)] = gi < n ? data[gi] : 0u;
    }
    __syncthreads();
    // thread t owns elements [t*ITEMS, t*ITEMS + ITEMS)
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const int li = t * SCAN_ITEMS + j;
        run += tile[li + (li >> 5)];
    }
    uint32_t total;
    const uint32_t off = block_excl_scan(run, &total);
    run = off;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const int li = t * SCAN_ITEMS + j;
        const uint32_t v = tile[li + (li >> 5)];
        tile[li + (li >> 5)] = run;
        run += v;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const int li = j * SCAN_BLOCK + t;
        const size_t gi = base + li;
        if (gi < n) data[gi] = tile[li + (li >> 5)];
    }
    if (t == 0 && sums) sums[blockIdx.x] = total;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_add(uint32_t *data, size_t n,
                                                         const uint32_t *sums) {
    const size_t base = (size_t)blockIdx.x * SCAN_TILE;
    const uint32_t add = sums[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const size_t gi = base + j * SCAN_BLOCK + threadIdx.x;
        if (gi < n) data[gi] += add;
    }
}

size_t scan_workspace_words(size_t n) {
    size_t words = 0;
    while (n > (size_t)SCAN_TILE) {
        n = (n + SCAN_TILE - 1) / SCAN_TILE;
        words += n;
    }
    return words + 1;
}

hipError_t exclusive_scan(uint32_t *data, size_t n, uint32_t *ws, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const size_t tiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (tiles == 1) {
        k_scan_tiles<<<1, SCAN_BLOCK, 0, s>>>(data, n, nullptr);
        return hipGetLastError();
    }
    uint32_t *sums = ws;
    k_scan_tiles<<<(unsigned)tiles, SCAN_BLOCK, 0, s>>>(data, n, sums);
    hipError_t e = exclusive_scan(sums, tiles, ws + tiles, s);
    if (e != hipSuccess) return e;
    k_scan_add<<<(unsigned)tiles, SCAN_BLOCK, 0, s>>>(data, n, sums);
    return hipGetLastError();
}

// ===========================================================================
// LSD radix sort of (128-bit key, uint32 tag): 16 stable passes of 8 bits.
// Pass = histogram per 4096-element tile -> exclusive scan over [digit][tile]
// -> stable scatter (wave match via 8 ballots + cross-wave prefix in LDS).
// ===========================================================================
constexpr int RS_BLOCK = 256;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_BLOCK * RS_ITEMS;

__global__ __launch_bounds__(RS_BLOCK) void k_rs_hist(const cell128 *keys, size_t n, int shift,
                                                      uint32_t *hist, uint32_t ntiles) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * RS_TILE;
#pragma unroll 4
    for (int j = 0; j < RS_ITEMS; ++j) {
        const size_t i = base + j * RS_BLOCK + threadIdx.x;
        if (i < n) {
            const uint32_t d = (uint32_t)bits64(ld128(keys + i), shift) & 0xFFu;
            atomicAdd(&h[d], 1u);
        }
    }
    __syncthreads();
    hist[(size_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// One barrier per item (round 6): the per-wave digit counts and the digit
// bases are double-buffered by item parity -- item j zeroes its wave's row of
// wcnt[j & 1] (last read by item j - 2, before item j - 1's barrier) and
// writes the next bases into base[(j + 1) & 1] (last read by item j - 1,
// before item j's barrier) -- and the next item's key and tag are loaded
// while this one is ranked.  (Round 5: four barriers per item, no prefetch;
// 0.38 ms per 2^24-key pass.)
__global__ __launch_bounds__(RS_BLOCK) void k_rs_scatter(const cell128 *kin, const uint32_t *tin,
                                                         cell128 *kout, uint32_t *tout, size_t n,
                                                         int shift, const uint32_t *offs,
                                                         uint32_t ntiles) {
    __shared__ uint32_t base[2][256];
    __shared__ uint32_t wcnt[2][RS_BLOCK / 64][256];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    base[0][t] = offs[(size_t)t * ntiles + blockIdx.x];
    const size_t tile0 = (size_t)blockIdx.x * RS_TILE;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    u128 nkey = 0;
    uint32_t ntag = 0;
    if (tile0 + t < n) {
        nkey = ld128(kin + tile0 + t);
        ntag = tin[tile0 + t];
    }
    for (int j = 0; j < RS_ITEMS; ++j) {
        const int cur = j & 1;
        const size_t i = tile0 + (size_t)j * RS_BLOCK + t;
        const bool valid = i < n;
        const u128 key = nkey;
        const uint32_t tag = ntag;
        if (j + 1 < RS_ITEMS && i + RS_BLOCK < n) {  // the next item, in flight meanwhile
            nkey = ld128(kin + i + RS_BLOCK);
            ntag = tin[i + RS_BLOCK];
        }
        // shift < 0: the tag's byte (-1 - shift) / 8 (the fallback's tag passes)
        const uint32_t d = !valid ? 0u
                           : shift >= 0 ? (uint32_t)bits64(key, shift) & 0xFFu
                                        : (tag >> (-1 - shift)) & 0xFFu;
#pragma unroll
        for (int r = 0; r < 4; ++r) wcnt[cur][wave][lane + 64 * r] = 0;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt_mask);
        __builtin_amdgcn_wave_barrier();  // the row's zeroes before its leaders' counts
        if (valid && rank == 0) wcnt[cur][wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pre = 0;
            for (int w = 0; w < wave; ++w) pre += wcnt[cur][w][d];
            const uint32_t pos = base[cur][d] + pre + rank;
            st128(kout + pos, key);
            tout[pos] = tag;
        }
        uint32_t add = 0;
#pragma unroll
        for (int w = 0; w < RS_BLOCK / 64; ++w) add += wcnt[cur][w][t];
        base[cur ^ 1][t] = base[cur][t] + add;
    }
}

// Tag digits (the fallback's first four passes): the tag's byte `shift / 8`.
__global__ __launch_bounds__(RS_BLOCK) void k_rs_hist_tag(const uint32_t *tags, size_t n,
                                                          int shift, uint32_t *hist,
                                                          uint32_t ntiles) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * RS_TILE;
#pragma unroll 4
    for (int j = 0; j < RS_ITEMS; ++j) {
        const size_t i = base + j * RS_BLOCK + threadIdx.x;
        if (i < n) atomicAdd(&h[(tags[i] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    hist[(size_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// ---------------------------------------------------------------------------
// Ring sort, MSD first (round 6): the ring's IDs are hash outputs, so the top
// kb = ceil(log2 n) - 8 bits split n keys into 2^kb buckets of ~256 keys.
//   top passes  ceil(kb / 8) stable LSD passes over the top bytes (2 at
//               2^24 keys): the keys grouped by bucket, in input order;
//   bounds      each bucket's end from the sorted top bits (one pass);
//   bucket      one block per bucket: its keys + tags in LDS, each element's
//               rank = #elements ordered before it by (key, tag), the element
//               written at its rank.
// 2 + 2 passes over the keys instead of the LSD sort's 16 x (histogram +
// scatter).  (key, tag) order is the LSD sort's stable order: every caller
// hands in tags ascending in input order (iota, or survivors' old indices
// then join tags).  A bucket above MS_CAP keys (clustered IDs) sets the
// overflow word and the caller falls back to the LSD sort with the tag as
// its lowest digits.  (A first version bucketed with one global atomic per
// key for the count and one for the slot: 5.0 ms at 2^24 -- device-scope
// atomics on 2^16 counters -- against 7.6 ms for the 16-pass LSD sort.)
// ---------------------------------------------------------------------------
constexpr uint32_t MS_CAP = 2048;
constexpr int MS_BLOCK = 256;

static int ms_bits(size_t n) {
    int lg = 0;
    while (((size_t)1 << lg) < n) ++lg;
    const int kb = lg - 8;
    return kb < 0 ? 0 : (kb > 24 ? 24 : kb);
}

__device__ __forceinline__ uint32_t ms_bucket(const cell128 *k, size_t i, int kb) {
    return kb ? (uint32_t)(k[i].hi >> (64 - kb)) : 0u;
}

// keys grouped by bucket (ascending top kb bits): end[b] = one past bucket b's
// last key, for every b in [0, nb) (empty buckets included).
__global__ void k_ms_bounds(const cell128 *keys, size_t n, int kb, uint32_t nb, uint32_t *end) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t b = ms_bucket(keys, i, kb);
        if (i == 0)
            for (uint32_t c = 0; c < b; ++c) end[c] = 0;
        const uint32_t nxt = i + 1 < n ? ms_bucket(keys, i + 1, kb) : nb;
        for (uint32_t c = b; c < nxt; ++c) end[c] = (uint32_t)(i + 1);
    }
}


// Block b sorts bucket b = [end[b-1], end[b]) of (kin, tin) into (kout, tout).
// An element's rank is counted on a 32-bit prefix first -- the ID bits just
// below the bucket's shared top kb bits, pre = bits [96 - kb, 128 - kb) --
// in a branch-free pass over the bucket's prefixes in LDS (4 B each, eight per
// step, every lane reading the same words: broadcasts); the few elements
// whose prefix is not unique in the bucket (a 2^-32 event per pair on hashed
// IDs; every pair of a clustered bucket) settle the tie by (key, tag) in a
// second pass over the equal prefixes, reading those keys from global memory.
// Only the prefixes live in LDS (8 KiB): 8 blocks per CU.  (Counting on the
// full (key, tag) per element took 3.5 ms at 2^24 keys; prefixes with the
// keys also in LDS, 3 blocks per CU, 0.94 ms.)
__global__ __launch_bounds__(MS_BLOCK) void k_ms_bucket(const cell128 *kin, const uint32_t *tin,
                                                        const uint32_t *end, uint32_t nb, int kb,
                                                        cell128 *kout, uint32_t *tout,
                                                        uint32_t *overflow) {
    __shared__ alignas(16) uint32_t sp[MS_CAP];  // read as uint4
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        const uint32_t lo = b ? end[b - 1] : 0u, hi = end[b];
        const uint32_t m = hi - lo;
        if (m > MS_CAP) {
            if (threadIdx.x == 0) atomicOr(overflow, 1u);
            continue;
        }
        if (m <= 1) {
            if (m == 1 && threadIdx.x == 0) {
                st128(kout + lo, ld128(kin + lo));
                tout[lo] = tin[lo];
            }
            continue;
        }
        for (uint32_t j = threadIdx.x; j < m; j += MS_BLOCK)
            sp[j] = (uint32_t)bits64(ld128(kin + lo + j), 96 - kb);
        for (uint32_t j = m + threadIdx.x; j < ((m + 7) & ~7u); j += MS_BLOCK)
            sp[j] = 0xFFFFFFFFu;  // pad to a multiple of 8: never "less", counted as equal
        __syncthreads();
        const uint32_t m8 = (m + 7) & ~7u;
        for (uint32_t j = threadIdx.x; j < m; j += MS_BLOCK) {
            const u128 kj = ld128(kin + lo + j);
            const uint32_t tj = tin[lo + j];
            const uint32_t pj = sp[j];
            uint32_t rank = 0, eq = 0;
            for (uint32_t x = 0; x < m8; x += 8) {
                const uint4 p = *reinterpret_cast<const uint4 *>(sp + x);
                const uint4 r = *reinterpret_cast<const uint4 *>(sp + x + 4);
                rank += (p.x < pj) + (p.y < pj) + (p.z < pj) + (p.w < pj) + (r.x < pj) +
                        (r.y < pj) + (r.z < pj) + (r.w < pj);
                eq += (p.x == pj) + (p.y == pj) + (p.z == pj) + (p.w == pj) + (r.x == pj) +
                      (r.y == pj) + (r.z == pj) + (r.w == pj);
            }
            // the padding words (0xFFFFFFFF) count as equal when pj is all ones
            if (eq > 1 + (pj == 0xFFFFFFFFu ? m8 - m : 0u)) {  // ties on the prefix: exact order
                for (uint32_t x = 0; x < m; ++x)
                    if (x != j && sp[x] == pj) {
                        const u128 kx = ld128(kin + lo + x);
                        rank += kx < kj || (kx == kj && tin[lo + x] < tj);
                    }
            }
            st128(kout + lo + rank, kj);
            tout[lo + rank] = tj;
        }
        __syncthreads();  // the LDS is refilled by the next bucket
    }
}

size_t sort_workspace_words(size_t n) {
    const size_t ntiles = (n + RS_TILE - 1) / RS_TILE;
    const size_t lsd = 256 * ntiles + scan_workspace_words(256 * ntiles);
    // + the MSD path's bucket ends (after the passes' words) + its overflow word
    return lsd + ((size_t)1 << ms_bits(n)) + 4;
}

// LSD passes over (k0, t0) <-> (k1, t1): `tag_passes` byte passes of the tag
// first (then the order of equal keys is the tags' order, whatever the input
// order), then the 16 key bytes; an even pass count leaves the result in
// (k0, t0).
static hipError_t lsd_sort(cell128 *k0, uint32_t *t0, cell128 *k1, uint32_t *t1, size_t n,
                           uint32_t *ws, int tag_passes, hipStream_t s) {
    const uint32_t ntiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    uint32_t *hist = ws;
    uint32_t *scan_ws = ws + (size_t)256 * ntiles;
    for (int pass = 0; pass < 16 + tag_passes; ++pass) {
        cell128 *ki = (pass & 1) ? k1 : k0, *ko = (pass & 1) ? k0 : k1;
        uint32_t *ti = (pass & 1) ? t1 : t0, *to = (pass & 1) ? t0 : t1;
        const bool tagd = pass < tag_passes;
        const int shift = tagd ? 8 * pass : 8 * (pass - tag_passes);
        if (tagd)
            k_rs_hist_tag<<<ntiles, RS_BLOCK, 0, s>>>(ti, n, shift, hist, ntiles);
        else
            k_rs_hist<<<ntiles, RS_BLOCK, 0, s>>>(ki, n, shift, hist, ntiles);
        hipError_t e = exclusive_scan(hist, (size_t)256 * ntiles, scan_ws, s);
        if (e != hipSuccess) return e;
        k_rs_scatter<<<ntiles, RS_BLOCK, 0, s>>>(ki, ti, ko, to, n, tagd ? -1 - shift : shift,
                                                 hist, ntiles);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t radix_sort_lsd(cell128 *k0, uint32_t *t0, cell128 *k1, uint32_t *t1, size_t n,
                          uint32_t *ws, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    return lsd_sort(k0, t0, k1, t1, n, ws, 0, s);
}

// Sorts (keys, tags) by (key, tag) -- the stable key order for tags ascending
// in input order -- into (k0, t0); (k1, t1) is scratch.  MSD bucket path
// first; one host synchronisation reads its overflow word; a clustered input
// then takes the LSD sort (4 tag + 16 key passes) over the partly sorted copy.
hipError_t radix_sort(cell128 *k0, uint32_t *t0, cell128 *k1, uint32_t *t1, size_t n,
                      uint32_t *ws, hipStream_t s) {
    if (n <= 1) return hipSuccess;
    if (n >= (1ull << 31)) return hipErrorInvalidValue;
    const int kb = ms_bits(n);
    const size_t nb = (size_t)1 << kb;
    const int tp = (kb + 7) / 8;  // top-byte passes
    const size_t wsw = sort_workspace_words(n);
    uint32_t *ovf = ws + wsw - 1;
    uint32_t *end = ws + wsw - 2 - nb;  // beyond the passes' histogram and scan words
    hipError_t e = hipMemsetAsync(ovf, 0, sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    const uint32_t ntiles = (uint32_t)((n + RS_TILE - 1) / RS_TILE);
    uint32_t *hist = ws, *scan_ws = ws + (size_t)256 * ntiles;
    cell128 *ka = k0, *kx = k1;
    uint32_t *ta = t0, *tx = t1;
    for (int p = 0; p < tp; ++p) {  // bytes 16 - tp ... 15, lowest first
        const int shift = 8 * (16 - tp + p);
        k_rs_hist<<<ntiles, RS_BLOCK, 0, s>>>(ka, n, shift, hist, ntiles);
        if ((e = exclusive_scan(hist, (size_t)256 * ntiles, scan_ws, s)) != hipSuccess) return e;
        k_rs_scatter<<<ntiles, RS_BLOCK, 0, s>>>(ka, ta, kx, tx, n, shift, hist, ntiles);
        std::swap(ka, kx);
        std::swap(ta, tx);
    }
    // (ka, ta): grouped by bucket; sorted into (kx, tx)
    k_ms_bounds<<<cx_grid(n, 256), 256, 0, s>>>(ka, n, kb, (uint32_t)nb, end);
    k_ms_bucket<<<(unsigned)(nb < 65535 * 8 ? nb : 65535 * 8), MS_BLOCK, 0, s>>>(
        ka, ta, end, (uint32_t)nb, kb, kx, tx, ovf);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    uint32_t o = 0;
    if ((e = hipMemcpyAsync(&o, ovf, sizeof(o), hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if (o) {
        // clustered: (ka, ta) holds every key; sort it by (key, tag): 20
        // passes leave the result in (ka, ta)
        e = lsd_sort(ka, ta, kx, tx, n, ws, 4, s);
        if (e != hipSuccess) return e;
        std::swap(ka, kx);
        std::swap(ta, tx);
    }
    if (kx != k0) {  // the result is in (kx, tx)
        if ((e = hipMemcpyAsync(k0, kx, n * sizeof(cell128), hipMemcpyDeviceToDevice, s)) != hipSuccess)
            return e;
        e = hipMemcpyAsync(t0, tx, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, s);
    }
    return e;
}

// *bad = 0 if (keys, tags) ascend by (key, tag), else nonzero (test / A/B).
__global__ void k_check_sorted(const cell128 *k, const uint32_t *t, size_t n, uint32_t *bad) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i + 1 < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const u128 a = ld128(k + i), b = ld128(k + i + 1);
        if (b < a || (a == b && t[i + 1] < t[i])) atomicOr(bad, 1u);
    }
}

hipError_t check_sorted(const cell128 *k, const uint32_t *t, size_t n, uint32_t *bad,
                        hipStream_t s) {
    hipError_t e = hipMemsetAsync(bad, 0, sizeof(uint32_t), s);
    if (e != hipSuccess || n < 2) return e;
    k_check_sorted<<<cx_grid(n, 256), 256, 0, s>>>(k, t, n, bad);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Bucket sort of a small batch of uniformly distributed keys (a churn's joins:
// 2^17 keys at 1 % of 2^24 peers).  The radix sort's 16 passes x 4 launches
// cost ~1 ms of launch-bound time there; this takes 2^kb buckets by the top kb
// bits (about one key per bucket), counts, scans, scatters, and sorts each
// bucket in place (one lane per bucket, insertion sort).  A bucket above
// BS_MAX keys (clustered input) sets *overflow and is left unsorted: the
// caller then sorts with radix_sort.  Not stable (equal keys are equal values).
// ---------------------------------------------------------------------------
constexpr uint32_t BS_MAX = 32;

__global__ void k_bs_count(const cell128 *keys, size_t n, int kb, uint32_t *cnt) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        atomicAdd(cnt + (kb ? keys[i].hi >> (64 - kb) : 0), 1u);
}

// cnt holds the buckets' exclusive offsets; afterwards cnt[b] = end of bucket b
__global__ void k_bs_scatter(const cell128 *keys, size_t n, int kb, uint32_t *cnt, cell128 *out) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const cell128 k = keys[i];
        const uint32_t pos = atomicAdd(cnt + (kb ? k.hi >> (64 - kb) : 0), 1u);
        out[pos] = k;
    }
}

__global__ void k_bs_sort(cell128 *v, const uint32_t *end, uint32_t nb, uint32_t *overflow) {
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nb; b += gridDim.x * blockDim.x) {
        const uint32_t lo = b ? end[b - 1] : 0u, hi = end[b];
        if (hi - lo > BS_MAX) {
            atomicOr(overflow, 1u);
            continue;
        }
        for (uint32_t x = lo + 1; x < hi; ++x) {
            const cell128 k = v[x];
            const u128 kk = ((u128)k.hi << 64) | k.lo;
            uint32_t y = x;
            while (y > lo) {
                const cell128 w = v[y - 1];
                if ((((u128)w.hi << 64) | w.lo) <= kk) break;
                v[y] = w;
                --y;
            }
            v[y] = k;
        }
    }
}

size_t bucket_sort_workspace_words(size_t n) {
    int kb = 0;
    while (((size_t)1 << kb) < n) ++kb;
    const size_t nb = (size_t)1 << kb;
    return nb + 1 + scan_workspace_words(nb + 1);
}

// keys (n) -> out (n) in ascending order unless *overflow (device word, zeroed
// here) comes back nonzero.
hipError_t bucket_sort(const cell128 *keys, size_t n, cell128 *out, uint32_t *ws,
                       uint32_t *overflow, hipStream_t s) {
    hipError_t e = hipMemsetAsync(overflow, 0, sizeof(uint32_t), s);
    if (e != hipSuccess || n == 0) return e;
    int kb = 0;
    while (((size_t)1 << kb) < n) ++kb;
    if (kb > 30) return hipErrorInvalidValue;
    const size_t nb = (size_t)1 << kb;
    uint32_t *cnt = ws, *scan_ws = ws + nb + 1;
    if ((e = hipMemsetAsync(cnt, 0, (nb + 1) * sizeof(uint32_t), s)) != hipSuccess) return e;
    k_bs_count<<<cx_grid(n, 256), 256, 0, s>>>(keys, n, kb, cnt);
    if ((e = exclusive_scan(cnt, nb + 1, scan_ws, s)) != hipSuccess) return e;
    k_bs_scatter<<<cx_grid(n, 256), 256, 0, s>>>(keys, n, kb, cnt, out);
    k_bs_sort<<<cx_grid(nb, 256), 256, 0, s>>>(out, cnt, (uint32_t)nb, overflow);
    return hipGetLastError();
}

// ===========================================================================
// Dedupe / compaction (equal IDs rejected, remote_peer_list.cpp:56-58).
// ===========================================================================
__global__ void k_flag_unique(const cell128 *keys, size_t n, uint32_t *flag) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        flag[i] = (i == 0 || ld128(keys + i) != ld128(keys + i - 1)) ? 1u : 0u;
}

// pos = exclusive scan of flags.  Keeps flagged keys; a kept tag < CX_TAG_JOIN
// (an old peer index) gets old_to_new[tag] = new position.
__global__ void k_compact_unique(const cell128 *keys, const uint32_t *tags, size_t n,
                                 const uint32_t *pos, cell128 *out, uint32_t *old_to_new) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const bool keep = (i == 0 || ld128(keys + i) != ld128(keys + i - 1));
        if (!keep) continue;
        const uint32_t p = pos[i];
        st128(out + p, ld128(keys + i));
        if (old_to_new && tags[i] < CX_TAG_JOIN) old_to_new[tags[i]] = p;
    }
}

__global__ void k_iota(uint32_t *t, size_t n, uint32_t base) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        t[i] = base + (uint32_t)i;
}

__global__ void k_fill_u32(uint32_t *t, size_t n, uint32_t v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        t[i] = v;
}

__global__ void k_count_last(const uint32_t *pos, const cell128 *keys, size_t n, uint32_t *out) {
    // unique count = pos[n-1] + flag[n-1]
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const bool keep = (n == 1) || ld128(keys + n - 1) != ld128(keys + n - 2);
        *out = pos[n - 1] + (keep ? 1u : 0u);
    }
}

hipError_t unique_sorted(const cell128 *keys, const uint32_t *tags, size_t n, uint32_t *pos,
                         uint32_t *scan_ws, cell128 *out, uint32_t *old_to_new,
                         uint32_t *d_count, hipStream_t s) {
    const unsigned g = cx_grid(n, 256);
    k_flag_unique<<<g, 256, 0, s>>>(keys, n, pos);
    hipError_t e = exclusive_scan(pos, n, scan_ws, s);
    if (e != hipSuccess) return e;
    k_count_last<<<1, 64, 0, s>>>(pos, keys, n, d_count);
    k_compact_unique<<<g, 256, 0, s>>>(keys, tags, n, pos, out, old_to_new);
    return hipGetLastError();
}

// Survivor compaction for churn: keep[p] = !gone[p].
__global__ void k_keep_flags(const uint8_t *gone, size_t n, uint32_t *flag) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        flag[i] = gone[i] ? 0u : 1u;
}
__global__ void k_compact_survivors(const cell128 *ring, const uint8_t *gone, size_t n,
                                    const uint32_t *pos, cell128 *out_keys, uint32_t *out_tags) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        if (gone[i]) continue;
        const uint32_t p = pos[i];
        st128(out_keys + p, ld128(ring + i));
        out_tags[p] = (uint32_t)i;
    }
}
__global__ void k_count_survivors(const uint32_t *pos, const uint8_t *gone, size_t n,
                                  uint32_t *out) {
    if (blockIdx.x == 0 && threadIdx.x == 0) *out = pos[n - 1] + (gone[n - 1] ? 0u : 1u);
}

hipError_t compact_survivors(const cell128 *ring, const uint8_t *gone, size_t n, uint32_t *pos,
                             uint32_t *scan_ws, cell128 *out_keys, uint32_t *out_tags,
                             uint32_t *d_count, hipStream_t s) {
    const unsigned g = cx_grid(n, 256);
    k_keep_flags<<<g, 256, 0, s>>>(gone, n, pos);
    hipError_t e = exclusive_scan(pos, n, scan_ws, s);
    if (e != hipSuccess) return e;
    k_count_survivors<<<1, 64, 0, s>>>(pos, gone, n, d_count);
    k_compact_survivors<<<g, 256, 0, s>>>(ring, gone, n, pos, out_keys, out_tags);
    return hipGetLastError();
}

// ===========================================================================
// Eytzinger build: E[k] = sorted[inorder rank of node k].
// ===========================================================================
__device__ __forceinline__ uint32_t eyt_rank(uint64_t k, uint32_t n, int h) {
    const int depth = 63 - __clzll((long long)k);
    uint64_t node = 1;
    uint32_t r = 0;
    for (int b = depth - 1, d = 0; b >= 0; --b, ++d) {
        if ((k >> b) & 1ull) {
            r += eyt_subtree(2 * node, d + 1, n, h) + 1u;
            node = 2 * node + 1;
        } else {
            node = 2 * node;
        }
    }
    return r + eyt_subtree(2 * k, depth + 1, n, h);
}

__global__ void k_eyt_build(const cell128 *sorted, uint32_t n, int h, cell128 *E) {
    for (size_t k = 1 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; k <= n;
         k += (size_t)gridDim.x * blockDim.x)
        st128(E + k, ld128(sorted + eyt_rank(k, n, h)));
}

hipError_t eyt_build(const cell128 *sorted, size_t n, cell128 *E, hipStream_t s) {
    const int h = 63 - __builtin_clzll((unsigned long long)n);
    k_eyt_build<<<cx_grid(n, 256), 256, 0, s>>>(sorted, (uint32_t)n, h, E);
    return hipGetLastError();
}

// ===========================================================================
// a5/a7: exact successor.  One lane per query; top CX_LDS_LEVELS of the
// Eytzinger tree in LDS (64 KiB), the rest gathered from HBM/L2.
// ===========================================================================
constexpr int SUCC_BLOCK = 1024;

// PRED: the owner's predecessor instead (converged GetPredecessor).
template <bool DIR, bool PRED = false>
__global__ __launch_bounds__(SUCC_BLOCK) void k_successor(SearchView sv, const cell128 *keys,
                                                          size_t q, uint32_t *owner) {
    __shared__ u128 lds[Searcher<DIR>::LDS];
    Searcher<DIR>::stage(sv, lds);
    const uint32_t n = sv.ev.n;
    // keys and owners stream (non-temporal): the caches keep directory and
    // ring lines instead (2^24 ring, 2^25 keys: 0.747 vs 0.765 ms,
    // profiles/r06/exact_succ/nt_ab/)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < q;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t s = Searcher<DIR>::find(sv, lds, ld128_nt(keys + i));
        __builtin_nontemporal_store(PRED ? (s == 0 ? n - 1 : s - 1) : s, owner + i);
    }
}

hipError_t successor(const SearchView &sv, const cell128 *keys, size_t q, uint32_t *owner,
                     hipStream_t s) {
    if (q == 0) return hipSuccess;
    if (sv.dir)
        k_successor<true><<<cx_grid(q, SUCC_BLOCK, 2048), SUCC_BLOCK, 0, s>>>(sv, keys, q, owner);
    else
        k_successor<false><<<cx_grid(q, SUCC_BLOCK, 512), SUCC_BLOCK, 0, s>>>(sv, keys, q, owner);
    return hipGetLastError();
}

hipError_t predecessor(const SearchView &sv, const cell128 *keys, size_t q, uint32_t *pred,
                       hipStream_t s) {
    if (q == 0) return hipSuccess;
    if (sv.dir)
        k_successor<true, true><<<cx_grid(q, SUCC_BLOCK, 2048), SUCC_BLOCK, 0, s>>>(sv, keys, q,
                                                                                    pred);
    else
        k_successor<false, true><<<cx_grid(q, SUCC_BLOCK, 512), SUCC_BLOCK, 0, s>>>(sv, keys, q,
                                                                                    pred);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Rings that fit LDS (a7 / GetPredecessor, search variants 1 (automatic) and
// 4): one table per ring, staged whole into every block -- the bucket
// offsets off[t] = first index whose top b ID bits are >= t (t = 0 .. 2^b;
// as int16 deviations from (t n) >> b when they fit, D16, which leaves room
// for one more bucket bit), then the 16-bit slices s(p) = ID bits
// [128 - b - 16, 128 - b) of every peer, each part padded to 16 B.  Within bucket t the slices are sorted, so
// a key's successor is the lower bound of its own slice in [off[t],
// off[t + 1]) -- exact unless that peer shares the key's top b + 16 bits
// (probability n / 2^(b + 16), 2^-12 at C2), which reads the full IDs.  One
// key line and LDS instead of a random directory line (and sometimes a ring
// line) per key: the directory search of a 2^20-key batch is L2-request-bound
// (profiles/r06/c2_pmc/).
// ---------------------------------------------------------------------------
__global__ void k_slice_tab_build(const cell128 *ring, uint32_t n, int b, uint32_t *off,
                                  uint16_t *sl) {
    const uint32_t nb = (1u << b) + 1u;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < (size_t)n + nb;
         i += (size_t)gridDim.x * blockDim.x) {
        if (i < n) {
            sl[i] = (uint16_t)(top_bits(ld128(ring + i), b + 16) & 0xFFFFu);
        } else {  // off[t]: lower bound of t over the top b bits
            const uint64_t t = i - n;
            uint32_t a = 0, z = n;
            while (a < z) {
                const uint32_t m = a + (z - a) / 2;
                if (top_bits(ld128(ring + m), b) < t) a = m + 1;
                else z = m;
            }
            off[t] = a;
        }
    }
}

// dev16: the offsets as int16 deviations from (t n) >> b (uniform rings: half
// the bytes, so one more bucket bit fits LDS)
size_t slice_tab_bytes(size_t n, int b, bool dev16) {
    const size_t nb = ((size_t)1 << b) + 1;
    // whole 1-KiB runs (one LDS-DMA instruction per wave moves 1 KiB)
    return ((nb * (dev16 ? 2 : 4) + 15) / 16 * 16 + (n * 2 + 15) / 16 * 16 + 1023) / 1024 * 1024;
}

hipError_t slice_tab_build(const cell128 *ring, size_t n, int b, void *tab, hipStream_t s) {
    const size_t nb = ((size_t)1 << b) + 1;
    uint32_t *off = reinterpret_cast<uint32_t *>(tab);
    uint16_t *sl = reinterpret_cast<uint16_t *>(reinterpret_cast<char *>(tab) + (nb * 4 + 15) / 16 * 16);
    hipError_t e = hipMemsetAsync(tab, 0, slice_tab_bytes(n, b), s);  // the padding too
    if (e != hipSuccess) return e;
    k_slice_tab_build<<<cx_grid(n + nb, 256), 256, 0, s>>>(ring, (uint32_t)n, b, off, sl);
    return hipGetLastError();
}

constexpr int SL_BLOCK = 1024;
constexpr int SL_KEYS = 4;  // keys per lane per trip, their searches interleaved

// steps: binary-search rounds that cover the largest bucket (ceil(log2(max + 1))).
template <bool PRED, bool D16>
__global__ __launch_bounds__(SL_BLOCK) void k_successor_lds(const uint4 *tab, uint32_t tab_v4,
                                                            int b, int steps, uint32_t n,
                                                            const cell128 *ring,
                                                            const cell128 *keys, size_t q,
                                                            uint32_t *out) {
    extern __shared__ uint4 lds4[];
    const uint32_t *loff = reinterpret_cast<const uint32_t *>(lds4);
    const int16_t *ldev = reinterpret_cast<const int16_t *>(lds4);
    const uint16_t *lsl = reinterpret_cast<const uint16_t *>(
        reinterpret_cast<const char *>(lds4) +
        ((((size_t)1 << b) + 1) * (D16 ? 2 : 4) + 15) / 16 * 16);
    const size_t per = (size_t)SL_BLOCK * SL_KEYS;
    size_t c0 = blockIdx.x * per;
    // this block's first keys are in flight while the table lands in LDS
    u128 x[SL_KEYS];
#pragma unroll
    for (int k = 0; k < SL_KEYS; ++k) {
        const size_t i = c0 + (size_t)k * SL_BLOCK + threadIdx.x;
        x[k] = i < q ? ld128(keys + i) : (u128)0;
    }
    // every 16-B piece of the table straight into LDS (LDS-DMA, no VGPRs),
    // all issued before one wait: lane j of wave w moves piece it * SL_BLOCK +
    // w * 64 + j to the same LDS offset (tab_v4: a multiple of 64 pieces)
    const uint32_t wbase = threadIdx.x & ~63u;
#pragma unroll
    for (uint32_t it = 0; it < (uint32_t)((SLICE_TAB_MAX / 16 + SL_BLOCK - 1) / SL_BLOCK); ++it) {
        const uint32_t v0 = it * SL_BLOCK + wbase;  // wave-uniform
        if (v0 < tab_v4) {
            const uint32_t v = v0 + (threadIdx.x & 63u);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void *)(tab + v),
                (__attribute__((address_space(3))) void *)(lds4 + v0), 16, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (; c0 < q; c0 += (size_t)gridDim.x * per) {
        uint32_t a[SL_KEYS], z[SL_KEYS], e[SL_KEYS], xs[SL_KEYS];
#pragma unroll
        for (int k = 0; k < SL_KEYS; ++k) {
            const uint32_t t = (uint32_t)top_bits(x[k], b);
            if (D16) {
                a[k] = (uint32_t)(((uint64_t)t * n >> b) + ldev[t]);
                z[k] = e[k] = (uint32_t)(((uint64_t)(t + 1) * n >> b) + ldev[t + 1]);
            } else {
                a[k] = loff[t];
                z[k] = e[k] = loff[t + 1];
            }
            xs[k] = (uint32_t)(top_bits(x[k], b + 16) & 0xFFFFu);
        }
        for (int it = 0; it < steps; ++it) {  // every lane the same rounds
#pragma unroll
            for (int k = 0; k < SL_KEYS; ++k) {
                const uint32_t m = (a[k] + z[k]) >> 1;
                const bool go = a[k] < z[k];
                const uint32_t sv = lsl[go ? m : 0];
                a[k] = go && sv < xs[k] ? m + 1 : a[k];
                z[k] = go && !(sv < xs[k]) ? m : z[k];
            }
        }
        u128 xn[SL_KEYS];
        const size_t c1 = c0 + (size_t)gridDim.x * per;
#pragma unroll
        for (int k = 0; k < SL_KEYS; ++k) {
            // peers sharing the key's top b + 16 bits (rare): the first one's
            // ID decides unless it is below the key and the next peer shares
            // them too; then the run of equal slices and the IDs in it by
            // binary search (clustered rings put whole buckets in one run)
            if (a[k] < e[k] && lsl[a[k]] == xs[k] &&
                ld128(ring + a[k]) < x[k] && ++a[k] < e[k] && lsl[a[k]] == xs[k]) {
                uint32_t u = a[k] + 1, w = e[k];
                while (u < w) {
                    const uint32_t m = (u + w) >> 1;
                    if (lsl[m] <= xs[k]) u = m + 1;
                    else w = m;
                }
                uint32_t lo = a[k];
                while (lo < u) {
                    const uint32_t m = (lo + u) >> 1;
                    if (ld128(ring + m) < x[k]) lo = m + 1;
                    else u = m;
                }
                a[k] = lo;
            }
            const size_t i = c0 + (size_t)k * SL_BLOCK + threadIdx.x;
            const size_t i1 = c1 + (size_t)k * SL_BLOCK + threadIdx.x;
            xn[k] = i1 < q ? ld128(keys + i1) : (u128)0;  // the next trip's keys
            if (i < q) {
                const uint32_t s = a[k] == n ? 0u : a[k];
                out[i] = PRED ? (s == 0 ? n - 1 : s - 1) : s;
            }
        }
#pragma unroll
        for (int k = 0; k < SL_KEYS; ++k) x[k] = xn[k];
    }
}

hipError_t successor_lds(const void *tab, int b, bool dev16, int steps, const cell128 *ring,
                         size_t n, const cell128 *keys, size_t q, uint32_t *out, bool pred,
                         hipStream_t s) {
    if (q == 0) return hipSuccess;
    const size_t bytes = slice_tab_bytes(n, b, dev16);
    if (bytes > SLICE_TAB_MAX || n == 0 || n > 0xFFFFFFFFull || b < 1 || b > 14 || steps < 0)
        return hipErrorInvalidValue;
    int dev = 0;
    (void)hipGetDevice(&dev);
    auto kern = pred ? (dev16 ? k_successor_lds<true, true> : k_successor_lds<true, false>)
                     : (dev16 ? k_successor_lds<false, true> : k_successor_lds<false, false>);
    static const bool lds_ok = [] {  // dynamic LDS above 64 KiB, once per kernel
        const int lim = (int)SLICE_TAB_MAX;
        bool ok = true;
        for (const void *k : {reinterpret_cast<const void *>(k_successor_lds<false, false>),
                              reinterpret_cast<const void *>(k_successor_lds<true, false>),
                              reinterpret_cast<const void *>(k_successor_lds<false, true>),
                              reinterpret_cast<const void *>(k_successor_lds<true, true>)})
            ok = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lim) ==
                     hipSuccess && ok;
        return ok;
    }();
    (void)lds_ok;  // a runtime without the attribute takes the launch as is
    // resident blocks for this table size, cached (the device and occupancy
    // queries cost host time on every ~8-us launch): key = bytes | device | pred
    static std::atomic<uint64_t> cached{0};
    const uint64_t key = ((uint64_t)bytes << 7) | ((uint64_t)(dev & 31) << 2) |
                         (dev16 ? 2u : 0u) | (pred ? 1u : 0u);
    const uint64_t c = cached.load(std::memory_order_relaxed);
    uint64_t resident = c >> 25 == 0 ? 0 : c & ((1ull << 25) - 1);
    if (c >> 25 != key || resident == 0) {
        int cus = 256, per_cu = 1;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, SL_BLOCK, bytes) !=
                hipSuccess || per_cu < 1)
            per_cu = 1;
        resident = (uint64_t)cus * per_cu;
        cached.store((key << 25) | resident, std::memory_order_relaxed);
    }
    // one resident round of blocks (each stages the table once)
    size_t g = (q + (size_t)SL_BLOCK * SL_KEYS - 1) / ((size_t)SL_BLOCK * SL_KEYS);
    if (g > resident) g = resident;
    kern<<<(unsigned)g, SL_BLOCK, bytes, s>>>(reinterpret_cast<const uint4 *>(tab),
                                                (uint32_t)(bytes / 16), b, steps, (uint32_t)n,
                                                ring, keys, q, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Search variant 2: wave-cooperative 16-ary search (static S+-tree over the
// sorted ring).  Level 0 is the ring; level l >= 1 holds every 16^l-th ID,
// S_l[j] = ring[j * 16^l], so block c of level l (16 consecutive entries) is
// the 16 children separators under entry c of level l+1 and S_l[16c] =
// S_{l+1}[c].  Sixteen lanes search one query: lane i loads entry 16c + i
// (one coalesced 256-B block per query and level), compares it with the key
// in 128 bits, and the wave's ballot, cut to the group's 16 bits and counted
// (a sorted block gives a prefix mask, popcount = its length), names the child:
// c <- 16c + cnt - 1 (cnt >= 1 below the top: the block's first entry is the
// parent separator, < key).  At level 0 the count is #{ids < key} = the
// successor index.  Four queries per wave instruction, U rounds interleaved
// so U loads per lane are in flight per level.  Levels 1.. take n/15 IDs: at
// 2^24 level 1 is 16 MiB (MALL-resident), levels 2-5 1 MiB and less (L2);
// level 0 is the ring.
// ---------------------------------------------------------------------------
__global__ void k_stree_level(const cell128 *ring, uint32_t sz, int shift, cell128 *out) {
    for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j < sz;
         j += (size_t)gridDim.x * blockDim.x)
        out[j] = ring[j << shift];
}

constexpr uint32_t ST_LDS = 4384;  // cells of staged top levels: 70 KB, 2 blocks of 1024 per CU
constexpr int ST_BLOCK = 1024;

STreeView stree_plan(const cell128 *ring, size_t n, cell128 *buf) {
    STreeView v{};
    v.lv[0] = ring;
    v.sz[0] = (uint32_t)n;
    int l = 0;
    size_t off = 0;
    while (v.sz[l] > 16 && l + 1 < CX_STREE_MAX) {
        v.sz[l + 1] = (v.sz[l] + 15) / 16;
        v.lv[l + 1] = buf ? buf + off : nullptr;
        off += v.sz[l + 1];
        ++l;
    }
    v.top = l;
    v.words = off;
    // stage the top levels in LDS while they fit (16 + 256 + 4096 cells at 2^24)
    uint32_t used = 0;
    v.lds_from = v.top + 1;
    for (int k = v.top; k >= 1 && used + v.sz[k] <= ST_LDS; --k) {
        v.lds_off[k] = used;
        used += v.sz[k];
        v.lds_from = k;
    }
    return v;
}

hipError_t stree_build(const STreeView &v, hipStream_t s) {
    for (int l = 1; l <= v.top; ++l) {
        k_stree_level<<<cx_grid(v.sz[l], 256), 256, 0, s>>>(v.lv[0], v.sz[l], 4 * l,
                                                            const_cast<cell128 *>(v.lv[l]));
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <bool PRED, int U>
__global__ __launch_bounds__(ST_BLOCK) void k_successor_stree(STreeView st, const cell128 *keys,
                                                              size_t q, uint32_t *owner) {
    __shared__ u128 lds[ST_LDS];
    for (int l = st.lds_from; l <= st.top; ++l)
        for (uint32_t k = threadIdx.x; k < st.sz[l]; k += blockDim.x)
            lds[st.lds_off[l] + k] = ld128(st.lv[l] + k);
    __syncthreads();
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t n = st.sz[0];
    const u128 inf = ~(u128)0;
    for (size_t base = wave * 4 * U; base < q; base += nwaves * 4 * U) {
        u128 x[U];
        uint32_t c[U];
        bool live[U], zero[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t qi = base + u * 4 + g;
            live[u] = qi < q;
            x[u] = live[u] ? ld128(keys + qi) : (u128)0;
            c[u] = 0;
            zero[u] = false;
        }
        for (int l = st.top; l >= 0; --l) {
            const cell128 *L = st.lv[l];
            const uint32_t sz = st.sz[l];
            u128 k[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t idx = c[u] * 16 + li;
                if (l >= st.lds_from)
                    k[u] = idx < sz ? lds[st.lds_off[l] + idx] : inf;
                else
                    k[u] = idx < sz ? ld128(L + idx) : inf;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool lt = live[u] && k[u] < x[u];
                const uint32_t m = (uint32_t)(__ballot(lt) >> (16 * g)) & 0xFFFFu;
                const uint32_t cnt = __popc(m);
                if (l > 0) {
                    if (cnt == 0) zero[u] = true;  // key <= ring[0] (top level only)
                    else if (!zero[u]) c[u] = c[u] * 16 + cnt - 1;
                } else {
                    c[u] = zero[u] ? 0 : c[u] * 16 + cnt;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t qi = base + u * 4 + g;
            if (live[u] && li == 0) {
                const uint32_t sidx = c[u] >= n ? 0u : c[u];
                owner[qi] = PRED ? (sidx == 0 ? n - 1 : sidx - 1) : sidx;
            }
        }
    }
}

hipError_t successor_stree(const STreeView &st, const cell128 *keys, size_t q, uint32_t *owner,
                           bool pred, hipStream_t s) {
    if (q == 0) return hipSuccess;
    constexpr int U = 4;
    const size_t waves = (q + 4 * U - 1) / (4 * U);
    const unsigned blocks = cx_grid(waves * 64, ST_BLOCK, 512);  // 2 per CU (LDS)
    if (pred)
        k_successor_stree<true, U><<<blocks, ST_BLOCK, 0, s>>>(st, keys, q, owner);
    else
        k_successor_stree<false, U><<<blocks, ST_BLOCK, 0, s>>>(st, keys, q, owner);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Search variant 3: wave-cooperative search of the Eytzinger layout itself
// (north_star's "Eytzinger-layout successor search whose top levels are
// staged in LDS, with wavefront-cooperative 128-bit compares using
// ballot/ctz").  Sixteen lanes take one query; a step covers four levels of
// the BFS tree below node k: lane j = 2^t - 1 + o (t < 4, o < 2^t) loads node
// k 2^t + o (the level's nodes are contiguous: 1, 2, 4 and 8 cells), compares
// it with the key in 128 bits, and the group's 16-bit ballot mask is walked
// from the root lane -- lane j's children are lanes 2j + 1 and 2j + 2 -- with
// one bit test per level; the last node on the path that is >= the key is the
// successor, mapped to its sorted index by a BFS -> sorted table (4 B per
// peer, built on first use) instead of summing subtree sizes per lane.  The top
// CX_LDS_LEVELS levels come from LDS, so at 2^24 three of the six steps gather
// from HBM (vs twelve dependent gathers per lane for variant 0).
// ---------------------------------------------------------------------------
template <bool PRED, int U>
__global__ __launch_bounds__(256) void k_successor_eyt16(EytView ev, const uint32_t *rank,
                                                         const cell128 *keys, size_t q,
                                                         uint32_t *owner) {
    __shared__ u128 lds[CX_LDS_NODES];
    eyt_stage_lds(ev, lds);
    const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
    const int lt_t = 31 - __builtin_clz((unsigned)(li + 1));  // level of lane li in the subtree
    const uint32_t lt_o = (uint32_t)(li + 1) - (1u << lt_t);
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
    const uint32_t n = ev.n;
    for (size_t base = wave * 4 * U; base < q; base += nwaves * 4 * U) {
        u128 x[U];
        uint64_t k[U], lb[U];
        bool live[U], run[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t qi = base + u * 4 + g;
            live[u] = qi < q;
            x[u] = live[u] ? ld128(keys + qi) : (u128)0;
            k[u] = 1;
            lb[u] = 0;  // BFS index of the last node >= key on the path (0: none)
            run[u] = live[u];
        }
        for (;;) {
            bool any = false;
#pragma unroll
            for (int u = 0; u < U; ++u) any |= run[u];
            if (__ballot(any) == 0) break;  // wave-uniform
            u128 e[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t node = (k[u] << lt_t) + lt_o;
                e[u] = ~(u128)0;
                if (run[u] && li < 15 && node <= n)
                    e[u] = node <= CX_LDS_NODES ? lds[node - 1] : ld128(ev.E + node);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool lt = run[u] && li < 15 && e[u] < x[u];
                const uint32_t m = (uint32_t)(__ballot(lt) >> (16 * g)) & 0xFFFFu;
                if (!run[u]) continue;
                // walk the four levels from the root lane (uniform in the group):
                // bit j of m says "node of lane j < key" -> go right
                uint32_t j = 0, o = 0;
                const uint64_t kk = k[u];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const uint64_t node = (kk << t) + o;
                    if (node > n) {  // the descent left the tree: done
                        run[u] = false;
                        break;
                    }
                    const uint32_t b = (m >> j) & 1u;
                    if (!b) lb[u] = node;
                    j = 2 * j + 1 + b;
                    o = 2 * o + b;
                }
                if (run[u]) {
                    k[u] = (kk << 4) + o;  // 16 k + the path's four bits
                    if (k[u] > n) run[u] = false;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t qi = base + u * 4 + g;
            if (live[u] && li == 0) {
                // successor = the last node on the path that is >= key; its
                // sorted index from the BFS -> sorted table; none: wrap to 0
                const uint32_t sidx = lb[u] ? rank[lb[u]] : 0u;
                owner[qi] = PRED ? (sidx == 0 ? n - 1 : sidx - 1) : sidx;
            }
        }
    }
}

// rank[k] = sorted index of Eytzinger node k (k = 1..n).
__global__ void k_eyt_rank(uint32_t n, int h, uint32_t *rank) {
    for (size_t k = 1 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; k <= n;
         k += (size_t)gridDim.x * blockDim.x)
        rank[k] = eyt_rank(k, n, h);
}

hipError_t eyt_rank_build(size_t n, uint32_t *rank, hipStream_t s) {
    const int h = 63 - __builtin_clzll((unsigned long long)n);
    k_eyt_rank<<<cx_grid(n, 256), 256, 0, s>>>((uint32_t)n, h, rank);
    return hipGetLastError();
}

hipError_t successor_eyt16(const EytView &ev, const uint32_t *rank, const cell128 *keys, size_t q,
                           uint32_t *owner, bool pred, hipStream_t s) {
    if (q == 0) return hipSuccess;
    constexpr int U = 4;
    const size_t waves = (q + 4 * U - 1) / (4 * U);
    const unsigned blocks = cx_grid(waves * 64, 256, 512);  // 2 per CU (64 KiB of LDS)
    if (pred)
        k_successor_eyt16<true, U><<<blocks, 256, 0, s>>>(ev, rank, keys, q, owner);
    else
        k_successor_eyt16<false, U><<<blocks, 256, 0, s>>>(ev, rank, keys, q, owner);
    return hipGetLastError();
}

// Directory build: lo[b] = first ring index whose ID is >= b << (128 - k).
// Thread j fills the buckets (bucket(ring[j-1]), bucket(ring[j])]; thread n
// fills the tail up to 2^k.
__global__ void k_dir_lo(const cell128 *ring, uint32_t n, int k, uint32_t *lo) {
    const size_t nb = (size_t)1 << k;
    for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j <= n;
         j += (size_t)gridDim.x * blockDim.x) {
        const long long pb = j == 0 ? -1 : (long long)top_bits(ld128(ring + j - 1), k);
        const long long cb = j == n ? (long long)nb : (long long)top_bits(ld128(ring + j), k);
        for (long long b = pb + 1; b <= cb; ++b) lo[b] = (uint32_t)j;
    }
}

__global__ void k_dir_pack(const cell128 *ring, uint32_t n, int k, const uint32_t *lo,
                           uint4 *dir) {
    const size_t nb = (size_t)1 << k;
    for (size_t b = blockIdx.x * (size_t)blockDim.x + threadIdx.x; b < nb;
         b += (size_t)gridDim.x * blockDim.x) {
        const uint32_t a = lo[b], z = lo[b + 1];
        uint64_t frac = 0;
        if (a < z) frac = mid_bits(ld128(ring + a), k);
        dir[b] = make_uint4(a, z, (uint32_t)frac, (uint32_t)(frac >> 32));
    }
}

hipError_t dir_build(const cell128 *ring, size_t n, int k, uint32_t *lo_tmp, uint4 *dir,
                     hipStream_t s) {
    k_dir_lo<<<cx_grid(n + 1, 256), 256, 0, s>>>(ring, (uint32_t)n, k, lo_tmp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    k_dir_pack<<<cx_grid((size_t)1 << k, 256), 256, 0, s>>>(ring, (uint32_t)n, k, lo_tmp, dir);
    return hipGetLastError();
}

// ===========================================================================
// a6: converged finger table.  Lane (p, i): succ(id_p + 2^i).  When 2^i is no
// larger than the gap to the next peer the answer is p+1 without a search.
// ===========================================================================
template <bool DIR>
__global__ __launch_bounds__(SUCC_BLOCK) void k_fingers(SearchView sv, const cell128 *ring,
                                                        uint32_t *F) {
    __shared__ u128 lds[Searcher<DIR>::LDS];
    Searcher<DIR>::stage(sv, lds);
    const uint32_t n = sv.ev.n;
    const size_t total = (size_t)n * CX_FINGERS;
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
         t += (size_t)gridDim.x * blockDim.x) {
        const uint32_t p = (uint32_t)(t >> 7);
        const int i = (int)(t & 127);
        uint32_t f = 0;
        if (n > 1) {
            const u128 idp = ld128(ring + p);
            const uint32_t nx = (p + 1 == n) ? 0u : p + 1;
            const u128 gap = ld128(ring + nx) - idp;  // clockwise distance to next peer
            const u128 step = pow2_128(i);
            f = (step <= gap) ? nx : Searcher<DIR>::find(sv, lds, idp + step);
        }
        F[t] = f;
    }
}

// ---------------------------------------------------------------------------
// Streaming finger build.  For a fixed level i the starts
// id_p + 2^i are increasing in p (clockwise from the first start of a block
// of consecutive peers), so their successors are too.  Two kernels:
//  * plan (one wave per block of FT_P peers): gap exponents glog_p (finger i
//    is the next peer iff i <= glog_p), the block's first level that needs a
//    search anywhere, and s0(i) = succ(id_a + 2^i) for the block's first peer
//    a and every search level i >= FT_L0 -- one directory search each, all in
//    parallel across the grid;
//  * tile (256 threads per block): each wave loads the ring windows
//    s0(i) .. s0(i) + FT_W - 1 of its levels of a chunk at once as 32-bit
//    ID slices (bits [kb, kb + 32) of each ID, kb = 108 - log2 n: coalesced
//    4-B reads of a per-ring slice array), keys them relative to the level's
//    first start, and every peer's successor is a branch-free binary search
//    in its level's window in LDS; the block's FT_P rows leave as full-line
//    16-B stores (next-peer entries filled at write-back).
// Decisions on the keys are exact unless a window key equals the start's or
// the start lies past the window: those entries take the exact directory
// search, as do search levels below FT_L0 = 80 (gaps under 2^80: clustered
// rings only).
// ---------------------------------------------------------------------------
constexpr int FT_P = 128;   // peers per block (rows of the LDS tile)
constexpr int FT_W = 192;   // window elements per level (block span + ~4 sigma)
constexpr int FT_CH = 8;    // levels whose windows are in LDS at once
constexpr int FT_COLS = 40; // tile columns: levels FT_L0..127
constexpr int FT_L0 = CX_FINGERS - FT_COLS;
static_assert(FT_L0 == FINGERS_TILE_L0, "header constant");
static_assert(FT_L0 >= 64, "tile levels need 2^i >= 2^64 (window keys from the top halves)");
constexpr int FT_ROW = FT_COLS + 1;  // padded row: conflict-free column writes

__global__ void k_ring_slice(const cell128 *ring, size_t n, int kb, uint32_t *key) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        key[i] = (uint32_t)bits64(ld128(ring + i), kb);
}

__global__ __launch_bounds__(256) void k_fingers_plan(SearchView sv, const cell128 *ring,
                                                      uint8_t *glog, uint8_t *lvl0,
                                                      uint32_t *S0, uint32_t nblk) {
    const uint32_t n = sv.ev.n;
    const int lane = threadIdx.x & 63;
    const uint32_t b = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (b >= nblk) return;  // wave-uniform
    const uint32_t a = b * FT_P;
    int g = 127;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t p = a + lane + 64 * k;
        if (p < n) {
            const uint32_t nx = p + 1 == n ? 0u : p + 1;
            const int gp = msb128(ld128(ring + nx) - ld128(ring + p));
            glog[p] = (uint8_t)gp;
            g = gp < g ? gp : g;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const int o = __shfl_xor(g, off, 64);
        g = o < g ? o : g;
    }
    const int l0 = g + 1;
    if (lane == 0) lvl0[b] = (uint8_t)(l0 > 128 ? 128 : l0);
    const int i = FT_L0 + lane;
    if (lane < FT_COLS && i >= l0)
        S0[(size_t)b * FT_COLS + lane] = dir_successor(sv, ld128(ring + a) + (pow2_128(i)));
}

// ROWS = false (F null, planes only): every search result goes straight to its
// level plane (coalesced across the wave's rows) instead of through the 21-KB
// row tile, so the block's LDS is the window keys alone (more blocks per CU).
template <bool ROWS>
__global__ __launch_bounds__(256) void k_fingers_tile(SearchView sv, const cell128 *ring,
                                                      const uint32_t *ring_key, int kb,
                                                      const uint8_t *glog_g, const uint8_t *lvl0_g,
                                                      const uint32_t *S0, uint32_t *F,
                                                      uint32_t *FT, int Lft) {
    constexpr int LPW = FT_CH / 4;    // levels per wave per chunk
    constexpr int EPL = FT_W / 64;    // window elements per lane per level
    static_assert(EPL * 64 == FT_W && LPW * 4 == FT_CH, "window geometry");
    __shared__ uint32_t tile[ROWS ? FT_P * FT_ROW : 1];
    __shared__ uint32_t win[4][LPW][256];  // per wave: 32-bit window keys, padded with ~0
    __shared__ uint32_t s0[FT_COLS];
    __shared__ uint8_t glog[FT_P];
    const uint32_t n = sv.ev.n;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t b = blockIdx.x, a = b * FT_P;
    const uint32_t rows = n - a < (uint32_t)FT_P ? n - a : (uint32_t)FT_P;
    const int l0 = lvl0_g[b];
    int lt = l0 > FT_L0 ? l0 : FT_L0;  // first tile level
    if (!F && Lft > lt) lt = Lft;  // planes only: nothing below the first plane level
    if (threadIdx.x < FT_COLS)
        s0[threadIdx.x] = threadIdx.x + FT_L0 >= (unsigned)l0 ? S0[(size_t)b * FT_COLS + threadIdx.x]
                                                             : 0u;
    if (threadIdx.x < rows) glog[threadIdx.x] = glog_g[a + threadIdx.x];
    const u128 ida = ld128(ring + a);
    const uint32_t ka = (uint32_t)bits64(ida, kb);
    // Window keys: for a level i >= kb the start t_p = id_p + 2^i carries
    // nothing into bits [kb, kb + 32) from below, so its slice is
    // slice(id_p) + 2^(i - kb) (mod 2^32) and the key of t_p relative to the
    // level's first start t_a, e_p = slice(t_p) - slice(t_a) = slice(id_p) -
    // slice(id_a) (mod 2^32), is the same at every tile level.  Relative keys
    // order correctly while offsets from t_a stay below 2^(kb + 32) (checked
    // on each window's exact last element and on each peer's offset); equal
    // keys are ties (exact search).
    const u128 lim = pow2_128(kb + 32);
    u128 idp[2];
    uint32_t cp[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t r = lane + 64 * k;
        idp[k] = r < rows ? ld128(ring + a + r) : ida;
        cp[k] = (uint32_t)bits64(idp[k], kb) - ka;
        if (idp[k] - ida >= lim) cp[k] = 0xFFFFFFFFu;  // off the key range: exact search
    }
    __syncthreads();
    // Each wave owns levels c0 + wave + 4q of every chunk: it loads their
    // windows (all EPL x LPW loads in flight at once), converts them to keys
    // in its own LDS rows and searches them; no block barrier until the tile
    // is complete.
    for (int c0 = lt; c0 < CX_FINGERS; c0 += FT_CH) {
        const int nl = CX_FINGERS - c0 < FT_CH ? CX_FINGERS - c0 : FT_CH;
        uint32_t v[LPW][EPL];
#pragma unroll
        for (int q = 0; q < LPW; ++q) {
            const int lv = wave + 4 * q;
            if (lv >= nl) break;  // wave-uniform
            const uint32_t base = s0[c0 + lv - FT_L0];
#pragma unroll
            for (int m = 0; m < EPL; ++m) {
                uint32_t e = base + (uint32_t)(lane + 64 * m);
                e = e >= n ? e - n : e;  // n > FT_W (launcher)
                v[q][m] = ring_key[e];
            }
        }
        // lane q: the arc of level q's window, from its exact last element
        bool arc = false;
        if (lane < LPW && wave + 4 * lane < nl) {
            const int lv = wave + 4 * lane;
            uint32_t e = s0[c0 + lv - FT_L0] + FT_W - 1;
            e = e >= n ? e - n : e;
            arc = (ld128(ring + e) - (ida + (pow2_128(c0 + lv)))) < lim;
        }
        const uint32_t arcbits = (uint32_t)__ballot(arc);
#pragma unroll
        for (int q = 0; q < LPW; ++q) {
            const int lv = wave + 4 * q;
            if (lv >= nl) break;
            const int lvl = c0 + lv;
            const uint32_t kta = ka + (lvl - kb < 32 ? 1u << (lvl - kb) : 0u);  // slice(t_a)
#pragma unroll
            for (int m = 0; m < EPL; ++m) win[wave][q][lane + 64 * m] = v[q][m] - kta;
            if (lane < 256 - FT_W) win[wave][q][FT_W + lane] = 0xFFFFFFFFu;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // both peers x LPW levels: independent branch-free searches, their LDS
        // reads issued together step by step
        uint32_t j[LPW][2];
#pragma unroll
        for (int q = 0; q < LPW; ++q) j[q][0] = j[q][1] = 0;
#pragma unroll
        for (uint32_t st = 128; st; st >>= 1) {
#pragma unroll
            for (int q = 0; q < LPW; ++q) {
                const uint32_t *w = win[wave][q];  // rows past nl hold stale keys: unused
#pragma unroll
                for (int k = 0; k < 2; ++k) j[q][k] += w[j[q][k] + st - 1] < cp[k] ? st : 0u;
            }
        }
#pragma unroll
        for (int q = 0; q < LPW; ++q) {
            const int lv = wave + 4 * q;
            if (lv >= nl) break;  // wave-uniform
            const int i = c0 + lv;
            const uint32_t base = s0[i - FT_L0];
            const uint32_t *w = win[wave][q];
            const bool aok = (arcbits >> q) & 1u;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t r = lane + 64 * k;
                if (r >= rows) continue;
                if (i <= glog[r]) {  // next peer: filled at write-back (rows) / now (planes)
                    if (!ROWS && i >= Lft)
                        __builtin_nontemporal_store(a + r + 1 == n ? 0u : a + r + 1,
                                                    FT + (size_t)(i - Lft) * n + a + r);
                    continue;
                }
                uint32_t f = CX_NONE;
                const uint32_t jj = j[q][k];
                if (aok && jj < FT_W && w[jj] != cp[k]) {
                    const uint32_t e = base + jj;
                    f = e >= n ? e - n : e;
                }
                if (f == CX_NONE)  // tie on the key / past the window / no arc
                    f = dir_successor(sv, idp[k] + (pow2_128(i)));
                if (ROWS)
                    tile[r * FT_ROW + (i - FT_L0)] = f;
                else if (i >= Lft)
                    __builtin_nontemporal_store(f, FT + (size_t)(i - Lft) * n + a + r);
            }
        }
        __builtin_amdgcn_wave_barrier();  // searches done before the next chunk's keys
    }
    if (!ROWS) {
        // planes only: the levels below the block's first tile level are the
        // next peer for every row (each gap is at least 2^(l0 - 1))
        for (int k = threadIdx.x; k < (lt - Lft) * (int)FT_P; k += blockDim.x) {
            const int c = k / FT_P, r = k - c * FT_P;
            if (r >= (int)rows) continue;
            const uint32_t p = a + r;
            __builtin_nontemporal_store(p + 1 == n ? 0u : p + 1, FT + (size_t)c * n + p);
        }
        return;
    }
    __syncthreads();
    // write-back: 8 rows per pass, 16 B per thread, full 512-B rows
    const int chunk = threadIdx.x & 31;
    for (int r = threadIdx.x >> 5; r < (int)rows; r += 8) {
        const uint32_t p = a + r;
        const uint32_t nx = p + 1 == n ? 0u : p + 1;
        const int g = glog[r];
        uint4 o;
        if (chunk * 4 + 3 <= g) {  // all four levels are the next peer
            o = make_uint4(nx, nx, nx, nx);
        } else {
            uint32_t v[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int i = chunk * 4 + c;
                if (i <= g)
                    v[c] = nx;
                else if (i >= FT_L0)
                    v[c] = tile[r * FT_ROW + (i - FT_L0)];
                else  // a gap under 2^88 (clustered rings): exact search
                    v[c] = dir_successor(sv, ld128(ring + p) + (pow2_128(i)));
            }
            o = make_uint4(v[0], v[1], v[2], v[3]);
        }
        // streaming store: 8 GiB of rows nobody re-reads soon from L2
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u ov = {o.x, o.y, o.z, o.w};
        __builtin_nontemporal_store(ov, reinterpret_cast<v4u *>(F + (size_t)p * CX_FINGERS) + chunk);
    }
    // optional: the level planes FT[(l - Lft) n + p] = F[p][l] for l >= Lft
    // (>= FT_L0) that the route-table build reads, straight from the tile --
    // 512 contiguous bytes per level and block instead of a transpose pass
    // over the finger table
    if (FT) {
        const uint32_t n_ = n;
        const int nlev = CX_FINGERS - Lft;
        for (int k = threadIdx.x; k < nlev * FT_P; k += blockDim.x) {
            const int c = k / FT_P, r = k - c * FT_P;
            if (r >= (int)rows) continue;
            const int i = Lft + c;
            const uint32_t p = a + r;
            const uint32_t v = i <= glog[r] ? (p + 1 == n_ ? 0u : p + 1)
                                             : tile[r * FT_ROW + (i - FT_L0)];
            __builtin_nontemporal_store(v, FT + (size_t)c * n_ + p);
        }
    }
}

// ---------------------------------------------------------------------------
// f2 finger repair (finger_table.h:148-168 AdjustFingers / ReplaceDeadPeer,
// abstract_chord_peer.cpp:615-645 FixOtherFingers, batched over a churn):
// the finger level planes of the new ring from the parent ring's planes.  A
// survivor p (old index o) keeps finger level l's target t = id_p + 2^l, and
// its old finger x = succ_old(t) satisfies t in (id_{x-1}, id_x].  If x
// survived (y = o2n[x]) and so did x - 1, with nothing inserted between them
// (o2n[x - 1] = y - 1, cyclic), the new ring holds no peer in
// (id_{x-1}, id_x) either, so succ_new(t) = y: the finger is remapped.
// Otherwise -- x left (ReplaceDeadPeer), a join landed in x's gap
// (AdjustFingers), x - 1 left, or p itself joined -- the finger is searched
// exactly on the new ring's directory.  Bit-identical to the streaming build.
// ---------------------------------------------------------------------------
__global__ void k_invert_o2n(const uint32_t *o2n, uint32_t n_old, uint32_t n_new, uint32_t *n2o) {
    for (uint32_t o = blockIdx.x * blockDim.x + threadIdx.x; o < n_old; o += gridDim.x * blockDim.x) {
        const uint32_t y = o2n[o];
        if (y < n_new) n2o[y] = o;
    }
}

constexpr int PR_MAX = CX_FINGERS - FINGERS_TILE_L0;  // plane levels at most (tile levels)
__global__ __launch_bounds__(256) void k_planes_repair(SearchView sv, const cell128 *ring,
                                                       uint32_t n, const uint32_t *Pold,
                                                       uint32_t n_old, const uint32_t *o2n,
                                                       const uint32_t *n2o, int L, int nl,
                                                       uint32_t *Pnew, uint32_t *nsearch) {
    // one lane per new peer; the remapped fingers go to LDS, the lane then
    // searches its own failed levels one per round (rounds = the wave's
    // largest count, not the number of levels any lane failed), and every
    // level leaves as one coalesced store per wave
    __shared__ uint32_t val[PR_MAX][256];
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = p < n;
    const uint32_t o = valid ? n2o[p] : CX_NONE;
    uint64_t miss = 0;
#pragma unroll
    for (int c = 0; c < PR_MAX; ++c) {
        if (c >= nl || !valid) break;
        uint32_t f = CX_NONE;
        if (o < n_old) {
            const uint32_t x = Pold[(size_t)c * n_old + o];
            if (x < n_old) {
                const uint32_t y = o2n[x];
                const uint32_t ym = o2n[x ? x - 1 : n_old - 1];
                if (y < n && ym == (y ? y - 1 : n - 1)) f = y;
            }
        }
        if (f == CX_NONE) miss |= 1ull << c;  // joined peer, or a churn event at the finger
        val[c][threadIdx.x] = f;
    }
    uint32_t searched = 0;
    if (miss) {
        const u128 idp = ld128(ring + p);
        while (miss) {
            const int c = __builtin_ctzll(miss);
            miss &= miss - 1;
            val[c][threadIdx.x] = dir_successor(sv, idp + (pow2_128(L + c)));
            ++searched;
        }
    }
    if (valid)
        for (int c = 0; c < nl; ++c)
            __builtin_nontemporal_store(val[c][threadIdx.x], Pnew + (size_t)c * n + p);
    if (nsearch && searched) atomicAdd(nsearch, searched);
}

hipError_t planes_repair(const SearchView &sv, const cell128 *ring, size_t n, const uint32_t *Pold,
                         size_t n_old, const uint32_t *o2n, uint32_t *n2o, int L, int nl,
                         uint32_t *Pnew, uint32_t *nsearch, hipStream_t s) {
    if (n == 0 || n_old == 0 || nl <= 0 || nl > PR_MAX || L < 0 || L + nl > CX_FINGERS || !sv.dir)
        return hipErrorInvalidValue;
    hipError_t e = fill_u32(n2o, n, CX_NONE, s);
    if (e != hipSuccess) return e;
    k_invert_o2n<<<cx_grid(n_old, 256), 256, 0, s>>>(o2n, (uint32_t)n_old, (uint32_t)n, n2o);
    k_planes_repair<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(sv, ring, (uint32_t)n, Pold,
                                                               (uint32_t)n_old, o2n, n2o, L, nl,
                                                               Pnew, nsearch);
    return hipGetLastError();
}

// Slice position of the streaming finger build: the expected span of a
// window (FT_W gaps, 2^(135.6 - log2 n)) stays far below 2^(kb + 32), and
// kb <= FT_L0 so every tile level is >= kb.
int finger_key_shift(size_t n) {
    int lg = 0;
    while (((size_t)1 << lg) < n) ++lg;
    const int kb = 108 - lg;
    return kb > FT_L0 ? FT_L0 : (kb < 0 ? 0 : kb);
}

hipError_t ring_slice_build(const cell128 *ring, size_t n, int kb, uint32_t *key, hipStream_t s) {
    k_ring_slice<<<cx_grid(n, 256), 256, 0, s>>>(ring, n, kb, key);
    return hipGetLastError();
}

// ring_key (n ID slices, ring_slice_build at finger_key_shift(n)) selects the
// streaming build for rings of 2^18 peers or more; smaller rings (whose
// windows would span too much of the circle for 32-bit keys) take one
// directory search per entry.
size_t fingers_workspace_bytes(size_t n) {
    const size_t nblk = (n + FT_P - 1) / FT_P;
    return n + nblk + nblk * FT_COLS * sizeof(uint32_t) + 16;
}

hipError_t fingers_build(const SearchView &sv, const cell128 *ring, const uint32_t *ring_key,
                         void *ws, uint32_t *F, hipStream_t s, uint32_t *FT, int Lft,
                         bool *planes_done) {
    const size_t n = sv.ev.n;
    if (planes_done) *planes_done = false;
    const bool stream_ok = ring_key && ws && sv.dir && n >= ((size_t)1 << 18);
    // F null = planes only: needs the streaming build and every plane a tile level
    if (!F && (!stream_ok || !FT || Lft < FT_L0 || Lft >= CX_FINGERS)) return hipErrorInvalidValue;
    if (stream_ok) {
        const uint32_t nblk = (uint32_t)((n + FT_P - 1) / FT_P);
        uint32_t *S0 = static_cast<uint32_t *>(ws);
        uint8_t *glog = reinterpret_cast<uint8_t *>(S0 + (size_t)nblk * FT_COLS);
        uint8_t *lvl0 = glog + n;
        k_fingers_plan<<<(nblk + 3) / 4, 256, 0, s>>>(sv, ring, glog, lvl0, S0, nblk);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        // planes straight from the tile when every plane level is a tile level
        const bool planes = FT && Lft >= FT_L0 && Lft < CX_FINGERS;
        if (F)
            k_fingers_tile<true><<<nblk, 256, 0, s>>>(sv, ring, ring_key, finger_key_shift(n), glog,
                                                      lvl0, S0, F, planes ? FT : nullptr, Lft);
        else
            k_fingers_tile<false><<<nblk, 256, 0, s>>>(sv, ring, ring_key, finger_key_shift(n), glog,
                                                       lvl0, S0, F, FT, Lft);
        if (planes_done) *planes_done = planes;
        return hipGetLastError();
    }
    const size_t total = n * CX_FINGERS;
    if (sv.dir)
        k_fingers<true><<<cx_grid(total, SUCC_BLOCK, 2048), SUCC_BLOCK, 0, s>>>(sv, ring, F);
    else
        k_fingers<false><<<cx_grid(total, SUCC_BLOCK, 512), SUCC_BLOCK, 0, s>>>(sv, ring, F);
    return hipGetLastError();
}

// ===========================================================================
// a7-a9: routed lookup, converged table.
// StoredLocally(src) = key in (ring[src-1], ring[src]] (min_key = pred + 1).
// Each hop: i = msb(key - id_cur) (= FingerTable::Lookup's first match),
// nxt = F[cur][i].  Because nxt = succ(id_cur + 2^i) and key - id_cur >= 2^i,
// StoredLocally(nxt) <=> key - id_cur <= id_nxt - id_cur: the hop needs only
// the finger and the next peer's ID (no predecessor gather).  The self ->
// predecessor substitution of ForwardRequest (chord_peer.cpp:195-197) cannot
// trigger on a converged table ("route").
// ===========================================================================
constexpr int ROUTE_BLOCK = 256;

__global__ __launch_bounds__(ROUTE_BLOCK) void k_route_conv(const cell128 *ring, uint32_t n,
                                                            const uint32_t *F,
                                                            const uint32_t *src,
                                                            const cell128 *keys, size_t q,
                                                            uint32_t *owner, uint8_t *hops,
                                                            uint8_t *status) {
    for (size_t qi = blockIdx.x * (size_t)blockDim.x + threadIdx.x; qi < q;
         qi += (size_t)gridDim.x * blockDim.x) {
        const u128 key = ld128(keys + qi);
        uint32_t cur = src[qi];
        uint32_t own = cur, h = 0;
        uint8_t st = CX_Q_OK;
        if (cur >= n) {
            own = CX_NONE;
            st = CX_Q_BADPEER;
        } else if (n > 1) {
            u128 idc = ld128(ring + cur);
            const u128 idp = ld128(ring + (cur == 0 ? n - 1 : cur - 1));
            const bool local = (key - idp - 1) <= (idc - idp - 1);
            if (!local) {
                for (;;) {
                    const u128 d = key - idc;
                    const int i = msb128(d);
                    const uint32_t nxt = F[(size_t)cur * CX_FINGERS + i];
                    if (nxt >= n) {  // corrupt table: never gather out of bounds
                        own = CX_NONE;
                        st = CX_Q_BADPEER;
                        break;
                    }
                    const u128 idn = ld128(ring + nxt);
                    ++h;
                    if (d <= idn - idc) {
                        own = nxt;
                        break;
                    }
                    if (h == CX_HOP_CAP) {
                        own = CX_NONE;
                        st = CX_Q_HOPCAP;
                        break;
                    }
                    cur = nxt;
                    idc = idn;
                }
            }
        }
        owner[qi] = own;
        hops[qi] = (uint8_t)h;
        if (status) status[qi] = st;
    }
}

// ChordKey::InBetween(lb, ub, true) (key.h:103-131) on canonical operands.
__device__ __forceinline__ bool in_between128(u128 v, u128 lb, u128 ub) {
    if (lb == ub) return v == ub;
    if (lb < ub) return lb <= v && v <= ub;
    return !(ub < v && v < lb);
}

// Liveness and successors_ lists of the peers (LitState): the dead-finger
// branch of ForwardRequest.  alive == nullptr: every server answers; succs ==
// nullptr: converged lists (the next min(ns, n-1) peers clockwise).
__device__ __forceinline__ bool lit_alive(const LitState &ls, uint32_t n, uint32_t p) {
    if (p >= n) return false;  // also CX_NONE: an unset RemotePeer never answers
    return ls.alive ? ls.alive[p] != 0 : true;
}
__device__ __forceinline__ uint32_t lit_succ(const LitState &ls, uint32_t n, uint32_t p, int j) {
    if (j >= ls.ns) return CX_NONE;
    if (ls.succs) return ls.succs[(size_t)p * ls.ns + j];
    if ((uint32_t)j >= n - 1) return CX_NONE;
    uint32_t e = p + 1 + (uint32_t)j;
    return e >= n ? e - n : e;
}
// RemotePeerList::Lookup(key, succ = true) (remote_peer_list.cpp:86-110): the
// first entry whose (previous, id] -- InBetween inclusive, previous starting at
// the list owner's id -- holds the key.  Also returns the list index.
__device__ __forceinline__ uint32_t lit_list_lookup(const LitState &ls, const cell128 *ring,
                                                    uint32_t n, uint32_t p, u128 key, int &at) {
    u128 prev = ld128(ring + p);
    for (int j = 0; j < ls.ns; ++j) {
        const uint32_t e = lit_succ(ls, n, p, j);
        if (e == CX_NONE) break;
        const u128 id = ld128(ring + e);
        if (in_between128(key, prev, id)) {
            at = j;
            return e;
        }
        prev = id;
    }
    at = -1;
    return CX_NONE;
}

// Literal walk for hand-edited tables / peer state: StoredLocally with the
// peer's own min_key_ (InBetween(min_key, id, true), key.h:103-131 on
// canonical operands), first-match finger (CX_NONE = no finger added for that
// range: "ChordKey not found", finger_table.h:129), self -> live predecessor
// substitution, and the dead-finger fallback of ChordPeer::ForwardRequest
// (chord_peer.cpp:201-208: successors_.Lookup if alive, else "Lookup failed")
// or DHashPeer::ForwardRequest (dhash_peer.cpp:516-526: LookupLiving -- whose
// scan for a later living entry never runs, remote_peer_list.cpp:123 -- else
// successors_[0] if alive, else "Lookup failed").
__global__ __launch_bounds__(ROUTE_BLOCK) void k_route_literal(
    const cell128 *ring, uint32_t n, const uint32_t *F, const cell128 *min_keys,
    const uint32_t *preds, LitState ls, const uint32_t *src, const cell128 *keys, size_t q,
    uint32_t *owner, uint8_t *hops, uint8_t *status) {
    for (size_t qi = blockIdx.x * (size_t)blockDim.x + threadIdx.x; qi < q;
         qi += (size_t)gridDim.x * blockDim.x) {
        const u128 key = ld128(keys + qi);
        uint32_t cur = src[qi], h = 0, own = CX_NONE;
        uint8_t st = CX_Q_OK;
        for (;;) {
            if (cur >= n) {
                st = CX_Q_BADPEER;
                own = CX_NONE;
                break;
            }
            const u128 id = ld128(ring + cur);
            const uint32_t pdef = (n == 1) ? CX_NONE : (cur == 0 ? n - 1 : cur - 1);
            const u128 mk = min_keys ? ld128(min_keys + cur)
                                     : ld128(ring + (n == 1 ? cur : pdef)) + 1;
            if (in_between128(key, mk, id)) {
                own = cur;
                break;
            }
            const int i = msb128(key - id);  // key != id here (id is always local)
            uint32_t nxt = F[(size_t)cur * CX_FINGERS + i];
            if (nxt == CX_NONE) {  // the range's finger was never added
                st = CX_Q_NOT_FOUND;
                own = CX_NONE;
                break;
            }
            const uint32_t pr = preds ? preds[cur] : pdef;
            if (nxt == cur && lit_alive(ls, n, pr)) {
                nxt = pr;
            } else if (!lit_alive(ls, n, nxt)) {
                int at;
                const uint32_t sl = lit_list_lookup(ls, ring, n, cur, key, at);
                if (ls.rule == CX_FWD_DHASH) {
                    const uint32_t s0 = lit_succ(ls, n, cur, 0);
                    nxt = lit_alive(ls, n, sl) ? sl : (lit_alive(ls, n, s0) ? s0 : CX_NONE);
                } else {
                    nxt = lit_alive(ls, n, sl) ? sl : CX_NONE;
                }
                if (nxt == CX_NONE) {
                    st = CX_Q_FAILED;
                    own = CX_NONE;
                    break;
                }
            }
            if (h == CX_HOP_CAP) {
                st = CX_Q_HOPCAP;
                own = CX_NONE;
                break;
            }
            ++h;
            cur = nxt;
        }
        owner[qi] = own;
        hops[qi] = (uint8_t)h;
        if (status) status[qi] = st;
    }
}

__global__ void k_ring_ext(const cell128 *ring, uint32_t n, cell128 *ext) {
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t <= n;
         t += (size_t)gridDim.x * blockDim.x)
        st128(ext + t, ld128(ring + (t == 0 ? n - 1 : t - 1)));
}

hipError_t ring_ext_build(const cell128 *ring, size_t n, cell128 *ring_ext, hipStream_t s) {
    k_ring_ext<<<cx_grid(n + 1, 256), 256, 0, s>>>(ring, (uint32_t)n, ring_ext);
    return hipGetLastError();
}

// Converged walks over a route table.  Each wave owns a contiguous chunk of
// queries and a scalar queue head; a lane that finishes takes the next index
// (ballot + mbcnt), so lanes never idle behind the wave's longest walk.  Every
// loop iteration is ONE dependent load round per lane.
constexpr int RT_BLOCK = 256;

// Level of the next hop, FingerTable::Lookup's first match = msb(key - id),
// for id in [lo, lo + w]:  -1 if the interval does not decide it.
__device__ __forceinline__ int level_iv(u128 key, u128 lo, u128 w) {
    const u128 a = key - lo;          // = key - id_min
    if (a <= w) return -1;            // key inside the interval (or d could be 0)
    const u128 b = a - w;             // = key - id_max  (> 0)
    const int i = msb128(a);
    return msb128(b) == i ? i : -1;
}

// StoredLocally(nxt) for the hop cur -> nxt: key in (id_cur, id_nxt].
// 1 = stored at nxt, 0 = not, -1 = undecided by the intervals.
__device__ __forceinline__ int term_iv(u128 key, u128 clo, u128 cw, u128 nlo, u128 nw) {
    const u128 a = key - clo;         // dk in [a - cw, a]   (a > cw: checked by level_iv)
    const u128 b = nlo - clo;         // dn in [b - cw, b + nw]
    if (b < cw) return -1;            // id_nxt may precede id_cur's interval end
    if (b + nw < b) return -1;        // wraps past 2^128
    if (a <= b - cw) return 1;        // dk_max <= dn_min
    if (a - cw > b + nw) return 0;    // dk_min > dn_max
    return -1;
}

// ---------------------------------------------------------------------------
// k_route_tree (the v4 lookahead-tree walk above 2^24 peers, and the arc
// walks over the cz table):
//  * result staging: a finished query's (owner, hops, status) goes to a
//    per-wave LDS window; 64 consecutive results are flushed as coalesced
//    stores (one 256-B owner store, two 64-B byte stores) instead of three
//    scattered stores per query.  The wave's queue never hands out an index
//    beyond flushed + RES_WIN, so every in-flight query has a window slot.
//  * a two-slot pipeline per lane: slot B prefetches the next query's key,
//    src and (pred, self) pair while slot A walks, so a new query starts
//    walking in the iteration its predecessor finishes (no init round).
// ---------------------------------------------------------------------------
constexpr int RES_WIN = 512;
// A_EXACT (cz walk): fetch id(cur) and id(cur + 1) for an exact hop below the
// table in the memory round, so the hop needs no load of its own
enum { A_NONE = 0, A_HOP = 1, A_FIXC = 2, A_FIXT = 3, A_EXACT = 4 };
enum { B_EMPTY = 0, B_KS = 1, B_PAIR = 2 };

struct PkCtx {
    const cell128 *ring;
    const uint32_t *F;
    uint32_t n;
    int l0, ib, S;
    uint64_t imask;
    u128 W;
    // variant 5 (cz): gap-code shift of a compressed node
    int gs;
    // arc mode (cz rows): levels >= Lh are replicated; below Lh only the M
    // peers plo, plo + 1, ... (cyclic: the rank's arc and its halo) have rows
    // and no finger table: exact below-table fingers by directory search
    bool arc;
    int Lh;
    uint32_t plo, M;
    SearchView sv;
};

__device__ __forceinline__ bool arc_row_local(const PkCtx &c, uint32_t cur) {
    const uint32_t j = cur >= c.plo ? cur - c.plo : cur + c.n - c.plo;
    return j < c.M;
}

// finger(p, i) = succ(id_p + 2^i) on the converged ring (k_fingers' rule).
__device__ __forceinline__ uint32_t finger_of(const SearchView &sv, const cell128 *ring, uint32_t n,
                                              uint32_t p, int i, u128 idp) {
    if (n == 1) return 0;
    const uint32_t nx = (p + 1 == n) ? 0u : p + 1;
    const u128 step = pow2_128(i);
    return (step <= ld128(ring + nx) - idp) ? nx : dir_successor(sv, idp + step);
}

__device__ __forceinline__ uint64_t pack_res(uint32_t own, uint32_t h, uint8_t st) {
    return (1ull << 63) | ((uint64_t)st << 40) | ((uint64_t)(h & 0xFF) << 32) | own;
}

// ---------------------------------------------------------------------------
// Variant 4: lookahead-tree route table.  Entry (p, i) is 64 B = 8 packed
// fingers (same 8-B packing as variant 2):
//   slot 0: A   = f(p, i)
//   slot 1: f(A, i-1)      slot 2: f(A, i-2)      slot 4: f(A, i-3)
//   slot 3: f(s1, i-2)     slot 5: f(s1, i-3)     slot 6: f(s2, i-3)
//   slot 7: f(s3, i-3)
// i.e. A's fingers one to three levels down and the next step along the most
// likely level-drop paths (1,1), (1,2), (2,1), (1,1,1): a walk whose levels
// follow a stored path hops with no gather (simulated: 45 % of hops gather,
// vs 71 % with one lookahead finger).  The 64 B are loaded by the 4 lanes of
// a quad with one 16-B load each (one coalesced request, measured at the
// 16-B single-lane rate), transposed through LDS; each lane keeps its entry in
// LDS and reads fingers by slot.
// Child table: slot s at offset o below the entry's root level -> child slot.
// ---------------------------------------------------------------------------
constexpr uint64_t TREE_CHILD = (1ull << 4) | (2ull << 8) | (4ull << 12) | (3ull << 24) |
                                (5ull << 28) | (6ull << 44) | (7ull << 60);

__device__ __forceinline__ int tree_child(int s, int o) {
    if (s > 3 || o < 1 || o > 3) return 0;
    return (int)((TREE_CHILD >> (4 * (s * 4 + o))) & 15);
}

__global__ void k_tree_build(const uint32_t *F, const cell128 *ring, uint32_t n, int l0, int R,
                             int ib, uint64_t *tree) {
    const size_t total = (size_t)n * R;
    const int S = 64 + ib;
    for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total;
         t += (size_t)gridDim.x * blockDim.x) {
        const size_t p = t / (unsigned)R;
        const int i = l0 + (int)(t - p * (unsigned)R);
        uint32_t f[8];
        // (parent slot, level offset) of slots 1..7
        const int par[8] = {-1, 0, 0, 1, 0, 1, 2, 3};
        const int off[8] = {0, 1, 2, 2, 3, 3, 3, 3};
        f[0] = F[p * CX_FINGERS + i];
#pragma unroll
        for (int sl = 1; sl < 8; ++sl) {
            const int lv = i - off[sl];
            f[sl] = lv >= 0 ? F[(size_t)f[par[sl]] * CX_FINGERS + lv] : CX_NONE;
        }
        uint64_t *e = tree + t * 8;
#pragma unroll
        for (int sl = 0; sl < 8; ++sl)
            e[sl] = f[sl] == CX_NONE ? ~0ull
                                     : ((bits64(ld128(ring + f[sl]), S) << ib) | f[sl]);
    }
}

hipError_t tree_build(const uint32_t *F, const cell128 *ring, size_t n, int l0, int R, int ib,
                      uint64_t *tree, hipStream_t s) {
    k_tree_build<<<cx_grid(n * (size_t)R, 256), 256, 0, s>>>(F, ring, (uint32_t)n, l0, R, ib,
                                                             tree);
    return hipGetLastError();
}

// Plan from cur using the lane's LDS entry `ent` (8 fingers) for free hops.
// cs = slot of the node we stand on (-1: no entry), ri = the entry's root level.
__device__ __forceinline__ int tree_plan(const PkCtx &c, u128 key, u128 &clo, bool &cex,
                                         uint32_t &cur, uint32_t &h, uint32_t &pn, int &mode,
                                         int &lvl, int &cs, int ri, const uint64_t *ent,
                                         uint32_t &own, uint8_t &st) {
    for (;;) {
        const u128 cw = cex ? (u128)0 : c.W;
        const int i = level_iv(key, clo, cw);
        if (i < 0) {
            mode = A_FIXC;
            return 0;
        }
        const int ch = cs >= 0 ? tree_child(cs, ri - i) : 0;
        if (ch) {
            cs = ch;
            const uint64_t f = ent[ch];
            const uint32_t nxt = (uint32_t)(f & c.imask);
            const u128 nlo = shl128((u128)(f >> c.ib), c.S);
            ++h;
            const int t = term_iv(key, clo, cw, nlo, c.W);
            if (t == 1) {
                own = nxt;
                return 1;
            }
            if (t < 0) {
                mode = A_FIXT;
                pn = nxt;
                return 0;
            }
            if (h == CX_HOP_CAP) {
                own = CX_NONE;
                st = CX_Q_HOPCAP;
                return 1;
            }
            cur = nxt;
            clo = nlo;
            cex = false;
            continue;
        }
        cs = -1;
        if (i >= c.l0) {
            mode = A_HOP;
            lvl = i;
            return 0;
        }
        // rare: below the table -> exact finger + exact ids
        const u128 idc = cex ? clo : ld128(c.ring + cur);
        const uint32_t nxt = c.F[(size_t)cur * CX_FINGERS + i];
        const u128 idn = ld128(c.ring + nxt);
        ++h;
        if (key - idc <= idn - idc) {
            own = nxt;
            return 1;
        }
        if (h == CX_HOP_CAP) {
            own = CX_NONE;
            st = CX_Q_HOPCAP;
            return 1;
        }
        cur = nxt;
        clo = idn;
        cex = true;
    }
}

// ---------------------------------------------------------------------------
// Variant 5 ("cz"): pattern-keyed window entries of sixteen 4-B nodes.
//
// The walk consumes the bits of d = key - id_cur from the top: a hop at level
// i = msb(d) clears bit i (plus the successor gap, ~2^104 at 2^24 peers), so
// the levels a walk visits after A = finger(p, i) follow the set bits of d
// below i.  Entry (p, i, b) is keyed by b = bit i-1 of d - 2^i, read by the
// gathering lane, and holds the peers of the window of four levels after the
// forced part of the path:
//   b = 0: slot v (v = a 4-bit subset of the levels i-2..i-5, bit w <-> level
//          i-2-w) = the peer reached from A by hops at v's levels (in
//          descending order); slot 0 = A itself;
//   b = 1: slot 15 = A; slot v = the peer reached from A' = finger(A, i-1) by
//          hops at v's levels (v = 15 is not stored).
// Simulated on a 2^24 ring: 0.34 gathers per hop, vs 0.44 for the 8-finger
// tree of variant 4 (0.39 for a 1-bit pattern with 8 fingers, 0.38 for a
// 16-finger tree), at twice variant 4's table size (one 64-B entry per bit b).
//
// A node is stored relative to its parent (the peer the hop leaves, at level
// l): bits 0..15 = idx - idx_par - E(l) + 2^15 (mod n, signed), with
// E(l) = round(n * 2^(l-128)) the expected index advance; bits 16..31 =
// (id - id_par - 2^l) >> gs, the successor gap in units of 2^gs (gs = 116 - ib:
// 16x the mean gap fits).  CZ_NONE = not representable (the walk then
// gathers or takes the exact finger).  Decoded IDs are intervals whose width
// grows by 2^gs - 1 per relative hop; every decision is taken on the
// interval, and an undecided one fetches the exact IDs (A_FIXC / A_FIXT).
// ---------------------------------------------------------------------------
constexpr uint32_t CZ_NONE = 0xFFFFFFFFu;
constexpr int CZ_RES_WIN = 256;  // 26 KB of LDS per 256-lane block: 6 blocks per CU
constexpr int CZ_WAVES = 5;      // waves per SIMD the VGPR budget allows (88 VGPRs; 6 spills)


__device__ __forceinline__ uint32_t cz_expect(uint32_t n, int l) {
    const int sh = 128 - l;
    return sh > 40 ? 0u : (uint32_t)(((uint64_t)n + (1ull << (sh - 1))) >> sh);
}

__device__ __forceinline__ uint32_t cz_next(uint32_t n, uint32_t cur, int l, uint32_t wd) {
    int t = (int)cur + (int)cz_expect(n, l) + (int)(wd & 0xFFFF) - 32768;  // n < 2^30
    if (t < 0)
        t += (int)n;
    else if (t >= (int)n)
        t -= (int)n;
    return (uint32_t)t;
}

// Level planes of the finger table: FT[(l - L) * n + p] = F[p][l] for
// l in [L, L + nl).  The cz build's gathers F[x][l] come from lanes whose x
// are neighbours (adjacent peers' fingers at one level are adjacent peers), so
// in planes a wave's 64 gathers touch a few cache lines instead of 64 rows
// 512 B apart.  One block = 64 peers: rows in (coalesced 4-B runs), LDS
// transpose, plane segments out.
__global__ void k_fingers_levels(const uint32_t *F, uint32_t n, int L, int nl, uint32_t *FT) {
    __shared__ uint32_t t[CX_FINGERS][65];
    const size_t p0 = (size_t)blockIdx.x * 64;
    const int rows = (int)(n - p0 < 64 ? n - p0 : 64);
    for (int k = threadIdx.x; k < rows * nl; k += blockDim.x) {
        const int r = k / nl, c = k - r * nl;
        t[c][r] = F[(p0 + r) * CX_FINGERS + L + c];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < nl * 64; k += blockDim.x) {
        const int c = k >> 6, r = k & 63;
        if (r < rows) __builtin_nontemporal_store(t[c][r], FT + (size_t)c * n + p0 + r);
    }
}

// Two-hop planes: C2[(l - L - 1) n + x] = F[F[x][l]][l - 1].  One gather per
// entry into the plane below (adjacent x -> adjacent fingers: coalesced-ish).
// Rings whose size is not a multiple of four: one lane per peer, a plane per
// grid row.
__global__ void k_fingers_pairs_1(const uint32_t *FT, uint32_t n, int nl, uint32_t *C2) {
    const size_t k = blockIdx.y;
    const uint32_t *up = FT + (k + 1) * (size_t)n, *lo = FT + k * (size_t)n;
    uint32_t *out = C2 + k * (size_t)n;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x) {
        const uint32_t y = up[x];
        __builtin_nontemporal_store(y < n ? lo[y] : CX_NONE, out + x);
    }
}

// One plane per grid row (no 64-bit division per element), four consecutive
// peers per lane: 16-B loads of the level-(l) plane, four gathers into the
// level-(l - 1) plane (near-consecutive: the fingers of consecutive peers),
// one 16-B streaming store.
__global__ void k_fingers_pairs(const uint32_t *FT, uint32_t n, int nl, uint32_t *C2) {
    const size_t k = blockIdx.y;  // C2 plane k = level L + 1 + k
    const uint32_t *up = FT + (k + 1) * (size_t)n, *lo = FT + k * (size_t)n;
    uint32_t *out = C2 + k * (size_t)n;
    const uint32_t n4 = n / 4;
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += gridDim.x * blockDim.x) {
        const uint4 y = reinterpret_cast<const uint4 *>(up)[q];
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u r = {y.x < n ? lo[y.x] : CX_NONE, y.y < n ? lo[y.y] : CX_NONE,
                       y.z < n ? lo[y.z] : CX_NONE, y.w < n ? lo[y.w] : CX_NONE};
        __builtin_nontemporal_store(r, reinterpret_cast<v4u *>(out) + q);
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3u)) {  // tail
        const uint32_t x = n4 * 4 + threadIdx.x;
        const uint32_t y = up[x];
        out[x] = y < n ? lo[y] : CX_NONE;
    }
}

hipError_t fingers_pairs(const uint32_t *FT, size_t n, int nl, uint32_t *C2, hipStream_t s) {
    if (n == 0 || nl < 2) return hipSuccess;
    // planes start at multiples of n words: 16-B aligned rows need n % 4 == 0;
    // otherwise one lane per peer
    if (n % 4 != 0 || (uintptr_t)FT % 16 != 0 || (uintptr_t)C2 % 16 != 0) {
        k_fingers_pairs_1<<<dim3(cx_grid(n, 256, 4096), (unsigned)(nl - 1)), 256, 0, s>>>(
            FT, (uint32_t)n, nl, C2);
        return hipGetLastError();
    }
    k_fingers_pairs<<<dim3(cx_grid(n / 4, 256, 4096), (unsigned)(nl - 1)), 256, 0, s>>>(
        FT, (uint32_t)n, nl, C2);
    return hipGetLastError();
}

hipError_t fingers_levels(const uint32_t *F, size_t n, int L, int nl, uint32_t *FT,
                          hipStream_t s) {
    if (n == 0 || nl <= 0) return hipSuccess;
    if (L < 0 || L + nl > CX_FINGERS) return hipErrorInvalidValue;
    k_fingers_levels<<<(unsigned)((n + 63) / 64), 256, 0, s>>>(F, (uint32_t)n, L, nl, FT);
    return hipGetLastError();
}

// High words of the ring IDs, packed (8 B per peer instead of 16 at a 16-B
// stride): what the build's gap codes read.
__global__ void k_ring_hi(const cell128 *ring, uint32_t n, uint64_t *hi) {
    for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < n;
         p += (size_t)gridDim.x * blockDim.x)
        hi[p] = ring[p].hi;
}

hipError_t ring_hi(const cell128 *ring, size_t n, uint64_t *hi, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_ring_hi<<<cx_grid(n, 256), 256, 0, s>>>(ring, (uint32_t)n, hi);
    return hipGetLastError();
}

// cz_encode from the IDs' high words.  The gap code (xid - pid - 2^l) >> gs
// with gs >= 64 and l >= 64 is (D - c) >> (gs - 64), D = xhi - phi - 2^(l-64)
// (mod 2^64), c = the borrow out of the low words (0 or 1): when D has a set
// bit below gs - 64 the borrow cannot reach bit gs - 64, and D alone decides.
// Otherwise (about 2^-28 of encodes) the IDs' low words give c.
__device__ __forceinline__ uint32_t cz_encode_hi(uint32_t n, int gs, uint32_t par, uint64_t phi,
                                                 int l, uint32_t x, uint64_t xhi,
                                                 const cell128 *ring) {
    // x, par < n < 2^30 and E(l) <= n/2: x - par - E lies in (-3n/2, n).  The
    // stored advance is its residue in [h + 1 - n, h] (h = n / 2); when the raw
    // difference already lies there and in the 16-bit field's range -- every
    // slot but those whose hop wraps the ring's end -- it is the residue, else
    // two conditional adds and a subtract give it (no modulo)
    int d = (int)x - (int)par - (int)cz_expect(n, l);
    const int h = (int)(n / 2);
    const int lo = h + 1 - (int)n > -32768 ? h + 1 - (int)n : -32768;  // uniform
    const int hi = h < 32766 ? h : 32766;
    if ((uint32_t)(d - lo) > (uint32_t)(hi - lo)) {
        if (d < 0) d += (int)n;
        if (d < 0) d += (int)n;
        if (d > h) d -= (int)n;  // [h + 1 - n, h]
    }
    const int sh = gs - 64;
    const uint64_t D = xhi - phi - (1ull << (l - 64));
    uint64_t code;
    if (D & ((1ull << sh) - 1)) {
        code = D >> sh;
    } else {  // the borrow out of the low words decides: one more load each
        code = (D - (uint64_t)(ring[x].lo < ring[par].lo)) >> sh;
    }
    if (d < -32768 || d > 32766 || code >= 0xFFFF) return CZ_NONE;
    return ((uint32_t)code << 16) | (uint32_t)(d + 32768);
}

// cz_encode from 32-bit ID slices s(id) = bits [gs - 15, gs + 17) of id (the
// root-centric build's default input: half the bytes and registers of the high
// words).  D = s(x) - s(par) - s(2^l) (mod 2^32) is bits [gs - 15, gs + 17) of
// V = x - par - 2^l less a borrow c in {0, 1} from the bits below; when D has
// a set bit among its low 15 the borrow cannot reach bit 15 and D >> 15 is
// bits [gs, gs + 17) of V exactly (else, about 2^-15 of encodes, the full IDs
// are read).  V < 2^(gs + 17) holds because V is at most the gap ending at x,
// and the caller takes this path only when every ring gap is below 2^(gs + 17).
__device__ __forceinline__ uint32_t cz_encode_s(uint32_t n, int gs, uint32_t par, uint32_t sp,
                                                int l, uint32_t x, uint32_t sx,
                                                const cell128 *ring) {
    int d = (int)x - (int)par - (int)cz_expect(n, l);
    const int h = (int)(n / 2);
    const int lo = h + 1 - (int)n > -32768 ? h + 1 - (int)n : -32768;  // uniform
    const int hi = h < 32766 ? h : 32766;
    if ((uint32_t)(d - lo) > (uint32_t)(hi - lo)) {
        if (d < 0) d += (int)n;
        if (d < 0) d += (int)n;
        if (d > h) d -= (int)n;  // [h + 1 - n, h]
    }
    const int sb = l - (gs - 15);  // l >= gs - 15 on every table level
    const uint32_t D = sx - sp - (sb < 32 ? 1u << sb : 0u);
    uint64_t code;
    if (D & 0x7FFFu) {
        code = D >> 15;
    } else {  // the full IDs (64-bit halves: no variable 128-bit shifts)
        const cell128 cx = ring[x], cp = ring[par];
        code = (cx.hi - cp.hi - (1ull << (l - 64)) - (uint64_t)(cx.lo < cp.lo)) >> (gs - 64);
    }
    if (d < -32768 || d > 32766 || code >= 0xFFFF) return CZ_NONE;
    return ((uint32_t)code << 16) | (uint32_t)(d + 32768);
}

// s(id) = bits [gs - 15, gs + 17) of every ID; *wide (device, zeroed here) =
// 1 if some cyclic ring gap reaches 2^(gs + 17) (then the slice codes are not
// exact and the build keeps the high words).  Only such gaps write the flag.
__global__ void k_ring_codes(const cell128 *ring, uint32_t n, int gs, uint32_t *rs,
                             uint32_t *wide) {
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < n; p += gridDim.x * blockDim.x) {
        const u128 id = ld128(ring + p);
        rs[p] = (uint32_t)bits64(id, gs - 15);
        const u128 nx = ld128(ring + (p + 1 == n ? 0u : p + 1));
        if (n == 1 || msb128(nx - id) >= gs + 17) atomicOr(wide, 1u);
    }
}

hipError_t ring_codes(const cell128 *ring, size_t n, int ib, uint32_t *rs, uint32_t *wide,
                      hipStream_t s) {
    hipError_t e = hipMemsetAsync(wide, 0, sizeof(uint32_t), s);
    if (e != hipSuccess || n == 0) return e;
    k_ring_codes<<<cx_grid(n, 256), 256, 0, s>>>(ring, (uint32_t)n, cz_shift(ib), rs, wide);
    return hipGetLastError();
}

// Planes [lvl_base, lvl_base + nlev) of the table for the M peers p_first,
// p_first + 1, ... (cyclic): the whole table (lvl_base = l0, nlev = R,
// p_first = 0, M = n), or an arc rank's replicated top levels / local rows.
// One lane per entry; a wave's 64 lanes are 64 consecutive peers of one
// plane, whose fingers at a level are (nearly) consecutive peers too, so with
// fingers in level planes (fv) and the IDs' packed high words (rh) each
// gather instruction touches a few cache lines.  At 2^24 (2^30 entries):
// 129 ms from row-major fingers, 62 ms from level planes, 56 ms with one
// entry per lane in dispatch order (resident waves on a compact window of
// rows, XCD-aware), 54 ms with streaming stores (profiles/r02/cz_build/).
// The build is bound by its 5-deep dependent finger chain (SQ_WAIT_ANY 86 %
// of wave cycles, 29 GB fetched + 64 GiB written = 1.7 TB/s).  MODE 2 takes
// each consecutive level pair of a slot's path as one gather from two-hop
// planes (chain 5 -> 3 gathers): 53.5 -> 47.9 ms, + 1.7 ms to build the
// planes (profiles/r02/cz_build/kernel_stats_modes.csv).  6 or 8 waves
// per SIMD (forced, with spills) are slower (60 / 71 ms); storing each 16-B
// row as soon as its slots are known serialised the gathers behind the
// stores (95 ms); a quad of lanes per entry (four columns of the slot square)
// issued more, less coalesced gathers (97 ms).
// MODE 0: row-major fingers; 1: level planes; 2: level + two-hop planes.
// The 64-B entries leave through LDS as whole-line streaming stores.
template <int MODE>
__global__ __launch_bounds__(256) void k_cz_build(FingerView fv, const cell128 *ring,
                                                  const uint64_t *rh, uint32_t n, int lvl_base,
                                                  int nlev, uint32_t p_first, uint32_t M, int gs,
                                                  uint4 *cz, uint32_t *esc, uint32_t K) {
    __shared__ uint4 cz_stage[256 * 4];
    // K = 0: grid.y = plane (i - lvl_base) * 2 + b, x over the plane's rows
    // (plane after plane).  K > 0: 1-D grid in chunks of K row-blocks: every
    // plane of a chunk of rows is dispatched before the next chunk, so planes
    // whose gathers land near the same rows (the lower levels, small E(l))
    // share them in L2/MALL.
    uint32_t plane, lb;
    if (K == 0) {
        plane = blockIdx.y;
        const uint32_t per = gridDim.x >> 3;
        lb = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    } else {
        const uint32_t P = (uint32_t)nlev * 2, B = blockIdx.x;
        const uint32_t chunk = B / (K * P), rem = B - chunk * K * P;
        plane = rem / K;
        const uint32_t sub = rem - plane * K;  // XCD sub % 8 takes a contiguous run
        lb = chunk * K + (sub & 7) * (K >> 3) + (sub >> 3);
    }
    const int b = (int)(plane & 1);
    const int i = lvl_base + (int)(plane >> 1);
    // finger (x, l): level planes -> plane base (uniform) + x; rows -> x * 128 + l
    auto fat = [&](uint32_t x, int l) -> uint32_t {
        if (MODE != 0) return fv.F[(size_t)(l - fv.L) * fv.sl + x];
        return fv.F[(size_t)x * CX_FINGERS + l];
    };
    // one entry per lane, no grid stride: the dispatcher walks blocks in
    // order, so the resident waves hold a compact window of rows of one or two
    // planes and their gathers (16 windows near p + E(l) per plane) stay in
    // L2/MALL.  XCD-aware: hardware block b runs on XCD b % 8; it takes logical
    // block (b % 8) * per + b / 8, so each XCD's L2 serves one contiguous run.
    uint32_t bad = 0, oob = 0;
    const uint32_t j = lb * blockDim.x + threadIdx.x;
    uint32_t out[16];
    if (j < M) {
        // level-major: entry plane * M + j (the walk's entry index)
        uint64_t pw = (uint64_t)p_first + j;  // p_first < n, j < M <= n
        if (pw >= n) pw -= n;
        const uint32_t p = (uint32_t)pw;
        uint32_t node[8];
        uint64_t nh[8];
        const uint64_t ph = rh[p];
        if (MODE == 2) {
            // two-hop planes cut the dependent chain from 5 gathers to 3:
            // slot v's node = its levels' fingers in descending order, with
            // each consecutive pair (l, l-1) taken as one C2 gather
            auto c2 = [&](uint32_t x, int l) -> uint32_t {
                return fv.C2[(size_t)(l - fv.L - 1) * fv.sl + x];
            };
            auto chk = [&](uint32_t x) -> uint32_t {
                if (x >= n) {  // not a converged finger table: reported, never followed
                    oob = 1;
                    return 0u;
                }
                return x;
            };
            uint32_t nd[16], A = 0, a = p;
            int al = i;
            if (b) {  // slot 15 = A = f(p, i); the window hangs off A' = f(A, i-1) = C2(p, i)
                A = chk(fat(p, i));
                a = A;
                al = i - 1;
                nd[0] = chk(c2(p, i));
            } else {
                nd[0] = chk(fat(p, i));
            }
            // depth 2 (bit w <-> level i-2-w)
            nd[1] = chk(fat(nd[0], i - 2));
            nd[2] = chk(fat(nd[0], i - 3));
            nd[3] = chk(c2(nd[0], i - 2));
            nd[4] = chk(fat(nd[0], i - 4));
            nd[6] = chk(c2(nd[0], i - 3));
            nd[8] = chk(fat(nd[0], i - 5));
            nd[12] = chk(c2(nd[0], i - 4));
            // depth 3
            nd[5] = chk(fat(nd[1], i - 4));
            nd[7] = chk(fat(nd[3], i - 4));
            nd[9] = chk(fat(nd[1], i - 5));
            nd[10] = chk(fat(nd[2], i - 5));
            nd[11] = chk(fat(nd[3], i - 5));
            nd[13] = chk(c2(nd[1], i - 4));
            nd[14] = chk(c2(nd[2], i - 4));
            nd[15] = b ? A : chk(c2(nd[3], i - 4));
            uint64_t hv[16];
#pragma unroll
            for (int v = 0; v < 16; ++v) hv[v] = rh[nd[v]];
            const uint64_t ah = b ? hv[15] : ph;
            out[0] = cz_encode_hi(n, gs, a, ah, al, nd[0], hv[0], ring);
#pragma unroll
            for (int v = 1; v < 16; ++v) {
                const int hb = 31 - __builtin_clz((unsigned)v);
                const int pv = v & ~(1 << hb);
                out[v] = cz_encode_hi(n, gs, nd[pv], hv[pv], i - 2 - hb, nd[v], hv[v], ring);
            }
            if (b) out[15] = cz_encode_hi(n, gs, p, ph, i, A, hv[15], ring);
        } else {
        uint32_t a = p;
        uint64_t ah = ph;
        int al = i;
        if (b) {  // slot 15 = A = f(p, i); the window hangs off A' = f(A, i-1)
            uint32_t A = fat(p, i);
            if (A >= n) {
                A = 0;
                oob = 1;
            }
            const uint64_t Ah = rh[A];
            out[15] = cz_encode_hi(n, gs, p, ph, i, A, Ah, ring);
            a = A;
            ah = Ah;
            al = i - 1;
        }
        node[0] = fat(a, al);
        if (node[0] >= n) {
            node[0] = 0;
            oob = 1;
        }
        nh[0] = rh[node[0]];
        out[0] = cz_encode_hi(n, gs, a, ah, al, node[0], nh[0], ring);
#pragma unroll
        for (int v = 1; v < 16; ++v) {
            const int hb = 31 - __builtin_clz((unsigned)v);
            const int pv = v & ~(1 << hb);
            const int lv = i - 2 - hb;
            if (v == 15 && b) continue;  // slot 15 of a b = 1 entry is A (above)
            uint32_t x = fat(node[pv], lv);
            if (x >= n) {  // not a converged finger table: reported, never followed
                x = 0;
                oob = 1;
            }
            const uint64_t xh = rh[x];
            out[v] = cz_encode_hi(n, gs, node[pv], nh[pv], lv, x, xh, ring);
            if (v < 8) {
                node[v] = x;
                nh[v] = xh;
            }
        }
        }  // chained path
#pragma unroll
        for (int v = 0; v < 16; ++v) bad += out[v] == CZ_NONE;
    }
    {
        // the wave's 64 entries (4 KiB, contiguous: one plane, consecutive
        // rows) leave through LDS as 4 stores of 1 KiB each, so every store
        // instruction writes whole lines instead of 16 B of 64 lines
        const int lane = threadIdx.x & 63;
        uint4 *ws = cz_stage + (threadIdx.x >> 6) * 256;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            ws[lane * 4 + k] = make_uint4(out[4 * k], out[4 * k + 1], out[4 * k + 2], out[4 * k + 3]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t j0 = lb * blockDim.x + (threadIdx.x & ~63u);  // the wave's first row
        const size_t t0 = (size_t)plane * M + j0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = k * 64 + lane;  // 16-B chunk of the wave's 4 KiB
            if (j0 + (c >> 2) < M) {
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                const uint4 u = ws[c];
                const v4u w = {u.x, u.y, u.z, u.w};
                v4u *dst = reinterpret_cast<v4u *>(cz + t0 * 4) + c;
                __builtin_nontemporal_store(w, dst);
            }
        }
    }
    if (oob) atomicOr(esc + 1, 1u);
    if (bad) atomicAdd(esc, bad);
}

// Root-centric build (table_build 0, the default): of the two entries (p, i, 0)
// and (p, i, 1) only one word depends on p -- enc(A rel p) with A = f(p, i),
// slot 0 of the b = 0 entry and slot 15 of the b = 1 entry -- while the other
// fifteen words of each are a function of (A, i): W0(A, i) = the window below
// A over levels i-2..i-5 (slots 1..15), W1(A, i) = A' = f(A, i-1) relative to
// A (slot 0) and the window below A' (slots 1..14).  A block takes up to
// CZ2_RMAX consecutive rows of one level (both planes), sized per level (host:
// cz2_plan) so that their distinct roots come to ~90 % of its 256 lanes: the
// rows' roots are non-decreasing along the ring (f(., i) is monotone up to one
// wrap), so the block compacts them to their distinct values (~0.5-0.97 per
// row by level on a uniform ring), computes both windows once per distinct
// root, one lane each, and writes the rows' entries as coalesced 16-B chunks
// assembled from LDS (whole lines per store instruction).  The row phase runs
// two rows per lane.  A block whose rows have more than 256 distinct roots
// (rare on a uniform ring, frequent on a clustered one) writes the rows of
// its first 256 roots and appends the rest (< 256 rows, so < 256 roots) to an
// overflow list that a second launch of the same kernel finishes.  LDS stays
// under 20 KB: the windows' buffer also stages the rows' roots before the
// window phase, and each window's word 0 (slot 0 of the b = 0 entry is the
// row's own word) carries its root into the W1 phase, with the window's
// CZ_NONE count in the spare top bits.  Dispatch: chunks of CZ2_CHUNK rows x
// all levels, a level's blocks spread over the XCDs.
// Same table, bit for bit, as k_cz_build (route_table_hash, tests/test_gpu_parity.py).
constexpr int CZ2_RMAX = 464;
constexpr uint32_t CZ2_CHUNK = 4096;  // rows of a dispatch chunk (all levels)

// Blocks per level per chunk: level l's bucket is clamp(floor(l - gl) + 6, 0,
// 7) with gl = log2 of the ring's mean gap (gl256 = 256 gl, rounded); byte k
// of the 64-bit table nbt is the block count of bucket k.
__device__ __forceinline__ uint32_t cz2_nb(int l, int gl256, uint64_t nbt) {
    int k = ((l * 256 - gl256) >> 8) + 6;  // arithmetic shift: floor
    k = k < 0 ? 0 : (k > 7 ? 7 : k);
    return (uint32_t)(nbt >> (8 * k)) & 0xFFu;
}

// items == nullptr: the main launch (blocks from the plan); else block b
// takes overflow item b = {first row j, level | rows << 8}.  Either appends
// its own overflow to ovf.
// 66 VGPRs: 7 waves per SIMD (8 forced spills and measured slower,
// profiles/r04/build_modes/wpe_ab).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7)))
void k_cz_build_roots2(FingerView fv, const cell128 *ring, uint32_t n, int lvl_base, int nlev,
                       uint32_t p_first, uint32_t M, int gs, uint4 *cz, uint32_t *esc,
                       int gl256, uint64_t nbt, const uint2 *items, uint32_t *ovf_cnt,
                       uint2 *ovf, uint32_t cap) {
    auto ld32 = [](const uint32_t *base, uint32_t x) -> uint32_t {
        return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(base) + x * 4u);
    };
    auto hiw = [&](uint32_t x) -> uint32_t { return ld32(fv.rs, x); };
    auto enc = [&](uint32_t par, uint32_t hpar, int l, uint32_t x, uint32_t hx) -> uint32_t {
        return cz_encode_s(n, gs, par, hpar, l, x, hx, ring);
    };
    // win: 256 windows x 16 words (W0: the root, slots 1..15; W1: slots 0..14,
    // its CZ_NONE count); before the window phase its first 2 x CZ2_RMAX words
    // stage the rows' roots A and two-hop roots A1 (compacted in place to the
    // distinct roots)
    __shared__ uint32_t win[256 * 16];
    __shared__ uint32_t ra1[256];  // A1 of each window's root, kept for W1
    __shared__ uint32_t e0s[CZ2_RMAX];
    __shared__ uint16_t ridx[CZ2_RMAX];
    __shared__ uint32_t wcnt[8];
    __shared__ uint32_t sbad;    // CZ_NONE words written by the block (rare)
    __shared__ uint32_t anybad;  // some window of the block holds one
    uint32_t *stA = win, *stA1 = win + CZ2_RMAX;
    uint32_t j0, rows;
    int lvl;
    if (items) {
        const uint2 it = items[blockIdx.x];
        j0 = it.x;
        lvl = (int)(it.y & 0xFFu);
        rows = it.y >> 8;
    } else {
        // block -> (chunk, level, block of the level in the chunk); the level's
        // blocks are spread over the XCDs with adjacent rows on one XCD
        uint32_t TB = 0;
        for (int l = 0; l < nlev; ++l) TB += cz2_nb(lvl_base + l, gl256, nbt);
        const uint32_t chunk = blockIdx.x / TB;
        uint32_t rem = blockIdx.x - chunk * TB;
        lvl = 0;
        uint32_t nbl = cz2_nb(lvl_base, gl256, nbt);
        while (rem >= nbl) {
            rem -= nbl;
            ++lvl;
            nbl = cz2_nb(lvl_base + lvl, gl256, nbt);
        }
        const uint32_t xm = nbl >> 3, xr = nbl & 7, xx = rem & 7;
        const uint32_t lbl = xx * xm + (xx < xr ? xx : xr) + (rem >> 3);
        const uint32_t RB = (CZ2_CHUNK + nbl - 1) / nbl;
        const uint32_t c0 = lbl * RB;
        if (c0 >= CZ2_CHUNK) return;  // block-uniform
        j0 = chunk * CZ2_CHUNK + c0;
        if (j0 >= M) return;
        rows = CZ2_CHUNK - c0 < RB ? CZ2_CHUNK - c0 : RB;
        if (M - j0 < rows) rows = M - j0;
    }
    const int i = lvl_base + lvl;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    // plane gathers through the caches: round 4 made them non-temporal (0.7 %
    // faster then, profiles/r04/store_ab/nt_gathers); a round-5 ABBA of the
    // current build (profiles/r05/build_ab/) has cached ones ahead, 24.5-24.7
    // vs 26.8-27.2 ms per fingers + table build and 29.5 vs 35.2 GB fetched
    // (neighbouring roots share plane lines in L2)
    auto fat = [&](uint32_t x, int l) -> uint32_t {
        return ld32(fv.F + (size_t)(l - fv.L) * fv.sl, x);
    };
    auto c2 = [&](uint32_t x, int l) -> uint32_t {
        return ld32(fv.C2 + (size_t)(l - fv.L - 1) * fv.sl, x);
    };
    bool oob = false;
    auto chk = [&](uint32_t x) -> uint32_t {
        if (__builtin_amdgcn_ballot_w64(x >= n)) oob = true;
        return x < n ? x : 0u;
    };
    if (t == 0) {
        sbad = 0;
        anybad = 0;
    }
    // ---- rows (two per lane): roots, two-hop roots, the row's own word ----
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t r = (uint32_t)t + 256u * k;
        if (r < rows) {
            uint64_t pw = (uint64_t)p_first + j0 + r;
            if (pw >= n) pw -= n;
            const uint32_t p = (uint32_t)pw;
            const uint32_t A = chk(fat(p, i)), A1 = chk(c2(p, i));
            const uint32_t e0 = enc(p, hiw(p), i, A, hiw(A));
            e0s[r] = e0;  // slot 0 of (p, i, 0) and slot 15 of (p, i, 1)
            stA[r] = A;
            stA1[r] = A1;
        }
    }
    __syncthreads();
    // distinct roots in row order: ballot per (row half, wave), eight counts
    uint32_t A[2], A1[2];
    bool first[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t r = (uint32_t)t + 256u * k;
        const bool v = r < rows;
        A[k] = v ? stA[r] : 0u;
        A1[k] = v ? stA1[r] : 0u;
        first[k] = v && (r == 0 || stA[r - 1] != A[k]);
    }
    const uint64_t fm0 = __ballot(first[0]), fm1 = __ballot(first[1]);
    if (lane == 0) {
        wcnt[wv] = (uint32_t)__popcll(fm0);
        wcnt[4 + wv] = (uint32_t)__popcll(fm1);
    }
    __syncthreads();
    uint32_t nr = 0, b0 = 0, b1 = 0;
    for (int w = 0; w < 8; ++w) {
        const uint32_t c = wcnt[w];
        b0 += w < wv ? c : 0u;
        b1 += w < 4 + wv ? c : 0u;
        nr += c;
    }
    const uint32_t rk0 = b0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(fm0 >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)fm0, 0u));
    const uint32_t rk1 = b1 + __builtin_amdgcn_mbcnt_hi((uint32_t)(fm1 >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)fm1, 0u));
    __syncthreads();  // every lane has read its neighbour's root
    if (first[0]) {
        stA[rk0] = A[0];
        stA1[rk0] = A1[0];
    }
    if (first[1]) {
        stA[rk1] = A[1];
        stA1[rk1] = A1[1];
    }
    if ((uint32_t)t < rows) ridx[t] = (uint16_t)(rk0 + first[0] - 1);
    if ((uint32_t)t + 256u < rows) ridx[t + 256] = (uint16_t)(rk1 + first[1] - 1);
    __syncthreads();
    // more than cap (256; smaller only to test this path) roots: this block
    // writes the rows of its first cap roots (rows [0, rhi)), an overflow
    // launch the rest; rhi = the first row of root cap
    uint32_t rhi = rows;
    if (nr > cap) {  // block-uniform
        uint32_t lo = 0, hi = rows;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (ridx[mid] < cap) lo = mid + 1;
            else hi = mid;
        }
        rhi = lo;
        nr = cap;
        if (t == 0) ovf[atomicAdd(ovf_cnt, 1u)] = make_uint2(j0 + rhi, (uint32_t)lvl | (rows - rhi) << 8);
    }
    // the row's own word, for the rows this block writes (a deferred row is
    // counted by the overflow launch that writes it)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t r = (uint32_t)t + 256u * k;
        if (r < rhi && e0s[r] == CZ_NONE) atomicAdd(&sbad, 2u);
    }
    const bool wl = (uint32_t)t < nr;
    uint32_t R = 0, RA1 = 0;
    if (wl) {
        R = stA[t];
        RA1 = stA1[t];
    }
    __syncthreads();  // the staged roots are read before win is written
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const size_t tp0 = (size_t)(2 * lvl) * M + j0;
    uint32_t *wr = win + t * 16;
    // W0: the window below R (b = 0 entry, slots 1..15; nd[0] = R)
    if (wl) {
        ra1[t] = RA1;
        uint32_t wbad = 0;
        uint32_t nd[16], hv[16];
        nd[0] = R;
        {
            nd[1] = chk(fat(R, i - 2));
            nd[2] = chk(fat(R, i - 3));
            nd[3] = chk(c2(R, i - 2));
            nd[4] = chk(fat(R, i - 4));
            nd[6] = chk(c2(R, i - 3));
            nd[8] = chk(fat(R, i - 5));
            nd[12] = chk(c2(R, i - 4));
            nd[5] = chk(fat(nd[1], i - 4));
            nd[7] = chk(fat(nd[3], i - 4));
            nd[9] = chk(fat(nd[1], i - 5));
            nd[10] = chk(fat(nd[2], i - 5));
            nd[11] = chk(fat(nd[3], i - 5));
            nd[13] = chk(c2(nd[1], i - 4));
            nd[14] = chk(c2(nd[2], i - 4));
            nd[15] = chk(c2(nd[3], i - 4));
#pragma unroll
            for (int v = 0; v < 16; ++v) hv[v] = hiw(nd[v]);
        }
        // word 0 (slot 0 is the row's own word) carries the root into W1, with
        // the window's CZ_NONE count (rare) in its spare top bits (the high two
        // beside A1); the 16 words leave as four 16-B LDS writes (a lane's
        // window is 64 contiguous bytes: four b128 writes per lane instead of
        // sixteen b32 writes 64 B apart, which hit two banks per wave)
        uint4 *w4 = reinterpret_cast<uint4 *>(wr);
#pragma unroll
        for (int g = 0; g < 4; ++g) {  // four words at a time, written when done
            uint32_t ov[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int v = 4 * g + u;
                if (v == 0) {
                    ov[u] = R;
                    continue;
                }
                const int hb = 31 - __builtin_clz((unsigned)v);
                const int pv = v & ~(1 << hb);
                ov[u] = enc(nd[pv], hv[pv], i - 2 - hb, nd[v], hv[v]);
                wbad += ov[u] == CZ_NONE;
            }
            w4[g] = make_uint4(ov[0], ov[1], ov[2], ov[3]);
        }
        if (wbad) {  // rare: read back beside the root and A1
            wr[0] |= (wbad & 3u) << 30;
            ra1[t] |= (wbad >> 2) << 30;
            anybad = 1;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // every row carries its root's W0 words
        const uint32_t r = (uint32_t)t + 256u * k;
        if (anybad && r < rhi) {
            const uint32_t x = ridx[r];
            const uint32_t wb = (win[x * 16] >> 30) | (ra1[x] >> 30) << 2;
            if (wb) atomicAdd(&sbad, wb);
        }
    }
    // plane 0: rows [0, rhi) x 4 chunks of 16 B, whole lines per store
    auto plane0 = [&]() {
        for (uint32_t c = t; c < 4u * rhi; c += 256u) {
            const uint32_t e = c >> 2, qq = c & 3u;
            // one 16-B LDS read per chunk (the window's words sit at their
            // slots; a lane pair of entries covers 32 banks): slot 0 is the
            // row's own word
            uint4 u = *reinterpret_cast<const uint4 *>(win + ridx[e] * 16 + qq * 4);
            if (qq == 0) u.x = e0s[e];
            const v4u wv4 = {u.x, u.y, u.z, u.w};
            // write-back stores (faster than streaming ones here, profiles/r04/store_ab)
            reinterpret_cast<v4u *>(cz + (tp0 + e) * 4)[qq] = wv4;
        }
    };
    plane0();
    __syncthreads();  // plane 0 has read every W0 word
    // W1: A' = f(R, i - 1) relative to R (slot 0), the window below A' (1..14)
    if (wl) {
        uint32_t wbad = 0;
        uint32_t nd[15], hv[15];
        uint32_t hR;
        nd[0] = ra1[t] & 0x3FFFFFFFu;
        {
            hR = hiw(wr[0] & 0x3FFFFFFFu);  // the root itself is re-read below
            nd[1] = chk(fat(nd[0], i - 2));
            nd[2] = chk(fat(nd[0], i - 3));
            nd[3] = chk(c2(nd[0], i - 2));
            nd[4] = chk(fat(nd[0], i - 4));
            nd[6] = chk(c2(nd[0], i - 3));
            nd[8] = chk(fat(nd[0], i - 5));
            nd[12] = chk(c2(nd[0], i - 4));
            nd[5] = chk(fat(nd[1], i - 4));
            nd[7] = chk(fat(nd[3], i - 4));
            nd[9] = chk(fat(nd[1], i - 5));
            nd[10] = chk(fat(nd[2], i - 5));
            nd[11] = chk(fat(nd[3], i - 5));
            nd[13] = chk(c2(nd[1], i - 4));
            nd[14] = chk(c2(nd[2], i - 4));
#pragma unroll
            for (int v = 0; v < 15; ++v) hv[v] = hiw(nd[v]);
        }
        const uint32_t Rw = wr[0] & 0x3FFFFFFFu;
        uint4 *w4 = reinterpret_cast<uint4 *>(wr);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            uint32_t ov[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int v = 4 * g + u;
                if (v == 15) {
                    ov[u] = wbad;
                    continue;
                }
                if (v == 0) {
                    ov[u] = enc(Rw, hR, i - 1, nd[0], hv[0]);
                } else {
                    const int hb = 31 - __builtin_clz((unsigned)v);
                    const int pv = v & ~(1 << hb);
                    ov[u] = enc(nd[pv], hv[pv], i - 2 - hb, nd[v], hv[v]);
                }
                wbad += ov[u] == CZ_NONE;
            }
            w4[g] = make_uint4(ov[0], ov[1], ov[2], ov[3]);
        }
        if (wbad) anybad = 1;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // ... and its W1 words
        const uint32_t r = (uint32_t)t + 256u * k;
        if (anybad && r < rhi) {
            const uint32_t wb = win[ridx[r] * 16 + 15];
            if (wb) atomicAdd(&sbad, wb);
        }
    }
    // plane 1: word 15 = the row's own word
    for (uint32_t c = t; c < 4u * rhi; c += 256u) {
        const uint32_t e = c >> 2, qq = c & 3u;
        uint4 u = *reinterpret_cast<const uint4 *>(win + ridx[e] * 16 + qq * 4);
        if (qq == 3) u.w = e0s[e];  // slot 15 is the row's own word
        const v4u wv4 = {u.x, u.y, u.z, u.w};
        reinterpret_cast<v4u *>(cz + (tp0 + M + e) * 4)[qq] = wv4;
    }
    if (oob) atomicOr(esc + 1, 1u);
    __syncthreads();
    if (t == 0 && sbad) atomicAdd(esc, sbad);
}

// Block counts of k_cz_build_roots2 (cz2_nb): rows per block ~ 230 /
// (expected distinct-root fraction of the level), from the level's finger
// distance 2^i against the ring's mean gap 2^128 / n (uniform ring, by
// simulation: 0.94 at 2^-4 of the mean gap, 0.89 at 2^-3, 0.80 at 2^-2, 0.685
// at 2^-1, 0.57 at 1x, 0.51 at 2x, 0.50 from 4x up); a block with more than
// 256 roots computes them in batches, so the estimate only sizes the blocks.
static void cz2_plan(size_t n, int &gl256, uint64_t &nbt, double target = 230.0) {
    const double gl = 128.0 - log2((double)n);
    gl256 = (int)lround(gl * 256.0);
    // bucket k covers floor(l - gl) = k - 6 (k = 0: <= -6, k = 7: >= 1)
    static const double frac[8] = {0.97, 0.94, 0.89, 0.80, 0.685, 0.57, 0.51, 0.50};
    nbt = 0;
    for (int k = 0; k < 8; ++k) {
        uint32_t rb = (uint32_t)(target / frac[k]);
        const uint32_t rmin = target > 128.0 ? 256u : 128u;
        if (rb < rmin) rb = rmin;
        if (rb > (uint32_t)CZ2_RMAX) rb = CZ2_RMAX;
        uint32_t nb = (CZ2_CHUNK + rb - 1) / rb;
        while ((CZ2_CHUNK + nb - 1) / nb > (uint32_t)CZ2_RMAX) ++nb;
        nbt |= (uint64_t)nb << (8 * k);
    }
}

hipError_t cz_build(const FingerView &fv, const cell128 *ring, const uint64_t *rh, size_t n,
                    int l0, int R, int ib, uint64_t *cz, uint32_t *esc, hipStream_t s,
                    uint32_t *ws) {
    return cz_build_part(fv, ring, rh, n, l0, R, 0, (uint32_t)n, ib, cz, esc, s, ws);
}

// Blocks of the main k_cz_build_roots2 launch.
static uint64_t cz2_blocks(size_t n, int lvl_base, int nlev, uint32_t M, double target = 230.0) {
    int gl256;
    uint64_t nbt;
    cz2_plan(n, gl256, nbt, target);
    uint64_t TB = 0;
    for (int l = 0; l < nlev; ++l) {
        int k = (((lvl_base + l) * 256 - gl256) >> 8) + 6;
        k = k < 0 ? 0 : (k > 7 ? 7 : k);
        TB += (nbt >> (8 * k)) & 0xFF;
    }
    return ((uint64_t)M + CZ2_CHUNK - 1) / CZ2_CHUNK * TB;
}

// Overflow lists of the default build: two counters (+ padding), then two
// lists of one uint2 per block.
size_t cz_build_ws_words(size_t n, int lvl_base, int nlev, uint32_t M) {
    if (n == 0 || M == 0 || nlev <= 0) return 4;
    return 4 + 4 * (size_t)cz2_blocks(n, lvl_base, nlev, M);
}

// Roots per block of k_cz_build_roots2 before it defers rows to an overflow
// launch: 256 (one window per lane); tests lower it to exercise that path.
static std::atomic<uint32_t> g_cz2_cap{256};
uint32_t cz2_cap() { return g_cz2_cap.load(); }
void cz2_set_cap(uint32_t cap) { g_cz2_cap.store(cap >= 1 && cap <= 256 ? cap : 256); }

hipError_t cz_build_part(const FingerView &fv, const cell128 *ring, const uint64_t *rh, size_t n,
                         int lvl_base, int nlev, uint32_t p_first, uint32_t M, int ib,
                         uint64_t *cz, uint32_t *esc, hipStream_t s, uint32_t *ws) {
    if (M == 0 || nlev <= 0) return hipSuccess;
    if (lvl_base - 5 < fv.L || lvl_base + nlev > fv.L + fv.nl) return hipErrorInvalidValue;
    // the high-word gap codes need every level >= 64 and gs >= 64
    if (lvl_base - 5 < 64 || cz_shift(ib) < 65) return hipErrorInvalidValue;
    if (p_first >= n || M > n || nlev * 2 > 65535) return hipErrorInvalidValue;
    if (n >= (1u << 30)) return hipErrorInvalidValue;
    const bool planes = fv.sx == 1;
    if (!planes && (fv.sx != CX_FINGERS || fv.sl != 1 || fv.L != 0 || fv.C2))
        return hipErrorInvalidValue;
    if (planes && fv.sl != n) return hipErrorInvalidValue;
    uint4 *out = reinterpret_cast<uint4 *>(cz);
    const int gs = cz_shift(ib);
    if (planes && fv.C2 && fv.roots && fv.rs && ws) {
        // default: root-centric blocks sized by distinct roots (k_cz_build_roots2)
        int gl256;
        uint64_t nbt;
        cz2_plan(n, gl256, nbt);
        const uint64_t blocks = cz2_blocks(n, lvl_base, nlev, M);
        if (blocks >= (1ull << 31) || nlev > 255) return hipErrorInvalidValue;
        // two overflow lists (ping-pong), counters in ws[0], ws[1]
        uint2 *list[2] = {reinterpret_cast<uint2 *>(ws + 4),  // 16-B aligned
                          reinterpret_cast<uint2 *>(ws + 4) + blocks};
        hipError_t e = hipMemsetAsync(ws, 0, 2 * sizeof(uint32_t), s);
        if (e != hipSuccess) return e;
        const uint32_t cap = cz2_cap();
        auto launch = [&](unsigned grid, const uint2 *it, uint32_t *oc, uint2 *ov) {
            k_cz_build_roots2<<<grid, 256, 0, s>>>(fv, ring, (uint32_t)n, lvl_base, nlev, p_first, M,
                                                   gs, out, esc, gl256, nbt, it, oc, ov, cap);
        };
        launch((unsigned)blocks, nullptr, ws, list[0]);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        // blocks with more than cap distinct roots left their last rows on a
        // list: one block per item takes them (with cap = 256 an item has
        // < 256 rows and finishes; every round shrinks each item by >= cap rows)
        for (int round = 0;; ++round) {
            uint32_t cnt = 0;
            if ((e = hipMemcpyAsync(&cnt, ws + (round & 1), sizeof(cnt), hipMemcpyDeviceToHost,
                                    s)) != hipSuccess ||
                (e = hipStreamSynchronize(s)) != hipSuccess)
                return e;
            if (cnt == 0) break;
            if (cnt > blocks || round >= CZ2_RMAX) return hipErrorInvalidValue;
            uint32_t *next = ws + ((round + 1) & 1);
            if ((e = hipMemsetAsync(next, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
            launch(cnt, list[round & 1], next, list[(round + 1) & 1]);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        return hipSuccess;
    }
    // one lane per entry (rings with a gap too wide for the 32-bit slices, or
    // no HBM for the two-hop planes / level planes): 1-D grid in chunks of 16
    // row-blocks x all planes, whole-line streaming stores through LDS
    // (37.6 ms at 2^24 with two-hop planes)
    constexpr uint32_t K = 16;
    const uint64_t nrb = ((uint64_t)M + 255) / 256, chunks = (nrb + K - 1) / K;
    const uint64_t blocks = chunks * K * (uint64_t)nlev * 2;
    if (blocks >= (1ull << 31)) return hipErrorInvalidValue;
    const dim3 grid((unsigned)blocks, 1);
    if (planes && fv.C2)
        k_cz_build<2><<<grid, 256, 0, s>>>(fv, ring, rh, (uint32_t)n, lvl_base, nlev, p_first, M,
                                           gs, out, esc, K);
    else if (planes)
        k_cz_build<1><<<grid, 256, 0, s>>>(fv, ring, rh, (uint32_t)n, lvl_base, nlev, p_first, M,
                                           gs, out, esc, K);
    else
        k_cz_build<0><<<grid, 256, 0, s>>>(fv, ring, rh, (uint32_t)n, lvl_base, nlev, p_first, M,
                                           gs, out, esc, K);
    return hipGetLastError();
}

// Order-sensitive hash of a table (A/B identity of two builds): sum over words
// of splitmix(w ^ golden * (index + 1)), wrapping.
__global__ void k_table_hash(const uint64_t *t, size_t words, unsigned long long *out) {
    uint64_t acc = 0;
    for (size_t k = blockIdx.x * (size_t)blockDim.x + threadIdx.x; k < words;
         k += (size_t)gridDim.x * blockDim.x) {
        uint64_t z = t[k] ^ (0x9E3779B97F4A7C15ull * (k + 1));
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        acc += z ^ (z >> 31);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

hipError_t table_hash(const void *t, size_t bytes, unsigned long long *out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(*out), s);
    if (e != hipSuccess || bytes < 8) return e;
    k_table_hash<<<cx_grid(bytes / 8, 256), 256, 0, s>>>(static_cast<const uint64_t *>(t),
                                                         bytes / 8, out);
    return hipGetLastError();
}

// The cz walk runs in units of u = 2^gs: d = key - id_cur lies in
// [dmin * u, dmax * u + u - 1] (two u64).  Every threshold it is compared with
// (2^l, 2^l + gap) is a multiple of u up to the gap's sub-unit part, so a hop
// is exact integer arithmetic on (dmin, dmax): with e = 2^(l-gs) + code,
//   StoredLocally(nxt) holds     if dmax <  e,
//   fails (d' = d - 2^l - gap)   if dmin >  e  ->  [dmin - e - 1, dmax - e],
//   is undecided otherwise (A_FIXT: exact IDs of cur and nxt).
// The level is gs + msb(dmin) when msb(dmin) == msb(dmax); otherwise, or
// when d < u, the walk needs cur's exact ID (cex: clo = id_cur).
__device__ __forceinline__ void cz_exact_d(const PkCtx &c, u128 key, u128 idc, uint64_t &dmin,
                                           uint64_t &dmax) {
    dmin = dmax = bits64(key - idc, c.gs);
}

// Exact hop from cur at level i through the finger table (below the table,
// or a root the entry cannot represent); needs clo = id_cur (cex).
// 1 = finished (own/st set), 0 = moved (cur, clo exact, dmin/dmax).
__device__ __forceinline__ int cz_exact(const PkCtx &c, u128 key, u128 &clo, uint64_t &dmin,
                                        uint64_t &dmax, uint32_t &cur, uint32_t &h, int i,
                                        uint32_t &own, uint8_t &st, uint32_t *xc = nullptr,
                                        bool nh_ok = false, u128 nh = 0) {
    if (xc) ++*xc;  // counter build only: one F gather + one ring gather
    uint32_t nxt;
    u128 idn;
    if (nh_ok) {
        // nh = id(cur + 1) from the memory round (A_EXACT): the finger is the
        // next peer unless the gap to it is below 2^i (then the directory)
        const uint32_t nx = cur + 1 == c.n ? 0u : cur + 1;
        const u128 step = pow2_128(i);
        if (c.n == 1) {
            nxt = 0;
            idn = clo;
        } else if (step <= nh - clo) {
            nxt = nx;
            idn = nh;
        } else {
            nxt = (c.arc || !c.F) ? dir_successor(c.sv, clo + step)
                                  : c.F[(size_t)cur * CX_FINGERS + i];
            idn = ld128(c.ring + nxt);
        }
    } else {
        // arc mode, or a ring whose row-major finger table is not materialised
        // (cx_fingers_build defers it: the cz walk reads it only here): the
        // finger from the ring (next peer) or the directory
        nxt = (c.arc || !c.F) ? finger_of(c.sv, c.ring, c.n, cur, i, clo)
                              : c.F[(size_t)cur * CX_FINGERS + i];
        idn = ld128(c.ring + nxt);
    }
    ++h;
    if (key - clo <= idn - clo) {
        own = nxt;
        return 1;
    }
    if (h == CX_HOP_CAP) {
        own = CX_NONE;
        st = CX_Q_HOPCAP;
        return 1;
    }
    cur = nxt;
    clo = idn;
    cz_exact_d(c, key, idn, dmin, dmax);
    return 0;
}

// One relative hop through node word wd at level i.  1 = finished, -1 =
// undecided (A_FIXT), 0 = moved.
__device__ __forceinline__ int cz_hop(const PkCtx &c, uint32_t wd, int i, uint64_t &dmin,
                                      uint64_t &dmax, uint32_t &cur, uint32_t &h, uint32_t &pn,
                                      uint32_t &own, uint8_t &st) {
    const uint64_t e = (1ull << (i - c.gs)) + (wd >> 16);
    const uint32_t nxt = cz_next(c.n, cur, i, wd);
    ++h;
    if (dmax < e) {
        own = nxt;
        return 1;
    }
    if (dmin <= e) {
        pn = nxt;
        return -1;
    }
    if (h == CX_HOP_CAP) {
        own = CX_NONE;
        st = CX_Q_HOPCAP;
        return 1;
    }
    cur = nxt;
    dmin -= e + 1;
    dmax -= e;
    return 0;
}

// Plan from cur using the lane's LDS entry (16 nodes) for free hops.  cs = the
// window subset we stand on (-1: none, 16: the root A of a b = 1 entry), ri =
// the entry's level.  Returns 0 = needs a load (mode set), 1 = finished.
__device__ __forceinline__ int cz_plan(const PkCtx &c, u128 key, u128 &clo, bool &cex,
                                       uint64_t &dmin, uint64_t &dmax, uint32_t &cur,
                                       uint32_t &h, uint32_t &pn, int &mode, int &lvl, int &rb,
                                       int &cs, int ri, const uint32_t *ent, uint32_t &own,
                                       uint8_t &st, uint32_t *xc = nullptr,
                                       bool nh_ok = false, u128 nh = 0) {
    for (;;) {
        int i;
        const int ma = 63 - __builtin_clzll(dmin | 1), mb = 63 - __builtin_clzll(dmax | 1);
        if (dmin != 0 && ma == mb) {
            i = ma + c.gs;
        } else if (!cex) {
            mode = A_FIXC;
            return 0;
        } else {
            i = msb128(key - clo);  // d < 2^gs, exact
        }
        const int o = ri - i;
        int v = -1;
        if (cs == 16) {
            if (o == 1) v = 0;
        } else if (cs >= 0 && o >= 2 && o <= 5) {
            v = cs | (1 << (o - 2));
            if (rb && v == 15) v = -1;
        }
        const uint32_t wd = v >= 0 ? ent[v] : CZ_NONE;
        if (wd != CZ_NONE) {
            const int t = cz_hop(c, wd, i, dmin, dmax, cur, h, pn, own, st);
            if (t > 0) return 1;
            if (t < 0) {
                mode = A_FIXT;
                return 0;
            }
            cs = v;
            cex = false;
            continue;
        }
        cs = -1;
        if (i >= c.l0) {
            // arc mode: a row below the replicated levels that this rank does
            // not hold -> the lookup continues on the rank of its key's arc
            if (c.arc && i < c.Lh && !arc_row_local(c, cur)) return 2;
            mode = A_HOP;
            lvl = i;
            rb = (int)((dmax >> (i - 1 - c.gs)) & 1);  // bit i-1 of d - 2^i
            return 0;
        }
        // below the table: the exact hop takes id(cur) and id(cur + 1) from one
        // memory round (A_EXACT; nh = id(cur + 1) once they are in)
        if (!cex || !nh_ok) {
            mode = A_EXACT;
            return 0;
        }
        if (cz_exact(c, key, clo, dmin, dmax, cur, h, i, own, st, xc, true, nh)) return 1;
        nh_ok = false;  // cur moved: the hint is stale
    }
}

// Arguments of the tree walk (replicated ring: lo = 0, hi = n; arc mode: the
// rank's arc, inputs and outcomes as 32-B ArcRec records).
struct TreeIO {
    const cell128 *ring_ext, *ring;
    uint32_t n;
    const uint4 *tree;
    int l0, R, ib;
    const uint32_t *F;
    int Lh;              // arc mode: first replicated level
    uint32_t plo, M;     // arc mode: local rows (cyclic peer range)
    SearchView sv;       // arc mode: directory of the replicated ring
    const uint32_t *src;
    const cell128 *keys;
    const ArcRec *in;
    ArcRec *out;
    int self;
    size_t q, chunk;
    uint32_t *owner;
    uint8_t *hops;
    uint8_t *status;
};

// Instantiations: <false, false> the lookahead-tree walk (rings above 2^24
// peers), <true, true> the record protocol's arc walk (chordx.arc "records";
// the default key-first arc walk is k_walk<false, true>, cx_walk.hip).
template <bool ARC, bool CZ>
__global__ __launch_bounds__(RT_BLOCK) __attribute__((amdgpu_waves_per_eu(CZ ? CZ_WAVES : 1)))
void k_route_tree(TreeIO io) {
    constexpr int RW = CZ ? CZ_RES_WIN : RES_WIN;  // cz: smaller window, more waves per CU
    static_assert(!ARC || CZ, "arc mode walks pattern-keyed (cz) rows");
    constexpr bool RIO = !ARC;  // results staged per wave, written in input order
    __shared__ uint64_t res_all[RIO ? RT_BLOCK / 64 : 1][RIO ? RW : 1];
    __shared__ uint4 ent_all[RT_BLOCK][4];       // each lane's current 64-B entry
    __shared__ uint64_t addr_all[RT_BLOCK];      // entry index + 1 wanted by each lane (0: none)
    const uint32_t n = io.n;
    const int l0 = io.l0, R = io.R, ib = io.ib;
    const int lane = threadIdx.x & 63;
    const int quad0 = threadIdx.x & ~3, qs = threadIdx.x & 3;
    uint64_t *res = res_all[RIO ? (threadIdx.x >> 6) : 0];
    const uint64_t *ent = reinterpret_cast<const uint64_t *>(ent_all[threadIdx.x]);
    const uint32_t *ent32 = reinterpret_cast<const uint32_t *>(ent_all[threadIdx.x]);
    if (RIO)
        for (int j = lane; j < RW; j += 64) res[j] = 0;
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
    const size_t base = wave * io.chunk;
    if (base >= io.q) return;  // wave-uniform
    const size_t end = (base + io.chunk < io.q) ? base + io.chunk : io.q;
    PkCtx c;
    c.ring = io.ring;
    c.F = io.F;
    c.n = n;
    c.l0 = l0;
    c.ib = ib;
    c.S = 64 + ib;
    c.imask = (1ull << ib) - 1;
    c.W = (pow2_128(c.S)) - 1;
    c.gs = cz_shift(ib);
    c.arc = ARC;
    c.Lh = io.Lh;
    c.plo = io.plo;
    c.M = io.M;
    c.sv = io.sv;
    size_t head = base, flushed = base;

    int mode = A_NONE, lvl = 0, cs = -1, ri = 0;
    size_t qi = 0;
    uint64_t qid = 0;
    u128 key = 0, clo = 0;
    bool cex = true;          // id(cur) = clo exactly (tree: else in [clo, clo + W])
    uint64_t dmin = 0, dmax = 0;  // cz: d = key - id(cur) in units of 2^gs
    int rb = 0;               // cz: pattern bit of the wanted entry
    uint32_t cur = 0, h = 0, pn = 0;
    int bst = B_EMPTY, pkind = 0;
    size_t pq = 0;
    uint64_t pqid = 0;
    u128 pkey = 0, pa = 0, pb = 0;
    uint32_t psrc = 0, ph = 0;
    uint32_t *xcp = nullptr;

    // outcome of a finished query (ARC: local delivery or a result record)
    auto deliver = [&](size_t idx, uint64_t id, uint32_t o, uint32_t hh, uint8_t stt) {
        if (RIO) {
            res[idx & (RW - 1)] = pack_res(o, hh, stt);
        } else {
            ArcRec r;
            if ((int)(id >> ARC_ORIGIN_SHIFT) == io.self) {
                const size_t li = id & ARC_INDEX_MASK;
                io.owner[li] = o;
                io.hops[li] = (uint8_t)hh;
                if (io.status) io.status[li] = stt;
                r.w0 = r.w1 = 0;
                r.qid = id;
                r.cur = 0;
                r.hk = ARC_NONE << 8;
            } else {
                r.w0 = (uint64_t)o | ((uint64_t)stt << 32);
                r.w1 = 0;
                r.qid = id;
                r.cur = o;
                r.hk = (hh & 0xFF) | (ARC_RESULT << 8);
            }
            io.out[idx] = r;
        }
    };

    for (;;) {
        // ---- refill slot B ----
        {
            size_t lim = end;
            if (RIO && flushed + RW < end) lim = flushed + RW;
            const size_t avail = lim > head ? lim - head : 0;
            const uint64_t want = __ballot(bst == B_EMPTY);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(want >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)want, 0u));
            if (bst == B_EMPTY && rank < avail) {
                pq = head + rank;
                if (ARC && io.in) {
                    const ArcRec r = io.in[pq];
                    pkey = ((u128)r.w1 << 64) | r.w0;
                    pqid = r.qid;
                    psrc = r.cur;
                    ph = r.hk & 0xFF;
                    pkind = (int)(r.hk >> 8);
                } else {  // a new lookup (arc mode: issued on this rank)
                    pkey = ld128(io.keys + pq);
                    psrc = io.src[pq];
                    pqid = ARC ? ((uint64_t)io.self << ARC_ORIGIN_SHIFT) | pq : pq;
                    ph = 0;
                    pkind = ARC_NEW;
                }
                bst = B_KS;
            }
            const size_t took = (size_t)__popcll(want);
            head += took < avail ? took : avail;
        }
        if (__ballot(mode != A_NONE || bst != B_EMPTY) == 0 && head >= end &&
            (!RIO || flushed >= end))  // every staged result written
            break;

        // ---- memory round ----
        {
            // v4 rows are peer-major ([peer][level]); the cz table is level-major
            // ([level][b][peer]): a wave's first hops leave ~64 consecutive
            // source peers, mostly at the top level or two, so their entries
            // share DRAM pages and 128-B lines instead of lying 4 KiB apart.
            uint64_t e;
            if (!CZ) {
                e = (uint64_t)cur * (unsigned)R + (unsigned)(lvl - l0);
            } else if (!ARC) {
                e = (uint64_t)((lvl - l0) * 2 + rb) * n + cur;
            } else if (lvl >= io.Lh) {  // replicated top planes, all peers
                e = (uint64_t)((lvl - io.Lh) * 2 + rb) * n + cur;
            } else {  // this rank's rows (arc + halo), after the top planes
                const uint32_t j = cur >= io.plo ? cur - io.plo : cur + n - io.plo;
                e = (uint64_t)(CX_FINGERS - io.Lh) * 2 * n +
                    (uint64_t)((lvl - l0) * 2 + rb) * io.M + j;
            }
            addr_all[threadIdx.x] = mode == A_HOP ? e + 1 : 0;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t a0 = addr_all[quad0], a1 = addr_all[quad0 + 1], a2 = addr_all[quad0 + 2],
                       a3 = addr_all[quad0 + 3];
        uint4 c0 = make_uint4(0, 0, 0, 0), c1 = c0, c2 = c0, c3 = c0;
        // non-temporal: a table entry is rarely read twice before it leaves L2
        // (1.4 % faster per launch than ordinary loads, profiles/r04/ntload_ab)
        typedef unsigned int v4n __attribute__((ext_vector_type(4)));
        auto ld_entry = [&](uint64_t a) -> uint4 {
            const v4n v = __builtin_nontemporal_load(reinterpret_cast<const v4n *>(io.tree) +
                                                     (a - 1) * 4 + qs);
            return make_uint4(v.x, v.y, v.z, v.w);
        };
        if (a0) c0 = ld_entry(a0);
        if (a1) c1 = ld_entry(a1);
        if (a2) c2 = ld_entry(a2);
        if (a3) c3 = ld_entry(a3);
        u128 xa = 0, xb = 0;
        if (mode == A_FIXC) {
            xa = ld128(io.ring + cur);
        } else if (mode == A_FIXT) {
            xa = ld128(io.ring + cur);
            xb = ld128(io.ring + pn);
        } else if (mode == A_EXACT) {  // (cur, cur + 1): adjacent cells
            xa = ld128(io.ring + cur);
            xb = ld128(io.ring + (cur + 1 == n ? 0u : cur + 1));
        }
        if (bst == B_KS) {
            if (pkind != ARC_RESULT && pkind != ARC_NONE && psrc < n) {
                // non-temporal (0.5 %, profiles/r04/ntload_ab/source_pair)
                if (pkind == ARC_NEW) pa = ld128_nt(io.ring_ext + psrc);  // pred: local check only
                pb = ld128_nt(io.ring_ext + psrc + 1);
            }
            bst = B_PAIR;
        }
        if (a0) ent_all[quad0][qs] = c0;
        if (a1) ent_all[quad0 + 1][qs] = c1;
        if (a2) ent_all[quad0 + 2][qs] = c2;
        if (a3) ent_all[quad0 + 3][qs] = c3;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // ---- compute slot A ----
        bool fin = false, plan = false;
        uint32_t own = CX_NONE;
        uint8_t st = CX_Q_OK;
        if (mode == A_HOP && CZ) {
            // root of entry (cur, lvl, rb): A = finger(cur, lvl)
            const uint32_t wd = ent32[rb ? 15 : 0];
            ri = lvl;
            if (wd != CZ_NONE) {
                const int t = cz_hop(c, wd, lvl, dmin, dmax, cur, h, pn, own, st);
                if (t > 0) {
                    fin = true;
                } else if (t < 0) {
                    mode = A_FIXT;
                } else {
                    cex = false;
                    cs = rb ? 16 : 0;
                    plan = true;
                }
            } else {
                cs = -1;
                if (!cex) {  // rare: exact id of cur for the exact hop
                    clo = ld128(io.ring + cur);
                    cex = true;
                }
                if (cz_exact(c, key, clo, dmin, dmax, cur, h, lvl, own, st, xcp))
                    fin = true;
                else
                    plan = true;
            }
        } else if (mode == A_HOP) {
            const uint64_t m0 = ent[0];
            ri = lvl;
            cs = 0;
            const uint32_t nxt = (uint32_t)(m0 & c.imask);
            const u128 nlo = shl128((u128)(m0 >> ib), c.S);
            ++h;
            const int t = term_iv(key, clo, cex ? (u128)0 : c.W, nlo, c.W);
            if (t == 1) {
                fin = true;
                own = nxt;
            } else if (t < 0) {
                mode = A_FIXT;
                pn = nxt;
            } else if (h == CX_HOP_CAP) {
                fin = true;
                st = CX_Q_HOPCAP;
            } else {
                cur = nxt;
                clo = nlo;
                cex = false;
                plan = true;
            }
        } else if (mode == A_FIXC || mode == A_EXACT) {
            clo = xa;
            cex = true;
            if (CZ) cz_exact_d(c, key, xa, dmin, dmax);
            plan = true;
        } else if (mode == A_FIXT) {
            if (key - xa <= xb - xa) {
                fin = true;
                own = pn;
            } else if (h == CX_HOP_CAP) {
                fin = true;
                st = CX_Q_HOPCAP;
            } else {
                cur = pn;
                clo = xb;
                cex = true;
                if (CZ) cz_exact_d(c, key, xb, dmin, dmax);
                plan = true;
            }
        }
        if (plan) {
            const int r =
                CZ ? cz_plan(c, key, clo, cex, dmin, dmax, cur, h, pn, mode, lvl, rb, cs, ri, ent32,
                             own, st, xcp, mode == A_EXACT, xb)
                   : tree_plan(c, key, clo, cex, cur, h, pn, mode, lvl, cs, ri, ent, own, st);
            if (r == 1) fin = true;
            if (ARC && r == 2) {  // continue on the rank of the key's arc
                ArcRec o;
                o.w0 = (uint64_t)key;
                o.w1 = (uint64_t)(key >> 64);
                o.qid = qid;
                o.cur = cur;
                o.hk = (h & 0xFF) | (ARC_WALK << 8);
                io.out[qi] = o;
                mode = A_NONE;
            }
        }
        if (fin) {
            deliver(qi, qid, own, h, st);
            mode = A_NONE;
        }
        // ---- promote slot B ----
        if (mode == A_NONE && bst == B_PAIR) {
            bst = B_EMPTY;
            qi = pq;
            qid = pqid;
            key = pkey;
            cur = psrc;
            h = ph;
            cs = -1;
            own = CX_NONE;
            st = CX_Q_OK;
            int done = 1;
            if (ARC && pkind == ARC_RESULT) {
                // a result coming home: deliver it (w0 = owner | status << 32)
                deliver(qi, qid, (uint32_t)pkey, h, (uint8_t)((uint64_t)pkey >> 32));
                done = 0;
            } else if (ARC && pkind == ARC_NONE) {
                ArcRec o = {};
                o.qid = qid;
                o.hk = ARC_NONE << 8;
                io.out[qi] = o;
                done = 0;
            } else if (cur >= n) {
                st = CX_Q_BADPEER;
            } else if (pkind == ARC_NEW && (n == 1 || (key - pa - 1) <= (pb - pa - 1))) {
                own = cur;  // StoredLocally at the source: 0 hops
            } else {
                clo = pb;
                cex = true;
                if (CZ) cz_exact_d(c, key, pb, dmin, dmax);
                done = CZ ? cz_plan(c, key, clo, cex, dmin, dmax, cur, h, pn, mode, lvl, rb, cs,
                                    ri, ent32, own, st, xcp)
                          : tree_plan(c, key, clo, cex, cur, h, pn, mode, lvl, cs, ri, ent, own,
                                      st);
                if (ARC && done == 2) {
                    ArcRec o;
                    o.w0 = (uint64_t)key;
                    o.w1 = (uint64_t)(key >> 64);
                    o.qid = qid;
                    o.cur = cur;
                    o.hk = (h & 0xFF) | (ARC_WALK << 8);
                    io.out[qi] = o;
                    mode = A_NONE;
                    done = 0;
                }
            }
            if (done == 1) {
                deliver(qi, qid, own, h, st);
                mode = A_NONE;
            }
        }

        // ---- flush complete 64-result segments (replicated mode) ----
        if (RIO) {
            for (int it = 0; it < 2; ++it) {
                if (flushed >= end) break;
                const size_t idx = flushed + lane;
                const bool inr = idx < end;
                const uint64_t v = inr ? res[idx & (RW - 1)] : 0ull;
                if (__ballot(!inr || (v >> 63)) != ~0ull) break;
                if (inr) {
                    io.owner[idx] = (uint32_t)v;
                    io.hops[idx] = (uint8_t)(v >> 32);
                    if (io.status) io.status[idx] = (uint8_t)(v >> 40);
                    res[idx & (RW - 1)] = 0;
                }
                flushed += 64;
            }
        }
    }
}

static void tree_geometry(size_t q, size_t &chunk, unsigned &blocks) {
    const size_t max_waves = 256 * 32;
    // >= 64 lookups per wave: a small batch spread over as many waves as it
    // fills (a walk is a chain of dependent gathers; cx_walk.hip WK_MIN_PER_WAVE)
    size_t waves = (q + 63) / 64;
    if (waves > max_waves) waves = max_waves;
    if (waves == 0) waves = 1;
    chunk = (q + waves - 1) / waves;
    waves = (q + chunk - 1) / chunk;
    blocks = (unsigned)((waves * 64 + RT_BLOCK - 1) / RT_BLOCK);
}

hipError_t route_tree(const cell128 *ring_ext, const cell128 *ring, size_t n,
                      const uint64_t *tree, int l0, int R, int ib, const uint32_t *F,
                      const uint32_t *src, const cell128 *keys, size_t q, uint32_t *owner,
                      uint8_t *hops, uint8_t *status, hipStream_t s) {
    if (q == 0) return hipSuccess;
    TreeIO io = {};
    io.ring_ext = ring_ext;
    io.ring = ring;
    io.n = (uint32_t)n;
    io.tree = reinterpret_cast<const uint4 *>(tree);
    io.l0 = l0;
    io.R = R;
    io.ib = ib;
    io.F = F;
    io.src = src;
    io.keys = keys;
    io.q = q;
    io.owner = owner;
    io.hops = hops;
    io.status = status;
    unsigned blocks;
    tree_geometry(q, io.chunk, blocks);
    k_route_tree<false, false><<<blocks, RT_BLOCK, 0, s>>>(io);
    return hipGetLastError();
}

template <class K>
static unsigned resident_grid(K kernel, int block);

// ---------------------------------------------------------------------------
// Arc-sharded mode (SURVEY 8e layout 2), two phases per lookup.  Every rank
// holds the replicated ring, the pattern-keyed (cz) planes of the top levels
// [Lh, 128) for all peers, and the planes below Lh only for its arc of peers
// plus a halo: the peers whose IDs lie within 2^Lh before the arc's first
// peer.  Phase 1 walks on the origin rank while the rows it needs are
// replicated; once the walk needs a level below Lh, d = key - id_cur < 2^Lh,
// so cur and every later peer lie in (key - 2^Lh, key]: inside the arc of the
// key's owner plus its halo.  The lookup travels there once (a WALK record)
// and finishes; results travel home once (RESULT records).
// ---------------------------------------------------------------------------
hipError_t route_arc(const cell128 *ring_ext, const cell128 *ring, size_t n, const uint64_t *cz,
                     int l0, int R, int ib, const SearchView &sv, int Lh, uint32_t plo, uint32_t M,
                     int self, const ArcRec *in, const uint32_t *src, const cell128 *keys, size_t q,
                     ArcRec *out, uint32_t *owner, uint8_t *hops, uint8_t *status, hipStream_t s) {
    if (q == 0) return hipSuccess;
    TreeIO io = {};
    io.src = src;  // in == nullptr: new lookups read straight from src / keys
    io.keys = keys;
    io.ring_ext = ring_ext;
    io.ring = ring;
    io.n = (uint32_t)n;
    io.tree = reinterpret_cast<const uint4 *>(cz);
    io.l0 = l0;
    io.R = R;
    io.ib = ib;
    io.sv = sv;
    io.Lh = Lh;
    io.plo = plo;
    io.M = M;
    io.in = in;
    io.out = out;
    io.self = self;
    io.q = q;
    io.owner = owner;
    io.hops = hops;
    io.status = status;
    static const unsigned resident = resident_grid(k_route_tree<true, true>, RT_BLOCK);
    size_t waves = (size_t)resident * (RT_BLOCK / 64);
    const size_t small = (q + 63) / 64;  // >= 64 lookups per wave (tree_geometry)
    if (small < waves) waves = small ? small : 1;
    io.chunk = (q + waves - 1) / waves;
    waves = (q + io.chunk - 1) / io.chunk;
    const unsigned blocks = (unsigned)((waves * 64 + RT_BLOCK - 1) / RT_BLOCK);
    k_route_tree<true, true><<<blocks, RT_BLOCK, 0, s>>>(io);
    return hipGetLastError();
}

// Initial records: query i issued at peer src[i] (kind NEW, qid = self:i).
__global__ void k_arc_seed(const uint32_t *src, const cell128 *keys, size_t q, int self,
                           ArcRec *out) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < q;
         i += (size_t)gridDim.x * blockDim.x) {
        const u128 k = ld128(keys + i);
        ArcRec r;
        r.w0 = (uint64_t)k;
        r.w1 = (uint64_t)(k >> 64);
        r.qid = ((uint64_t)self << ARC_ORIGIN_SHIFT) | i;
        r.cur = src[i];
        r.hk = ARC_NEW << 8;
        out[i] = r;
    }
}

hipError_t arc_seed(const uint32_t *src, const cell128 *keys, size_t q, int self, ArcRec *out,
                    hipStream_t s) {
    if (q == 0) return hipSuccess;
    k_arc_seed<<<cx_grid(q, 256), 256, 0, s>>>(src, keys, q, self, out);
    return hipGetLastError();
}

// Destination rank of an outcome record: WALK -> the rank whose arc holds the
// owner of the record's key (bounds: the last peer ID of every non-empty arc,
// ascending, with its rank), RESULT -> origin rank, NONE -> -1.
__device__ __forceinline__ int arc_dest(const ArcRec &r, const ArcBound *bounds, int nb, int G) {
    const uint32_t kind = r.hk >> 8;
    if (kind == ARC_RESULT) {
        const uint64_t o = r.qid >> ARC_ORIGIN_SHIFT;
        return o < (uint64_t)G ? (int)o : -1;
    }
    // WALK records, and NEW lookups sent ahead by key (ArcRouter key_first):
    // the rank whose arc holds the key's owner
    if ((kind != ARC_WALK && kind != ARC_NEW) || nb == 0) return -1;
    const u128 k = ((u128)r.w1 << 64) | r.w0;
    int lo = 0, hi = nb;  // first bound >= key; past the last one the owner wraps to arc 0
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (((u128)bounds[mid].hi << 64 | bounds[mid].lo) < k) lo = mid + 1;
        else hi = mid;
    }
    return (int)bounds[lo == nb ? 0 : lo].rank;
}

// Bucket outcome records by destination: per-block LDS histograms, one global
// atomic per (block, destination) to reserve ranges, LDS-local offsets.
constexpr int ARC_MAX_RANKS = 64;

// Records to bucket: stored ones, or (SEED) NEW lookups synthesised from the
// caller's src / keys as k_arc_seed writes them (no seed array in HBM).
template <bool SEED>
struct ArcIn {
    const ArcRec *recs;
    const uint32_t *src;
    const cell128 *keys;
    int self;
    __device__ __forceinline__ ArcRec get(size_t i) const {
        if (!SEED) return recs[i];
        const u128 k = ld128(keys + i);
        ArcRec r;
        r.w0 = (uint64_t)k;
        r.w1 = (uint64_t)(k >> 64);
        r.qid = ((uint64_t)self << ARC_ORIGIN_SHIFT) | i;
        r.cur = src[i];
        r.hk = ARC_NEW << 8;
        return r;
    }
};

// Per-destination counts of one wave's records: one ballot per destination,
// one LDS atomic per (wave, destination) present; returns the record's slot
// among the block's records for its destination (base from the LDS counter).
__device__ __forceinline__ uint32_t arc_wave_slots(int d, int G, uint32_t *h) {
    const int lane = threadIdx.x & 63;
    uint32_t slot = 0;
    for (int j = 0; j < G; ++j) {
        const uint64_t m = __ballot(d == j);
        if (!m) continue;  // wave-uniform
        const int leader = __builtin_ctzll(m);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&h[j], (uint32_t)__popcll(m));
        base = __shfl(base, leader, 64);
        if (d == j)
            slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    }
    return slot;
}

template <bool SEED>
__global__ __launch_bounds__(256) void k_arc_count(ArcIn<SEED> in, size_t q,
                                                   const ArcBound *bounds, int nb, int G,
                                                   uint32_t *counts) {
    __shared__ uint32_t h[ARC_MAX_RANKS];
    __shared__ ArcBound sb[ARC_MAX_RANKS];
    for (int j = threadIdx.x; j < G; j += blockDim.x) h[j] = 0;
    for (int j = threadIdx.x; j < nb; j += blockDim.x) sb[j] = bounds[j];
    __syncthreads();
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i0 = blockIdx.x * (size_t)blockDim.x; i0 < q; i0 += stride) {  // uniform trips
        const size_t i = i0 + threadIdx.x;
        const int d = i < q ? arc_dest(in.get(i), sb, nb, G) : -1;
        (void)arc_wave_slots(d, G, h);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < G; j += blockDim.x)
        if (h[j]) atomicAdd(&counts[j], h[j]);
}

// Four records per thread per pass (1024 per block): the block's slot
// reservation (LDS histogram, one global atomic per destination, three
// barriers) is paid once per 1024 records instead of once per 256.
constexpr int ARC_SCAT_R = 4;

template <bool SEED>
__global__ __launch_bounds__(256) void k_arc_scatter(ArcIn<SEED> in, size_t q,
                                                     const ArcBound *bounds, int nb, int G,
                                                     uint32_t *cursor, ArcRec *send) {
    __shared__ uint32_t h[ARC_MAX_RANKS], basep[ARC_MAX_RANKS];
    __shared__ ArcBound sb[ARC_MAX_RANKS];
    for (int j = threadIdx.x; j < nb; j += blockDim.x) sb[j] = bounds[j];
    const size_t per = (size_t)blockDim.x * ARC_SCAT_R;
    for (size_t b0 = (size_t)blockIdx.x * per; b0 < q; b0 += (size_t)gridDim.x * per) {
        for (int j = threadIdx.x; j < G; j += blockDim.x) h[j] = 0;
        __syncthreads();
        ArcRec r[ARC_SCAT_R];
        int d[ARC_SCAT_R];
        uint32_t slot[ARC_SCAT_R];
#pragma unroll
        for (int k = 0; k < ARC_SCAT_R; ++k) {
            const size_t i = b0 + (size_t)k * blockDim.x + threadIdx.x;
            d[k] = -1;
            if (i < q) {
                r[k] = in.get(i);
                d[k] = arc_dest(r[k], sb, nb, G);
            }
        }
#pragma unroll
        for (int k = 0; k < ARC_SCAT_R; ++k) slot[k] = arc_wave_slots(d[k], G, h);
        __syncthreads();
        for (int j = threadIdx.x; j < G; j += blockDim.x)
            basep[j] = h[j] ? atomicAdd(&cursor[j], h[j]) : 0u;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < ARC_SCAT_R; ++k)
            if (d[k] >= 0) send[basep[d[k]] + slot[k]] = r[k];
        __syncthreads();
    }
}

// Key-first partition, structure of arrays: this rank's lookups grouped by the
// rank of their key's arc, as the exchange sends them -- keys (16 B), sources
// (4 B) -- and, kept at the origin, the send slot of every lookup (slot[i],
// written in lookup order: coalesced).  Results come back in send order (the
// arc rank answers its receive buffer in order and the return exchange swaps
// the splits), so no record carries an origin or an index across xGMI.
// cap > 0 (single-pass partition, cx_arc_partition_regions): destination d
// owns the region [d cap, (d + 1) cap) of the send arrays and cursor[d]
// starts at d cap, so no count pass is needed before the scatter; a block
// whose reservation would cross its region's end writes nothing of it and
// raises *ovf (the caller then partitions with the two-pass kernel).
// hint (sd != nullptr): the origin resolves the lookup's start at its source,
// reading (pred, self) of src from ring_ext in lookup order (coalesced: src =
// q mod N is sequential), and sends d = (key - id_src) >> gs with it, or
// ARC_HINT_LOCAL when StoredLocally holds at the source (0 hops), so the arc
// rank's walk starts without the source pair -- a random 32-B gather per
// lookup there, since the lookups it receives come from every origin.
__global__ __launch_bounds__(256) void k_arc_scatter_soa(ArcIn<true> in, size_t q,
                                                         const ArcBound *bounds, int nb, int G,
                                                         uint32_t *cursor, cell128 *skeys,
                                                         uint32_t *ssrc, uint32_t *slot_of,
                                                         uint32_t cap, uint32_t *ovf,
                                                         uint64_t *sd, const cell128 *ring_ext,
                                                         uint32_t n, int gs, const int64_t *pref,
                                                         int skip) {
    __shared__ uint32_t h[ARC_MAX_RANKS], basep[ARC_MAX_RANKS], off[ARC_MAX_RANKS];
    __shared__ ArcBound sb[ARC_MAX_RANKS];
    for (int j = threadIdx.x; j < nb; j += blockDim.x) sb[j] = bounds[j];
    if (threadIdx.x == 0) {  // exact layout: region d starts at the sum of counts below d
        uint64_t acc = 0;
        for (int j = 0; j < G; ++j) {
            off[j] = (uint32_t)acc;
            acc += pref && j != skip ? (uint64_t)pref[j] : 0u;
        }
    }
    const size_t per = (size_t)blockDim.x * ARC_SCAT_R;
    for (size_t b0 = (size_t)blockIdx.x * per; b0 < q; b0 += (size_t)gridDim.x * per) {
        for (int j = threadIdx.x; j < G; j += blockDim.x) h[j] = 0;
        __syncthreads();
        ArcRec r[ARC_SCAT_R];
        int d[ARC_SCAT_R];
        uint32_t slot[ARC_SCAT_R];
#pragma unroll
        for (int k = 0; k < ARC_SCAT_R; ++k) {
            const size_t i = b0 + (size_t)k * blockDim.x + threadIdx.x;
            d[k] = -1;
            if (i < q) {
                r[k] = in.get(i);
                d[k] = arc_dest(r[k], sb, nb, G);
                if (d[k] == skip) {  // walked in place by the rank itself: no slot
                    slot_of[i] = 0xFFFFFFFFu;
                    d[k] = -1;
                }
            }
        }
        uint64_t dh[ARC_SCAT_R];
        if (sd) {
#pragma unroll
            for (int k = 0; k < ARC_SCAT_R; ++k) {
                dh[k] = ARC_HINT_BAD;
                if (d[k] >= 0 && r[k].cur < n) {
                    const u128 key = ((u128)r[k].w1 << 64) | r[k].w0;
                    const u128 pa = ld128(ring_ext + r[k].cur), pb = ld128(ring_ext + r[k].cur + 1);
                    dh[k] = (n == 1 || (key - pa - 1) <= (pb - pa - 1)) ? ARC_HINT_LOCAL
                                                                         : (uint64_t)((key - pb) >> 64) >> (gs - 64);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < ARC_SCAT_R; ++k) slot[k] = arc_wave_slots(d[k], G, h);
        __syncthreads();
        for (int j = threadIdx.x; j < G; j += blockDim.x) {
            basep[j] = h[j] ? off[j] + atomicAdd(&cursor[j], h[j]) : 0u;
            if (cap && h[j] && (uint64_t)basep[j] + h[j] > (uint64_t)(j + 1) * cap) {
                atomicOr(ovf, 1u);
                basep[j] = 0xFFFFFFFFu;  // nothing of this destination is written
            }
            // exact layout: counts that do not match these lookups (a caller's
            // error) never write past the arrays
            if (pref && h[j] && (uint64_t)basep[j] + h[j] > q) basep[j] = 0xFFFFFFFFu;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < ARC_SCAT_R; ++k)
            if (d[k] >= 0 && basep[d[k]] != 0xFFFFFFFFu) {
                const uint32_t o = basep[d[k]] + slot[k];
                skeys[o] = cell128{r[k].w0, r[k].w1};
                ssrc[o] = r[k].cur;
                if (sd) sd[o] = dh[k];
                slot_of[r[k].qid & ARC_INDEX_MASK] = o;
            }
        __syncthreads();
    }
}

// Results back at the origin: res[j] answers the lookup in send slot j; lookup
// i reads res[slot_of[i]] (an 8-B gather) and its outputs are written in
// lookup order (coalesced, no scattered byte stores).
__global__ void k_arc_deliver(const uint64_t *res, const uint32_t *slot_of, size_t q,
                              uint32_t *owner, uint8_t *hops, uint8_t *status) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < q;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t sl = slot_of ? slot_of[i] : (uint32_t)i;
        if (sl == 0xFFFFFFFFu) continue;  // the origin's own lookup: answered in place
        const uint64_t v = res[sl];
        owner[i] = (uint32_t)v;
        hops[i] = (uint8_t)(v >> 32);
        if (status) status[i] = (uint8_t)(v >> 40);
    }
}

// cursor[g] = exclusive prefix sum of counts (one wave).
__global__ void k_arc_offsets(const uint32_t *counts, int G, uint32_t *cursor) {
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int g = 0; g < G; ++g) {
            cursor[g] = acc;
            acc += counts[g];
        }
    }
}

template <bool SEED>
static hipError_t arc_bucket_in(const ArcIn<SEED> &in, size_t q, const ArcBound *bounds, int nb,
                                int G, uint32_t *counts_dev, uint32_t *cursor_dev, ArcRec *send,
                                hipStream_t s, bool scatter) {
    if (!scatter) {  // counts, and the scatter cursors from them (device side)
        if (q) k_arc_count<SEED><<<cx_grid(q, 256, 2048), 256, 0, s>>>(in, q, bounds, nb, G,
                                                                       counts_dev);
        if (cursor_dev) k_arc_offsets<<<1, 64, 0, s>>>(counts_dev, G, cursor_dev);
        return hipGetLastError();
    }
    if (q)
        k_arc_scatter<SEED><<<cx_grid((q + ARC_SCAT_R - 1) / ARC_SCAT_R, 256, 2048), 256, 0,
                              s>>>(in, q, bounds, nb, G, cursor_dev, send);
    return hipGetLastError();
}

hipError_t arc_partition(const uint32_t *src, const cell128 *keys, size_t q,
                         const ArcBound *bounds, int nb, int G, uint32_t *counts_dev,
                         uint32_t *cursor_dev, cell128 *skeys, uint32_t *ssrc, uint32_t *perm,
                         hipStream_t s) {
    const ArcIn<true> in{nullptr, src, keys, 0};
    hipError_t e = arc_bucket_in(in, q, bounds, nb, G, counts_dev, cursor_dev, nullptr, s, false);
    if (e != hipSuccess || q == 0) return e;
    k_arc_scatter_soa<<<cx_grid((q + ARC_SCAT_R - 1) / ARC_SCAT_R, 256, 2048), 256, 0, s>>>(
        in, q, bounds, nb, G, cursor_dev, skeys, ssrc, perm, 0u, nullptr, nullptr, nullptr, 0u,
        0, nullptr, -1);
    return hipGetLastError();
}

// Single pass: cursor_dev[d] = d * cap already (the caller's), ovf zeroed.
hipError_t arc_partition_regions(const uint32_t *src, const cell128 *keys, size_t q,
                                 const ArcBound *bounds, int nb, int G, uint32_t cap,
                                 uint32_t *cursor_dev, uint32_t *ovf, cell128 *skeys,
                                 uint32_t *ssrc, uint32_t *perm, uint64_t *sd,
                                 const cell128 *ring_ext, size_t n, int ib, hipStream_t s) {
    if (q == 0) return hipSuccess;
    const ArcIn<true> in{nullptr, src, keys, 0};
    k_arc_scatter_soa<<<cx_grid((q + ARC_SCAT_R - 1) / ARC_SCAT_R, 256, 2048), 256, 0, s>>>(
        in, q, bounds, nb, G, cursor_dev, skeys, ssrc, perm, cap, ovf, sd, ring_ext,
        (uint32_t)n, cz_shift(ib), nullptr, -1);
    return hipGetLastError();
}

// Count pass of the exact-layout partition, one kernel: counts[d] (int64) =
// lookups whose key's arc is rank d's, and with own_idx the indices of rank
// `me`'s lookups.  Keys only (16 B per lookup).  Block b takes the contiguous
// lookups [b per, (b + 1) per), per <= 64 rounds of 256; lane j of each wave
// accumulates the wave's count for rank j from one ballot per (round, rank),
// so the histogram costs no LDS atomics per lookup, and each lane keeps one
// bit per round for "rank me's".  At the end the block reserves its own
// lookups' run with one atomic on *cursor and writes them there ascending
// (runs in block completion order: own_idx is a permutation of the own
// lookups, ascending within each block's run).  Round 5 wrote a destination
// byte per lookup and compacted in a second kernel (132 + 70 us at 2^25).
constexpr int ARC_CNT_ROUNDS = 64;  // rounds of 256 lookups per block at most

__global__ __launch_bounds__(256) void k_arc_count_keys(const cell128 *keys, size_t q,
                                                        const ArcBound *bounds, int nb, int G,
                                                        unsigned long long *counts, int me,
                                                        uint32_t *own_idx, uint32_t *cursor,
                                                        size_t per) {
    __shared__ uint32_t h[ARC_MAX_RANKS];
    __shared__ ArcBound sb[ARC_MAX_RANKS];
    __shared__ uint32_t wc[ARC_CNT_ROUNDS * 4];  // own lookups per (round, wave), then offsets
    __shared__ uint32_t wsum[4], base_s;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int j = t; j < G; j += blockDim.x) h[j] = 0;
    for (int j = t; j < nb; j += blockDim.x) sb[j] = bounds[j];
    wc[t] = 0;  // blockDim.x == 256 == ARC_CNT_ROUNDS * 4
    __syncthreads();
    const size_t lo = blockIdx.x * per, hi = lo + per < q ? lo + per : q;
    const int rounds = (int)((hi - lo + 255) / 256);
    uint32_t acc = 0;   // lane j < G: this wave's lookups bound for rank j
    uint64_t mine = 0;  // bit r: this lane's lookup of round r is rank me's
    // the next trip's keys are loaded before this trip's are classified, so a
    // wave keeps its loads in flight through the compares and ballots
    u128 kn[ARC_SCAT_R];
#pragma unroll
    for (int k = 0; k < ARC_SCAT_R; ++k) {
        const size_t i = lo + (size_t)k * 256 + t;
        kn[k] = i < hi ? ld128(keys + i) : (u128)0;
    }
    for (int r0 = 0; r0 < rounds; r0 += ARC_SCAT_R) {  // uniform trips
        u128 kc[ARC_SCAT_R];
#pragma unroll
        for (int k = 0; k < ARC_SCAT_R; ++k) {
            kc[k] = kn[k];
            const size_t i = lo + (size_t)(r0 + ARC_SCAT_R + k) * 256 + t;
            kn[k] = i < hi ? ld128(keys + i) : (u128)0;
        }
        int d[ARC_SCAT_R];
#pragma unroll
        for (int k = 0; k < ARC_SCAT_R; ++k) {
            const size_t i = lo + (size_t)(r0 + k) * 256 + t;
            d[k] = -1;
            if (i < hi) {
                ArcRec r;
                r.w0 = (uint64_t)kc[k];
                r.w1 = (uint64_t)(kc[k] >> 64);
                r.hk = ARC_NEW << 8;
                d[k] = arc_dest(r, sb, nb, G);
            }
        }
        for (int j = 0; j < G; ++j) {
            uint32_t c = 0;
#pragma unroll
            for (int k = 0; k < ARC_SCAT_R; ++k) c += (uint32_t)__popcll(__ballot(d[k] == j));
            if (lane == j) acc += c;
        }
        if (own_idx) {
#pragma unroll
            for (int k = 0; k < ARC_SCAT_R; ++k) {
                const uint64_t m = __ballot(d[k] == me);
                if (d[k] == me) mine |= 1ull << (r0 + k);
                if (lane == 0 && r0 + k < ARC_CNT_ROUNDS) wc[(r0 + k) * 4 + w] = (uint32_t)__popcll(m);
            }
        }
    }
    if (lane < G && acc) atomicAdd(&h[lane], acc);
    __syncthreads();
    for (int j = t; j < G; j += blockDim.x)
        if (h[j]) atomicAdd(&counts[j], (unsigned long long)h[j]);
    if (!own_idx) return;  // block-uniform
    // exclusive offsets of the (round, wave) runs, in index order
    const uint32_t v = wc[t];
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t ex = x - v;
    for (int j = 0; j < w; ++j) ex += wsum[j];
    wc[t] = ex;
    if (t == 0) {
        const uint32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        base_s = tot ? atomicAdd(cursor, tot) : 0u;
    }
    __syncthreads();
    const uint32_t base = base_s;
    for (int r = 0; r < rounds; ++r) {  // uniform trips
        const bool b = (mine >> r) & 1;
        const uint64_t m = __ballot(b);
        if (!m) continue;
        if (b)
            own_idx[base + wc[r * 4 + w] +
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] =
                (uint32_t)(lo + (size_t)r * 256 + t);
    }
}

// counts[0..G) and the own-run cursor zeroed in one launch.
__global__ void k_arc_count_zero(unsigned long long *counts, int G, uint32_t *cursor) {
    const int j = threadIdx.x;
    if (j < G) counts[j] = 0;
    if (j == 0 && cursor) *cursor = 0;
}

// own_ws: one word, the own-run cursor.
hipError_t arc_count_keys(const cell128 *keys, size_t q, const ArcBound *bounds, int nb, int G,
                          int64_t *counts, int me, uint32_t *own_idx, uint32_t *own_ws,
                          hipStream_t s) {
    uint32_t *cursor = own_idx ? own_ws : nullptr;
    auto *c64 = reinterpret_cast<unsigned long long *>(counts);
    k_arc_count_zero<<<1, 64, 0, s>>>(c64, G, cursor);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || q == 0) return e;
    // ~2048 blocks when the batch allows (1024-lookup tiles, at most 16 a block)
    const size_t tiles = (q + 1023) / 1024;
    size_t tpb = (tiles + 2047) / 2048;
    if (tpb > (size_t)ARC_CNT_ROUNDS / 4) tpb = ARC_CNT_ROUNDS / 4;
    const size_t per = tpb * 1024;
    const unsigned g = (unsigned)((q + per - 1) / per);
    k_arc_count_keys<<<g, 256, 0, s>>>(keys, q, bounds, nb, G, c64, own_idx ? me : -1, own_idx,
                                       cursor, per);
    return hipGetLastError();
}

// Exact-layout scatter: destination d's lookups at [sum_{j<d} counts[j], ...)
// of the send arrays (counts from arc_count_keys over the same lookups, read
// on the device: the scatter needs no host round trip); cursor: G words of
// the caller's, zeroed here.  skip >= 0: that destination's lookups (the
// rank's own, walked in place) take no slot (perm = 0xFFFFFFFF, counted as 0).
hipError_t arc_scatter_exact(const uint32_t *src, const cell128 *keys, size_t q,
                             const ArcBound *bounds, int nb, int G, const int64_t *counts,
                             uint32_t *cursor, cell128 *skeys, uint32_t *ssrc, uint32_t *perm,
                             uint64_t *sd, const cell128 *ring_ext, size_t n, int ib, int skip,
                             hipStream_t s) {
    hipError_t e = hipMemsetAsync(cursor, 0, (size_t)G * sizeof(uint32_t), s);
    if (e != hipSuccess || q == 0) return e;
    const ArcIn<true> in{nullptr, src, keys, 0};
    k_arc_scatter_soa<<<cx_grid((q + ARC_SCAT_R - 1) / ARC_SCAT_R, 256, 2048), 256, 0, s>>>(
        in, q, bounds, nb, G, cursor, skeys, ssrc, perm, 0u, nullptr, sd, ring_ext, (uint32_t)n,
        cz_shift(ib), counts, skip);
    return hipGetLastError();
}

// Region cursors of the single-pass partition (cursor[g] = g cap) and its
// overflow flag, set on the device (no host copy in the partition path).
__global__ void k_arc_cursor_init(uint32_t *cursor, uint32_t *ovf, int G, uint32_t cap) {
    const int g = threadIdx.x;
    if (g < G) cursor[g] = (uint32_t)g * cap;
    if (g == 0) *ovf = 0;
}

// counts[g] = cursor[g] - g cap (int64, a collective's input), counts[G] = overflow.
__global__ void k_arc_counts_out(const uint32_t *cursor, const uint32_t *ovf, int G, uint32_t cap,
                                 int64_t *counts) {
    const int g = threadIdx.x;
    if (g < G) counts[g] = (int64_t)(cursor[g] - (uint32_t)g * cap);
    if (g == 0) counts[G] = *ovf ? 1 : 0;
}

hipError_t arc_cursor_init(uint32_t *cursor, uint32_t *ovf, int G, uint32_t cap, hipStream_t s) {
    k_arc_cursor_init<<<1, 64, 0, s>>>(cursor, ovf, G, cap);
    return hipGetLastError();
}

hipError_t arc_counts_out(const uint32_t *cursor, const uint32_t *ovf, int G, uint32_t cap,
                          int64_t *counts, hipStream_t s) {
    k_arc_counts_out<<<1, 64, 0, s>>>(cursor, ovf, G, cap, counts);
    return hipGetLastError();
}

hipError_t arc_deliver(const uint64_t *res, const uint32_t *perm, size_t q, uint32_t *owner,
                       uint8_t *hops, uint8_t *status, hipStream_t s) {
    if (q == 0) return hipSuccess;
    k_arc_deliver<<<cx_grid(q, 256, 8192), 256, 0, s>>>(res, perm, q, owner, hops, status);
    return hipGetLastError();
}

hipError_t arc_bucket(const ArcRec *recs, size_t q, const ArcBound *bounds, int nb, int G,
                      uint32_t *counts_dev, uint32_t *cursor_dev, ArcRec *send, hipStream_t s,
                      bool scatter) {
    return arc_bucket_in(ArcIn<false>{recs, nullptr, nullptr, 0}, q, bounds, nb, G, counts_dev,
                         cursor_dev, send, s, scatter);
}

hipError_t arc_bucket_seed(const uint32_t *src, const cell128 *keys, int self, size_t q,
                           const ArcBound *bounds, int nb, int G, uint32_t *counts_dev,
                           uint32_t *cursor_dev, ArcRec *send, hipStream_t s, bool scatter) {
    return arc_bucket_in(ArcIn<true>{nullptr, src, keys, self}, q, bounds, nb, G, counts_dev,
                         cursor_dev, send, s, scatter);
}

hipError_t route(const cell128 *ring, size_t n, const uint32_t *F, const cell128 *min_keys,
                 const uint32_t *preds, const LitState &ls, bool literal, const uint32_t *src,
                 const cell128 *keys, size_t q, uint32_t *owner, uint8_t *hops, uint8_t *status,
                 hipStream_t s) {
    if (q == 0) return hipSuccess;
    const unsigned g = cx_grid(q, ROUTE_BLOCK, 1u << 20);
    if (literal)
        k_route_literal<<<g, ROUTE_BLOCK, 0, s>>>(ring, (uint32_t)n, F, min_keys, preds, ls, src,
                                                  keys, q, owner, hops, status);
    else
        k_route_conv<<<g, ROUTE_BLOCK, 0, s>>>(ring, (uint32_t)n, F, src, keys, q, owner, hops,
                                               status);
    return hipGetLastError();
}

// ===========================================================================
// a10/a11: n-successor windows.
// ===========================================================================
// Rows of `w` elements for keys [base, base + cnt) are staged in LDS by the
// block and written as one contiguous, coalesced range.
constexpr int ROW_BLOCK = 256;

// Rows of `w` bytes (the target rows), staged in LDS, leave in 16-B streaming
// stores as one contiguous range; the stage is refilled with 0xFF (no target)
// for the next tile, each lane refilling what it stored.
__device__ __forceinline__ void flush_rows_refill(uint8_t *stage, uint8_t *out, size_t base,
                                                  int cnt, int w) {
    const int total = cnt * w;
    uint8_t *dst = out + base * (size_t)w;
    int t0 = 0;
    if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(stage)) & 15) == 0) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const int nv = total >> 4;
        v4u *sv = reinterpret_cast<v4u *>(stage);
        v4u *dv = reinterpret_cast<v4u *>(dst);
        const v4u none = {~0u, ~0u, ~0u, ~0u};
        for (int t = threadIdx.x; t < nv; t += blockDim.x) {
            __builtin_nontemporal_store(sv[t], dv + t);
            sv[t] = none;
        }
        t0 = nv << 4;
    }
    for (int t = t0 + threadIdx.x; t < total; t += blockDim.x) {
        dst[t] = stage[t];
        stage[t] = 0xFF;
    }
}

// Rows of `w` ring indices (s[k] + j) mod N for j < nvalid, CX_NONE after, for
// keys [base, base + cnt) of the block, s[k] staged in LDS: every word of the
// block's contiguous output range is computed where it is stored (16-B
// streaming stores), with no staging of the rows themselves.
__device__ __forceinline__ void flush_window(const uint32_t *s, uint32_t *out, size_t base,
                                             int cnt, int w, int nvalid, uint32_t N) {
    const int total = cnt * w;
    uint32_t *dst = out + base * (size_t)w;
    auto val = [&](int k, int j) -> uint32_t {
        uint32_t v = s[k] + (uint32_t)j;
        if (v >= N) v -= N;
        return j < nvalid ? v : CX_NONE;
    };
    int t0 = 0;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const int nv = total >> 2;
        v4u *dv = reinterpret_cast<v4u *>(dst);
        // (row k, column j) of word 4t, advanced by 4 blockDim words a step
        // (one division per call instead of one per store)
        const int step = 4 * (int)blockDim.x, dk = step / w, dj = step - dk * w;
        int k = (4 * (int)threadIdx.x) / w, j = 4 * (int)threadIdx.x - k * w;
        for (int t = threadIdx.x; t < nv; t += blockDim.x) {
            const int k0 = k, j0 = j;
            k += dk;
            j += dj;
            if (j >= w) {
                j -= w;
                ++k;
            }
            int kk = k0, jj = j0;
            uint32_t x[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                x[u] = val(kk, jj);
                if (++jj == w) {
                    jj = 0;
                    ++kk;
                }
            }
            const v4u xv = {x[0], x[1], x[2], x[3]};
            __builtin_nontemporal_store(xv, dv + t);
        }
        t0 = nv << 2;
    }
    for (int t = t0 + threadIdx.x; t < total; t += blockDim.x) {
        const int k = t / w;
        dst[t] = val(k, t - k * w);
    }
}

template <bool DIR>
__global__ __launch_bounds__(ROW_BLOCK) void k_nsucc(SearchView sv, const cell128 *keys, size_t q,
                                                     int nlist, uint32_t *lists, uint8_t *count) {
    __shared__ u128 lds[Searcher<DIR>::LDS];
    __shared__ uint32_t s_succ[ROW_BLOCK];
    Searcher<DIR>::stage(sv, lds);
    const uint32_t n = sv.ev.n;
    const int nn = (uint32_t)nlist < n ? nlist : (int)n;
    for (size_t base = (size_t)blockIdx.x * ROW_BLOCK; base < q;
         base += (size_t)gridDim.x * ROW_BLOCK) {
        const size_t i = base + threadIdx.x;
        const int cnt = (q - base < (size_t)ROW_BLOCK) ? (int)(q - base) : ROW_BLOCK;
        if (i < q) {
            s_succ[threadIdx.x] = Searcher<DIR>::find(sv, lds, ld128(keys + i));
            count[i] = (uint8_t)nn;
        }
        __syncthreads();
        flush_window(s_succ, lists, base, cnt, nlist, nn, n);
        __syncthreads();
    }
}

hipError_t nsucc(const SearchView &sv, const cell128 *keys, size_t q, int n, uint32_t *lists,
                 uint8_t *count, hipStream_t s) {
    if (q == 0) return hipSuccess;
    if (sv.dir)
        k_nsucc<true><<<cx_grid(q, ROW_BLOCK, 8192), ROW_BLOCK, 0, s>>>(sv, keys, q, n, lists,
                                                                        count);
    else
        k_nsucc<false><<<cx_grid(q, ROW_BLOCK, 512), ROW_BLOCK, 0, s>>>(sv, keys, q, n, lists,
                                                                        count);
    return hipGetLastError();
}

// ===========================================================================
// a12: churn support + misplaced scan.
// ===========================================================================
template <bool DIR>
__global__ __launch_bounds__(SUCC_BLOCK) void k_mark_leaves(SearchView sv, const cell128 *ring,
                                                            const cell128 *leaves, size_t nl,
                                                            uint8_t *gone) {
    __shared__ u128 lds[Searcher<DIR>::LDS];
    Searcher<DIR>::stage(sv, lds);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nl;
         i += (size_t)gridDim.x * blockDim.x) {
        const u128 x = ld128(leaves + i);
        const uint32_t s0 = Searcher<DIR>::find(sv, lds, x);
        if (ld128(ring + s0) == x) gone[s0] = 1;
    }
}

hipError_t mark_leaves(const SearchView &sv, const cell128 *ring, const cell128 *leaves,
                       size_t nl, uint8_t *gone, hipStream_t s) {
    if (nl == 0) return hipSuccess;
    if (sv.dir)
        k_mark_leaves<true><<<cx_grid(nl, SUCC_BLOCK, 512), SUCC_BLOCK, 0, s>>>(sv, ring, leaves,
                                                                                nl, gone);
    else
        k_mark_leaves<false><<<cx_grid(nl, SUCC_BLOCK, 512), SUCC_BLOCK, 0, s>>>(sv, ring, leaves,
                                                                                 nl, gone);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Merge-based churn: the surviving old ring is already
// sorted, so only the joins are sorted; every element's new index follows from
// two prefix sums over old positions,
//   G[p] = 1 if old peer p leaves,  A[p] = # kept joins whose lower_bound is p,
//   new(survivor p) = p - SG[p] + SA[p+1],
//   new(kept join j) = rank of j among kept joins + pos_j - SG[pos_j],
// and the new ring is written by one streaming scatter (no full re-sort).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(SUCC_BLOCK) void k_mark_leaves32(SearchView sv, const cell128 *ring,
                                                              const cell128 *leaves, size_t nl,
                                                              uint32_t *gone) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nl;
         i += (size_t)gridDim.x * blockDim.x) {
        const u128 x = ld128(leaves + i);
        const uint32_t s0 = dir_successor(sv, x);
        if (ld128(ring + s0) == x) gone[s0] = 1;
    }
}

// pos_j = first old index with id >= x (n if none); keep_j = not a repeat of
// the previous sorted join and not the ID of a surviving peer (survivors win,
// remote_peer_list.cpp:56-58).
__global__ __launch_bounds__(SUCC_BLOCK) void k_join_pos(SearchView sv, const cell128 *ring,
                                                         uint32_t n, const uint32_t *gone,
                                                         const cell128 *J, size_t nj,
                                                         uint32_t *pos, uint32_t *keep,
                                                         uint32_t *A) {
    for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j < nj;
         j += (size_t)gridDim.x * blockDim.x) {
        const u128 x = ld128(J + j);
        uint32_t P = dir_successor(sv, x);
        const u128 idp = ld128(ring + P);
        if (P == 0 && idp < x) P = n;  // above the largest ID: appended at the end
        const bool dup = j > 0 && ld128(J + j - 1) == x;
        const bool coll = P < n && idp == x && !gone[P];
        const uint32_t k = (!dup && !coll) ? 1u : 0u;
        pos[j] = P;
        keep[j] = k;
        if (k) atomicAdd(&A[P], 1u);
    }
}

__global__ void k_merge_survivors(const cell128 *ring, uint32_t n, const uint32_t *SG,
                                  const uint32_t *SA, cell128 *out, uint32_t *o2n) {
    for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < n;
         p += (size_t)gridDim.x * blockDim.x) {
        const uint32_t sg = SG[p];
        if (SG[p + 1] != sg) {
            o2n[p] = CX_NONE;
        } else {
            const uint32_t ni = (uint32_t)p - sg + SA[p + 1];
            st128(out + ni, ld128(ring + p));
            o2n[p] = ni;
        }
    }
}

__global__ void k_merge_joins(const cell128 *J, size_t nj, const uint32_t *pos,
                              const uint32_t *kidx, const uint32_t *SG, cell128 *out) {
    for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j < nj;
         j += (size_t)gridDim.x * blockDim.x) {
        if (kidx[j + 1] == kidx[j]) continue;
        const uint32_t P = pos[j];
        st128(out + (kidx[j] + P - SG[P]), ld128(J + j));
    }
}

hipError_t merge_mark(const SearchView &sv, const cell128 *ring, const cell128 *leaves,
                      size_t nl, uint32_t *gone, hipStream_t s) {
    if (nl == 0) return hipSuccess;
    k_mark_leaves32<<<cx_grid(nl, SUCC_BLOCK, 2048), SUCC_BLOCK, 0, s>>>(sv, ring, leaves, nl,
                                                                          gone);
    return hipGetLastError();
}

hipError_t merge_join_pos(const SearchView &sv, const cell128 *ring, size_t n,
                          const uint32_t *gone, const cell128 *J, size_t nj, uint32_t *pos,
                          uint32_t *keep, uint32_t *A, hipStream_t s) {
    if (nj == 0) return hipSuccess;
    k_join_pos<<<cx_grid(nj, SUCC_BLOCK, 2048), SUCC_BLOCK, 0, s>>>(sv, ring, (uint32_t)n, gone,
                                                                     J, nj, pos, keep, A);
    return hipGetLastError();
}

hipError_t merge_scatter(const cell128 *ring, size_t n, const uint32_t *SG, const uint32_t *SA,
                         const cell128 *J, size_t nj, const uint32_t *pos, const uint32_t *kidx,
                         cell128 *out, uint32_t *o2n, hipStream_t s) {
    if (n) k_merge_survivors<<<cx_grid(n, 256), 256, 0, s>>>(ring, (uint32_t)n, SG, SA, out, o2n);
    if (nj) k_merge_joins<<<cx_grid(nj, 256), 256, 0, s>>>(J, nj, pos, kidx, SG, out);
    return hipGetLastError();
}

__global__ void k_copy_tagged(const cell128 *src, size_t n, uint32_t tag_base, cell128 *dk,
                              uint32_t *dt) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        st128(dk + i, ld128(src + i));
        dt[i] = tag_base + (uint32_t)i;
    }
}

hipError_t copy_tagged(const cell128 *src, size_t n, uint32_t tag_base, cell128 *dk,
                       uint32_t *dt, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_copy_tagged<<<cx_grid(n, 256), 256, 0, s>>>(src, n, tag_base, dk, dt);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Churn directory (misplaced scan after cx_churn).  The merged ring = old ring
// U joining peers in ID order; merged entry m is tagged 1 (departed old peer),
// 2 (joiner) or 3 (survivor).  For a key whose first merged entry at or after
// it is m: the old successor is so(m) = #old entries before m, the new one
// sn(m) = #new entries before m, and the old n-window's holders follow from
// the tags after m -- a survivor at old rank j holds new rank r = #new entries
// from m before it, a departed one is CX_NONE (dhash_peer.cpp:322-328 on the
// mapping cx_churn returns).  Bucket b (top kb bits, load factor <= 1/4) is
// one 32-B entry: {hint0 | so_b | sn_b}, {old mask | new mask | hint1 | cnt}
// with m_b = the bucket's first merged entry, bit k of the old / new mask =
// merged entry m_b + k is an old / new ring entry (its tag's two bits), hint = ID bits
// [64 - kb, 128 - kb) (hint1's low two bits hold cnt = entries in the bucket,
// capped at 3).  One 32-B gather replaces two directory searches and the
// 64-B window of old_to_new entries; keys it cannot settle (a third entry in
// the bucket, an equal hint, a window with too many joiners) take the
// two-search path.
// ---------------------------------------------------------------------------
struct ChurnDir {
    const uint4 *cd;          // [2^kb][2]
    int kb;
    const cell128 *ring_old, *ring_new;
    const uint32_t *ok;       // device flag: old_to_new equals cx_churn's mapping
};

// The key's 32-B bucket entry.
__device__ __forceinline__ void cd_fetch(const ChurnDir &c, u128 key, uint4 &A, uint4 &B) {
    const size_t b = (size_t)top_bits(key, c.kb);
    A = c.cd[2 * b];
    B = c.cd[2 * b + 1];
}

// Bit mask of positions 0 .. k.
__device__ __forceinline__ uint32_t cd_upto(int k) { return k >= 31 ? 0xFFFFFFFFu : (2u << k) - 1u; }

// Position of the c-th (1-based) set bit of M, which has at least c: k rises
// to c - 1 + (clear bits of M in [0, k]) until it stops (each step skips the
// clear bits found; a window has few).
__device__ __forceinline__ int cd_nth_bit(uint32_t M, int c) {
    int k = c - 1;
    for (;;) {
        const int nk = c - 1 + __popc(~M & cd_upto(k));
        if (nk == k) return k;
        k = nk;
    }
}

// x without the bit positions of Z (higher bits move down); x is clear at Z.
__device__ __forceinline__ uint32_t cd_drop(uint32_t x, uint32_t Z) {
    while (Z) {  // highest first, so the lower positions stay valid
        const int p = 31 - __builtin_clz(Z);
        Z ^= 1u << p;
        const uint32_t lo = (1u << p) - 1u;
        x = (x & lo) | ((x >> 1) & ~lo);
    }
    return x;
}

// 1 = settled (so, sn, has, mis set), 0 = take the search path.  A, B = the
// key's bucket entry (cd_fetch).
__device__ __forceinline__ int cd_lookup(const ChurnDir &c, u128 key, const uint4 A,
                                         const uint4 B, uint32_t n_old, uint32_t n_new, int no,
                                         int nn, uint32_t &so, uint32_t &sn, uint32_t &has,
                                         uint32_t &mis) {
    const uint64_t xf = mid_bits(key, c.kb);
    const uint64_t h0 = ((uint64_t)A.y << 32) | A.x;
    uint32_t O = B.x, N = B.y;  // bit k: merged entry m + k is old / new
    const uint64_t h1c = ((uint64_t)B.w << 32) | B.z;
    const int cnt = (int)(h1c & 3);
    uint32_t o = A.z, w = A.w;  // so / sn at the bucket's first merged entry
    int t = 0;
    if (cnt >= 1) {
        if (xf == h0) {  // exact compare with the first entry's ID
            const u128 id = (O & 1) ? ld128(c.ring_old + o) : ld128(c.ring_new + w);
            t = key > id;
        } else {
            t = xf > h0;
        }
        if (t) {
            o += O & 1u;
            w += N & 1u;
            if (o >= n_old) o -= n_old;
            if (w >= n_new) w -= n_new;
            O >>= 1;
            N >>= 1;
            if (cnt >= 2) {
                int t2;
                if ((xf >> 2) == (h1c >> 2)) {
                    const u128 id = (O & 1) ? ld128(c.ring_old + o) : ld128(c.ring_new + w);
                    t2 = key > id;
                } else {
                    t2 = (xf >> 2) > (h1c >> 2);
                }
                if (t2) {
                    if (cnt == 3) return 0;  // a third entry may precede the key
                    o += O & 1u;
                    w += N & 1u;
                    if (o >= n_old) o -= n_old;
                    if (w >= n_new) w -= n_new;
                    O >>= 1;
                    N >>= 1;
                }
            }
        }
    }
    so = o;
    sn = w;
    // The old window is the first no old entries from the key on (positions
    // up to the no-th set bit of O).  A survivor (old and new) at position k
    // has old rank j = |O below k| and new rank r = |N below k|: it already
    // holds the key's new-list rank r when r < nn (positions up to the nn-th
    // new entry), else holder j is misplaced.  r and j are the survivor's
    // index once the positions without a new (old) entry are dropped.
    if (__popc(O) < no) return 0;  // the window ran out of tags
    const uint32_t act = cd_upto(cd_nth_bit(O, no));
    const uint32_t S = O & N & act;
    const uint32_t early = __popc(N & act) >= nn ? cd_upto(cd_nth_bit(N, nn)) : 0xFFFFFFFFu;
    has = cd_drop(S & early, ~N & act);
    mis = cd_drop(S & ~early, ~O & act);
    return 1;
}

// Misplaced scan core.  Holder ranks j in order; `has` = mask of new-list ranks
// already holding the key; membership of a holder in the new window is
// (holder - s_new) mod n_new < nn.  Rows (new list, targets) are staged in LDS
// per block of 256 consecutive keys and written coalesced.  CD: the churn
// directory settles most keys in one gather (cd_lookup) when *cd.ok.
// old_lists / old_count (CHURN, may be null): the keys' old n-successor lists
// as cx_nsucc on the old ring gives them -- the scan already holds the old
// successor, so DHash placement + maintenance share one pass over the keys.
template <bool CHURN, bool DIR, bool CD = false>
__global__ __launch_bounds__(ROW_BLOCK) void k_misplaced(SearchView sv_new, SearchView sv_old,
                                                         const uint32_t *old_to_new,
                                                         const uint32_t *holders, int nh,
                                                         const cell128 *keys, size_t q, int nlist,
                                                         uint32_t *new_lists, uint8_t *count,
                                                         uint16_t *mask, uint8_t *target,
                                                         ChurnDir cd, uint32_t *old_lists = nullptr,
                                                         uint8_t *old_count = nullptr) {
    __shared__ u128 lds_new[Searcher<DIR>::LDS];
    __shared__ u128 lds_old[CHURN ? Searcher<DIR>::LDS : 1];
    __shared__ uint32_t s_sn[ROW_BLOCK], s_so[ROW_BLOCK];  // the tile's successors
    __shared__ __attribute__((aligned(16))) uint8_t stage_t[ROW_BLOCK * CX_MAX_NSUCC];
    Searcher<DIR>::stage(sv_new, lds_new);
    if (CHURN) Searcher<DIR>::stage(sv_old, lds_old);
    const uint32_t n_new = sv_new.ev.n;
    const int nn = (uint32_t)nlist < n_new ? nlist : (int)n_new;
    const uint32_t n_old = CHURN ? sv_old.ev.n : 0;
    const int no = CHURN ? ((uint32_t)nlist < n_old ? nlist : (int)n_old) : nh;
    const int nslots = CHURN ? nlist : nh;
    const uint32_t full = (nn >= 32) ? 0xFFFFFFFFu : ((1u << nn) - 1u);
    const bool o2n_al = CHURN && ((uintptr_t)old_to_new & 15) == 0;
    const bool use_cd = CD && *cd.ok;  // wave-uniform
    static_assert(CX_MAX_NSUCC <= 17, "five 16-B o2n loads cover 17 entries");
    static_assert(ROW_BLOCK * CX_MAX_NSUCC % 16 == 0, "stage_t in 16-B chunks");
    for (int t = threadIdx.x; t < ROW_BLOCK * CX_MAX_NSUCC / 16; t += blockDim.x)
        reinterpret_cast<uint4 *>(stage_t)[t] = make_uint4(~0u, ~0u, ~0u, ~0u);
    __syncthreads();
    // software pipeline: the next tile's key is loaded when a tile starts and
    // its churn-directory entry before the tile's rows are flushed, so neither
    // gather sits between one tile's stores and the next tile's search
    const size_t stride = (size_t)gridDim.x * ROW_BLOCK;
    u128 key_n = 0;
    uint4 A_n = {0, 0, 0, 0}, B_n = {0, 0, 0, 0};
    if ((size_t)blockIdx.x * ROW_BLOCK + threadIdx.x < q) {
        key_n = ld128_nt(keys + (size_t)blockIdx.x * ROW_BLOCK + threadIdx.x);
        if (use_cd) cd_fetch(cd, key_n, A_n, B_n);
    }
    for (size_t base = (size_t)blockIdx.x * ROW_BLOCK; base < q; base += stride) {
        const size_t i = base + threadIdx.x;
        const int cnt = (q - base < (size_t)ROW_BLOCK) ? (int)(q - base) : ROW_BLOCK;
        const u128 key = key_n;
        const uint4 A = A_n, B = B_n;
        const bool more = i + stride < q;
        // keys stream (non-temporal): 3.376 vs 3.401 ms at C5, alternating
        // processes (profiles/r06/c5_ntkeys/)
        if (more) key_n = ld128_nt(keys + i + stride);
        if (i < q) {
            uint32_t sn = 0, so = 0, has = 0, m = 0;
            const bool settled =
                use_cd && cd_lookup(cd, key, A, B, n_old, n_new, no, nn, so, sn, has, m);
            if (!settled) {
                // Both searches are issued together: deriving the new successor
                // from a verified old->new mapping saves a search for ~98 % of
                // keys but serialises it behind the old one for the rest, and
                // with 64 lanes a wave almost always holds one of those
                // (measured 7 % slower).
                sn = Searcher<DIR>::find(sv_new, lds_new, key);
                if (CHURN) so = Searcher<DIR>::find(sv_old, lds_old, key);
                // holders: old n-window mapped to the new ring, or the caller's list
                uint32_t hv[CX_MAX_NSUCC];
                // the old window's o2n entries are contiguous: five aligned 16-B
                // loads cover [so, so + no) for no <= 17 (one request each instead
                // of one dword request per entry); the window may not wrap or pass
                // the end
                const uint32_t ob = so & ~3u;
                const bool wide = CHURN && o2n_al && (size_t)ob + 20 <= n_old;
                if (wide) {
                    const uint4 *w4 = reinterpret_cast<const uint4 *>(old_to_new + ob);
                    uint32_t w[20];
#pragma unroll
                    for (int t = 0; t < 5; ++t) {
                        const uint4 x = w4[t];
                        w[4 * t] = x.x;
                        w[4 * t + 1] = x.y;
                        w[4 * t + 2] = x.z;
                        w[4 * t + 3] = x.w;
                    }
                    const uint32_t sh = so & 3u;
#pragma unroll
                    for (int j = 0; j < CX_MAX_NSUCC; ++j)
                        hv[j] = j >= no ? CX_NONE
                                        : (sh == 0 ? w[j] : sh == 1 ? w[j + 1] : sh == 2 ? w[j + 2]
                                                                               : w[j + 3]);
                }
#pragma unroll
                for (int j = 0; j < CX_MAX_NSUCC; ++j) {
                    if (wide) break;
                    uint32_t hj = CX_NONE;
                    if (j < no) {
                        if (CHURN) {
                            uint32_t o = so + (uint32_t)j;
                            if (o >= n_old) o -= n_old;
                            hj = old_to_new[o];
                        } else {
                            hj = holders[i * (size_t)nh + j];
                        }
                    }
                    hv[j] = hj;
                }
                // pass 1: which new-list ranks already hold the key, and which
                // holders are misplaced: any value but CX_NONE is a holder; one
                // that is not a ring index is never in the new list (oracle
                // misplaced_one)
#pragma unroll
                for (int j = 0; j < CX_MAX_NSUCC; ++j) {
                    const uint32_t hj = hv[j];
                    if (hj == CX_NONE) continue;
                    const uint32_t r = hj >= n_new ? 0xFFFFFFFFu
                                                   : (hj >= sn ? hj - sn : hj + n_new - sn);
                    if (r < (uint32_t)nn) has |= 1u << r;
                    else if (j < nslots) m |= 1u << j;
                }
            }
            s_sn[threadIdx.x] = sn;
            s_so[threadIdx.x] = so;
            count[i] = (uint8_t)nn;
            if (CHURN && old_lists) old_count[i] = (uint8_t)no;
            // pass 2: misplaced holders in rank order take the first lacking
            // ranks (the row is 0xFF already: most keys have none)
            uint8_t *tg = stage_t + threadIdx.x * nslots;
            uint32_t mm = m, free_ranks = ~has & full;
            while (mm && free_ranks) {
                tg[__builtin_ctz(mm)] = (uint8_t)__builtin_ctz(free_ranks);
                mm &= mm - 1u;
                free_ranks &= free_ranks - 1u;
            }
            mask[i] = (uint16_t)m;
        }
        if (use_cd && more) cd_fetch(cd, key_n, A_n, B_n);
        __syncthreads();
        // new lists (sn + j mod n_new, j < nn) and old lists (so + j mod
        // n_old, j < no <= n_old: one wrap at most) straight from the successors
        flush_window(s_sn, new_lists, base, cnt, nlist, nn, n_new);
        if (CHURN && old_lists) flush_window(s_so, old_lists, base, cnt, nlist, no, n_old);
        flush_rows_refill(stage_t, target, base, cnt, nslots);
        __syncthreads();
    }
}

hipError_t misplaced_churn(const SearchView &sv_old, const SearchView &sv_new,
                           const uint32_t *old_to_new, const cell128 *keys, size_t q, int n,
                           uint32_t *lists, uint8_t *count, uint16_t *mask, uint8_t *target,
                           const ChurnDirArgs *cda, hipStream_t s, uint32_t *old_lists,
                           uint8_t *old_count) {
    if (q == 0) return hipSuccess;
    if ((old_lists == nullptr) != (old_count == nullptr)) return hipErrorInvalidValue;
    ChurnDir cd = {};
    if (cda) cd = ChurnDir{cda->cd, cda->kb, sv_old.ring, sv_new.ring, cda->ok};
    const unsigned g = cx_grid(q, ROW_BLOCK, 8192);
    if (cda && sv_new.dir && sv_old.dir)
        k_misplaced<true, true, true><<<g, ROW_BLOCK, 0, s>>>(
            sv_new, sv_old, old_to_new, nullptr, 0, keys, q, n, lists, count, mask, target, cd,
            old_lists, old_count);
    else if (sv_new.dir && sv_old.dir)
        k_misplaced<true, true><<<cx_grid(q, ROW_BLOCK, 8192), ROW_BLOCK, 0, s>>>(
            sv_new, sv_old, old_to_new, nullptr, 0, keys, q, n, lists, count, mask, target, cd,
            old_lists, old_count);
    else
        k_misplaced<true, false><<<cx_grid(q, ROW_BLOCK, 256), ROW_BLOCK, 0, s>>>(
            sv_new, sv_old, old_to_new, nullptr, 0, keys, q, n, lists, count, mask, target, cd,
            old_lists, old_count);
    return hipGetLastError();
}

// ---- churn directory build (see ChurnDir) ----------------------------------
// dflag[o] = old peer o departed; jflag[p] = new peer p joined (no old peer
// maps to it).  Both arrays carry a trailing 0 so their exclusive scans end in
// the totals.
__global__ void k_cd_flags(const uint32_t *o2n, uint32_t n_old, uint32_t n_new, uint32_t *dflag,
                           uint32_t *jflag) {
    for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < n_old;
         o += (size_t)gridDim.x * blockDim.x) {
        const uint32_t u = o2n[o];
        dflag[o] = u == CX_NONE;
        if (u < n_new) jflag[u] = 0;
    }
}

// Merged entry of old peer o: survivor u = o2n[o] sits at u + (departed
// before o); a departed one at (#new IDs below it) + (departed before o).
__global__ void k_cd_place_old(SearchView sv_new, const cell128 *ring_old, const uint32_t *o2n,
                               const uint32_t *dex, uint32_t n_old, uint32_t n_new,
                               cell128 *mid, uint32_t *mso, uint32_t *msn, uint8_t *mtag) {
    for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < n_old;
         o += (size_t)gridDim.x * blockDim.x) {
        const u128 id = ld128(ring_old + o);
        const uint32_t u = o2n[o];
        uint32_t c = u, tag = 3;
        if (u == CX_NONE) {
            c = dir_lower_bound(sv_new, id);
            tag = 1;
        }
        const size_t m = (size_t)c + dex[o];
        st128(mid + m, id);
        mso[m] = (uint32_t)o;
        msn[m] = c == n_new ? 0u : c;
        mtag[m] = (uint8_t)tag;
    }
}

// Merged entry of joiner p: p + (departed old peers below its ID).
__global__ void k_cd_place_join(SearchView sv_old, const cell128 *ring_new, const uint32_t *jex,
                                uint32_t n_old, uint32_t n_new, cell128 *mid, uint32_t *mso,
                                uint32_t *msn, uint8_t *mtag) {
    for (size_t p = blockIdx.x * (size_t)blockDim.x + threadIdx.x; p < n_new;
         p += (size_t)gridDim.x * blockDim.x) {
        if (jex[p + 1] == jex[p]) continue;  // survivor: placed from the old side
        const u128 id = ld128(ring_new + p);
        const uint32_t c = dir_lower_bound(sv_old, id);  // old IDs below it
        const size_t m = (size_t)p + c - (p - jex[p]);
        st128(mid + m, id);
        mso[m] = c == n_old ? 0u : c;
        msn[m] = (uint32_t)p;
        mtag[m] = 2;
    }
}

// lo[b] = first merged entry whose bucket is >= b (k_dir_lo on the merged IDs).
__global__ void k_cd_lo(const cell128 *mid, uint32_t M, int kb, uint32_t *lo) {
    const size_t nb = (size_t)1 << kb;
    for (size_t j = blockIdx.x * (size_t)blockDim.x + threadIdx.x; j <= M;
         j += (size_t)gridDim.x * blockDim.x) {
        const long long pb = j == 0 ? -1 : (long long)top_bits(ld128(mid + j - 1), kb);
        const long long cb = j == M ? (long long)nb : (long long)top_bits(ld128(mid + j), kb);
        for (long long b = pb + 1; b <= cb; ++b) lo[b] = (uint32_t)j;
    }
}

__global__ void k_cd_pack(const cell128 *mid, const uint32_t *mso, const uint32_t *msn,
                          const uint8_t *mtag, const uint32_t *lo, uint32_t M, int kb, uint4 *cd) {
    const size_t nb = (size_t)1 << kb;
    for (size_t b = blockIdx.x * (size_t)blockDim.x + threadIdx.x; b < nb;
         b += (size_t)gridDim.x * blockDim.x) {
        const uint32_t a = lo[b], z = lo[b + 1];
        const uint32_t cnt = z - a < 3 ? z - a : 3;
        const uint32_t m0 = a < M ? a : 0;
        const uint64_t h0 = cnt >= 1 ? mid_bits(ld128(mid + a), kb) : 0;
        const uint64_t h1 = cnt >= 2 ? mid_bits(ld128(mid + a + 1), kb) : 0;
        uint32_t om = 0, nm = 0;  // old / new masks of the 32 merged entries
        uint32_t m = m0;
        for (int j = 0; j < 32; ++j) {
            const uint32_t g = mtag[m];
            om |= (g & 1u) << j;
            nm |= (g >> 1) << j;
            if (++m == M) m = 0;
        }
        const uint64_t h1c = (h1 & ~3ull) | cnt;
        cd[2 * b] = make_uint4((uint32_t)h0, (uint32_t)(h0 >> 32), mso[m0], msn[m0]);
        cd[2 * b + 1] = make_uint4(om, nm, (uint32_t)h1c, (uint32_t)(h1c >> 32));
    }
}

// Compares a caller's old_to_new with cx_churn's (ok = 1 iff equal).
__global__ void k_cd_same(const uint32_t *a, const uint32_t *b, size_t n, uint32_t *ok) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        if (a[i] != b[i]) *ok = 0;
}

size_t churn_dir_workspace_bytes(size_t n_old, size_t n_new) {
    const size_t M = n_old + n_new;  // upper bound of the merged size
    return ((n_old + 1) + (n_new + 1)) * 4 + M * (16 + 4 + 4 + 1) + 64 * 6;
}

hipError_t churn_dir_build(const SearchView &sv_old, const SearchView &sv_new,
                           const uint32_t *o2n, int kb, void *ws, uint32_t *lo, uint4 *cd,
                           uint32_t *scan_ws, uint32_t *M_out, hipStream_t s) {
    const uint32_t n_old = sv_old.ev.n, n_new = sv_new.ev.n;
    const size_t Mcap = (size_t)n_old + n_new;
    char *w = static_cast<char *>(ws);
    auto carve = [&](size_t bytes) {
        char *r = w;
        w += (bytes + 63) & ~(size_t)63;
        return r;
    };
    uint32_t *dflag = reinterpret_cast<uint32_t *>(carve((n_old + 1) * 4));
    uint32_t *jflag = reinterpret_cast<uint32_t *>(carve((n_new + 1) * 4));
    cell128 *mid = reinterpret_cast<cell128 *>(carve(Mcap * 16));
    uint32_t *mso = reinterpret_cast<uint32_t *>(carve(Mcap * 4));
    uint32_t *msn = reinterpret_cast<uint32_t *>(carve(Mcap * 4));
    uint8_t *mtag = reinterpret_cast<uint8_t *>(carve(Mcap));
    hipError_t e = fill_u32(jflag, n_new, 1u, s);
    if (e == hipSuccess) e = hipMemsetAsync(jflag + n_new, 0, 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(dflag + n_old, 0, 4, s);
    if (e != hipSuccess) return e;
    k_cd_flags<<<cx_grid(n_old, 256), 256, 0, s>>>(o2n, n_old, n_new, dflag, jflag);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = exclusive_scan(dflag, (size_t)n_old + 1, scan_ws, s)) != hipSuccess) return e;
    if ((e = exclusive_scan(jflag, (size_t)n_new + 1, scan_ws, s)) != hipSuccess) return e;
    uint32_t D = 0;
    if ((e = hipMemcpyAsync(&D, dflag + n_old, 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
        return e;
    if ((e = hipStreamSynchronize(s)) != hipSuccess) return e;
    const uint32_t M = n_new + D;
    *M_out = M;
    k_cd_place_old<<<cx_grid(n_old, 256), 256, 0, s>>>(sv_new, sv_old.ring, o2n, dflag, n_old,
                                                      n_new, mid, mso, msn, mtag);
    k_cd_place_join<<<cx_grid(n_new, 256), 256, 0, s>>>(sv_old, sv_new.ring, jflag, n_old, n_new,
                                                       mid, mso, msn, mtag);
    k_cd_lo<<<cx_grid((size_t)M + 1, 256), 256, 0, s>>>(mid, M, kb, lo);
    k_cd_pack<<<cx_grid((size_t)1 << kb, 256), 256, 0, s>>>(mid, mso, msn, mtag, lo, M, kb, cd);
    return hipGetLastError();
}

hipError_t churn_dir_same(const uint32_t *a, const uint32_t *b, size_t n, uint32_t *ok,
                          hipStream_t s) {
    hipError_t e = fill_u32(ok, 1, 1u, s);
    if (e != hipSuccess || n == 0) return e;
    k_cd_same<<<cx_grid(n, 256, 4096), 256, 0, s>>>(a, b, n, ok);
    return hipGetLastError();
}

hipError_t misplaced_holders(const SearchView &sv, const uint32_t *holders, int nh,
                             const cell128 *keys, size_t q, int n, uint32_t *lists,
                             uint8_t *count, uint16_t *mask, uint8_t *target, hipStream_t s) {
    if (q == 0) return hipSuccess;
    if (sv.dir)
        k_misplaced<false, true><<<cx_grid(q, ROW_BLOCK, 8192), ROW_BLOCK, 0, s>>>(
            sv, sv, nullptr, holders, nh, keys, q, n, lists, count, mask, target, ChurnDir{});
    else
        k_misplaced<false, false><<<cx_grid(q, ROW_BLOCK, 512), ROW_BLOCK, 0, s>>>(
            sv, sv, nullptr, holders, nh, keys, q, n, lists, count, mask, target, ChurnDir{});
    return hipGetLastError();
}

// ===========================================================================
// a2: InBetween on raw uint256 operands (key.h:103-131).
// ===========================================================================
struct u256v {
    uint64_t w[4];
};
__device__ __forceinline__ int cmp256(const u256v &a, const u256v &b) {
#pragma unroll
    for (int i = 3; i >= 0; --i) {
        if (a.w[i] < b.w[i]) return -1;
        if (a.w[i] > b.w[i]) return 1;
    }
    return 0;
}
__global__ void k_in_between(const cx_u256 *v, const cx_u256 *lb, const cx_u256 *ub, size_t q,
                             int inclusive, uint8_t *out) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < q;
         i += (size_t)gridDim.x * blockDim.x) {
        u256v V, L, U;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            V.w[j] = v[i].w[j];
            L.w[j] = lb[i].w[j];
            U.w[j] = ub[i].w[j];
        }
        bool r;
        if (cmp256(L, U) == 0) {
            r = cmp256(V, U) == 0;
        } else {
            u256v ml = {{L.w[0], L.w[1], 0, 0}}, mu = {{U.w[0], U.w[1], 0, 0}},
                  mv = {{V.w[0], V.w[1], 0, 0}};
            if (cmp256(L, U) < 0)
                r = inclusive ? (cmp256(ml, mv) <= 0 && cmp256(mv, U) <= 0)
                              : (cmp256(ml, mv) < 0 && cmp256(mv, U) < 0);
            else
                r = inclusive ? !(cmp256(mu, mv) < 0 && cmp256(mv, ml) < 0)
                              : !(cmp256(mu, mv) <= 0 && cmp256(mv, ml) <= 0);
        }
        out[i] = r ? 1 : 0;
    }
}

hipError_t in_between(const cx_u256 *v, const cx_u256 *lb, const cx_u256 *ub, size_t q,
                      int inclusive, uint8_t *out, hipStream_t s) {
    if (q == 0) return hipSuccess;
    k_in_between<<<cx_grid(q, 256), 256, 0, s>>>(v, lb, ub, q, inclusive, out);
    return hipGetLastError();
}

// ===========================================================================
// Synthetic keys.
// ===========================================================================
__global__ void k_splitmix(cell128 *out, size_t count, uint64_t seed, uint64_t offset) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t c = offset + i;
        cell128 v;
        v.lo = splitmix64(seed, 2 * c);
        v.hi = splitmix64(seed, 2 * c + 1);
        out[i] = v;
    }
}

hipError_t fill_splitmix(cell128 *out, size_t count, uint64_t seed, uint64_t offset,
                         hipStream_t s) {
    if (count == 0) return hipSuccess;
    k_splitmix<<<cx_grid(count, 256), 256, 0, s>>>(out, count, seed, offset);
    return hipGetLastError();
}

hipError_t iota(uint32_t *t, size_t n, uint32_t base, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_iota<<<cx_grid(n, 256), 256, 0, s>>>(t, n, base);
    return hipGetLastError();
}

hipError_t fill_u32(uint32_t *t, size_t n, uint32_t v, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_fill_u32<<<cx_grid(n, 256), 256, 0, s>>>(t, n, v);
    return hipGetLastError();
}

// ===========================================================================
// a1: batched UUIDv5 (RFC 4122, DNS namespace) of plaintext names -- the
// peer/key ID construction of GenerateSha1Hash (key.h:29-33) + uint256_t(uuid)
// big-endian (key.h:77-78).  One lane per name; SHA-1 (FIPS 180-4) over
// ns || name with a 16-word rolling schedule.
// ===========================================================================
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

__global__ void k_uuid5(const uint8_t *bytes, const uint64_t *offs, size_t count, cell128 *out) {
    const uint8_t ns[16] = {0x6b, 0xa7, 0xb8, 0x10, 0x9d, 0xad, 0x11, 0xd1,
                            0x80, 0xb4, 0x00, 0xc0, 0x4f, 0xd4, 0x30, 0xc8};
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t o = offs[i], len = offs[i + 1] - o;
        const uint64_t total = 16 + len;
        const uint64_t nblk = (total + 8) / 64 + 1;
        const uint64_t bits = total * 8;
        uint32_t h0 = 0x67452301u, h1 = 0xEFCDAB89u, h2 = 0x98BADCFEu, h3 = 0x10325476u,
                 h4 = 0xC3D2E1F0u;
        for (uint64_t blk = 0; blk < nblk; ++blk) {
            uint32_t w[16];
            for (int j = 0; j < 16; ++j) {
                uint32_t v = 0;
                for (int b = 0; b < 4; ++b) {
                    const uint64_t p = blk * 64 + (uint64_t)(j * 4 + b);
                    uint32_t c;
                    if (p < 16) c = ns[p];
                    else if (p < total) c = bytes[o + p - 16];
                    else if (p == total) c = 0x80;
                    else if (blk == nblk - 1 && p >= nblk * 64 - 8)
                        c = (uint32_t)(bits >> (8 * (nblk * 64 - 1 - p))) & 0xFF;
                    else c = 0;
                    v = (v << 8) | c;
                }
                w[j] = v;
            }
            uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
#pragma unroll
            for (int t = 0; t < 80; ++t) {
                uint32_t wt;
                if (t < 16) {
                    wt = w[t];
                } else {
                    wt = rotl32(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15], 1);
                    w[t & 15] = wt;
                }
                uint32_t f, k;
                if (t < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
                else if (t < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
                else if (t < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
                else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
                const uint32_t tmp = rotl32(a, 5) + f + e + k + wt;
                e = d; d = c; c = rotl32(b, 30); b = a; a = tmp;
            }
            h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
        }
        h1 = (h1 & 0xFFFF0FFFu) | 0x00005000u;  // version 5 (byte 6 high nibble)
        h2 = (h2 & 0x3FFFFFFFu) | 0x80000000u;  // RFC 4122 variant (byte 8)
        cell128 r;
        r.hi = ((uint64_t)h0 << 32) | h1;
        r.lo = ((uint64_t)h2 << 32) | h3;
        out[i] = r;
    }
}

hipError_t uuid5(const uint8_t *bytes, const uint64_t *offs, size_t count, cell128 *out,
                 hipStream_t s) {
    if (count == 0) return hipSuccess;
    k_uuid5<<<cx_grid(count, 256), 256, 0, s>>>(bytes, offs, count, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Hex codec of keys on the wire.  Parse: ChordKey(hex, hashed = true) =
// uint256("0x" + s) (key.h:73-75) -- hex digits of either case, no prefix;
// the engine keeps the value mod 2^128 (what every ring comparison reads,
// key.h:103-131) and flags ok = 2 when the raw uint256 (which wraps mod
// 2^256, Boost's unchecked cpp_int) is >= 2^128, i.e. bits 128..255 of it
// are not all zero.  Format: std::string(key) = IntToHexStr (key.h:41-47):
// lowercase, no leading zeros, "0" for zero; one 32-byte slot per key.
// ---------------------------------------------------------------------------
__global__ void k_hex_parse(const uint8_t *bytes, const uint64_t *offs, size_t count,
                            cell128 *out, uint8_t *ok) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t o = offs[i], e = offs[i + 1];
        u128 v = 0, hi = 0;  // raw value = hi:v mod 2^256
        bool good = e > o;
        for (uint64_t k = o; k < e; ++k) {
            const uint32_t c = bytes[k];
            uint32_t d;
            if (c >= '0' && c <= '9') d = c - '0';
            else if (c >= 'a' && c <= 'f') d = c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') d = c - 'A' + 10;
            else { good = false; d = 0; }
            hi = (hi << 4) | (v >> 124);
            v = (v << 4) | d;
        }
        st128(out + i, good ? v : (u128)0);
        ok[i] = good ? (hi != 0 ? 2 : 1) : 0;
    }
}

__global__ void k_hex_format(const cell128 *keys, size_t count, uint4 *out, uint8_t *len) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x) {
        const u128 v = ld128(keys + i);
        const int nd = v == 0 ? 1 : msb128(v) / 4 + 1;
        uint32_t w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            uint32_t word = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int pos = 4 * j + b;
                if (pos < nd) {
                    const uint32_t d = (uint32_t)bits64(v, 4 * (nd - 1 - pos)) & 15u;
                    word |= (d < 10 ? '0' + d : 'a' + d - 10) << (8 * b);
                }
            }
            w[j] = word;
        }
        out[2 * i] = make_uint4(w[0], w[1], w[2], w[3]);
        out[2 * i + 1] = make_uint4(w[4], w[5], w[6], w[7]);
        len[i] = (uint8_t)nd;
    }
}

hipError_t hex_parse(const uint8_t *bytes, const uint64_t *offs, size_t count, cell128 *out,
                     uint8_t *ok, hipStream_t s) {
    if (count == 0) return hipSuccess;
    k_hex_parse<<<cx_grid(count, 256), 256, 0, s>>>(bytes, offs, count, out, ok);
    return hipGetLastError();
}

hipError_t hex_format(const cell128 *keys, size_t count, char *out, uint8_t *len, hipStream_t s) {
    if (count == 0) return hipSuccess;
    k_hex_format<<<cx_grid(count, 256), 256, 0, s>>>(keys, count, reinterpret_cast<uint4 *>(out),
                                                     len);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Rabin IDA (DHash payload coding): src/ida/ida.cpp and
// src/ida/matrix_math.cpp.  Ragged blocks; block b has S_b = ceil(len_b / m)
// segments of m values and seg[b] = prefix sum of S_b.
//   encode: fragment i value s = sum_k a^k v_k mod p, a = i + 1
//           (ConstructEncodingMatrix + InnerProduct, ida.cpp:59-73)
//   decode: inverse Vandermonde of the fragment indices (VandermondeInverse,
//           matrix_math.cpp:103-168, int arithmetic wrapping as compiled) times
//           the fragment rows, read segment-wise, trailing zeros dropped
//           (ida.cpp:120-162).
// HBM-bound byte/integer streams: one lane per segment, m-value rows read and
// written coalesced across the wave; no MFMA (values are mod p, 14 MACs/byte).
// ---------------------------------------------------------------------------
constexpr int IDA_MAX_N = 32;

// Bounds checks of the decode path's index arithmetic (run_of, run_start,
// the block cursor, fragment offsets): a violation skips the access and sets
// a bit in the call's error word, which cx_ida_decode reports.
enum : uint32_t {
    IDA_ERR_RUN_OF = 1u,      // run_of[b] >= runs
    IDA_ERR_RUN_START = 2u,   // run_start[r] >= blocks
    IDA_ERR_CURSOR = 4u,      // block cursor past the last block / segment outside it
    IDA_ERR_RUN_INDEX = 8u,   // k_ida_run_index produced r >= runs
    IDA_ERR_GUARD = 16u       // the guard words after the inverses were overwritten
};

// Block owning global segment g: largest b with seg[b] <= g.
__device__ __forceinline__ size_t seg_block(const uint64_t *seg, size_t blocks, uint64_t g) {
    size_t lo = 0, hi = blocks;  // seg[lo] <= g < seg[hi]
    while (hi - lo > 1) {
        const size_t mid = (lo + hi) >> 1;
        if (seg[mid] <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

// x mod p via a float reciprocal when the quotient is < 2^21 (every use
// below: encode sums < m (p-1) 255, decode sums < m (p-1) 65535 with
// quotient < m 65535): the estimate is off by at most one, fixed up with
// two selects; 24-bit multiply, all full-rate VALU.
__device__ __forceinline__ uint32_t modp_f(uint32_t x, uint32_t p, float inv_p) {
    const uint32_t q = (uint32_t)((float)x * inv_p);
    int32_t r = (int32_t)(x - __umul24(q, p));
    r += r < 0 ? (int32_t)p : 0;
    r -= r >= (int32_t)p ? (int32_t)p : 0;
    return (uint32_t)r;
}

// x mod p with one fix-up: the biased estimate q = floor(x/p - 1/2 +- err) is
// floor(x/p) or one less while |err| < 1/2, i.e. x/p < 2^20 (encode: x/p <
// m 255; decode with m <= 12: x/p < m 65535); r in [0, 2p) then needs one
// unsigned min.  cvt, fma, cvt, mul24, sub, sub, min: 7 full-rate VALU.
__device__ __forceinline__ uint32_t modp_fast(uint32_t x, uint32_t p, float inv_p) {
    const uint32_t q = (uint32_t)__builtin_fmaf((float)x, inv_p, -0.5f);  // < 0 -> 0
    const uint32_t r = x - __umul24(q, p);
    return r < r - p ? r : r - p;
}

typedef unsigned short cx_us2 __attribute__((ext_vector_type(2)));

// Encoding rows in LDS, bytes packed for v_dot4_u32_u8: row i = 8 words of
// low bytes of E[i][0..31] then 8 words of high bytes (E < 46340 < 2^16).
constexpr int IDA_EROW = 16;

// Per-lane cursor over blocks: the block holding segment g and its bounds,
// reloaded only when g passes the block's end (segments only move forward).
struct BlockCursor {
    size_t b;
    uint64_t sb, sb1;  // seg[b], seg[b+1]
    uint64_t ob, ob1;  // offs[b], offs[b+1] (encode only)
};

template <bool OFFS>
__device__ __forceinline__ void cursor_init(BlockCursor &k, const uint64_t *seg,
                                            const uint64_t *offs, size_t b) {
    k.b = b;
    k.sb = seg[b];
    k.sb1 = seg[b + 1];
    if (OFFS) {
        k.ob = offs[b];
        k.ob1 = offs[b + 1];
    }
}

template <bool OFFS>
__device__ __forceinline__ void cursor_advance(BlockCursor &k, const uint64_t *seg,
                                               const uint64_t *offs, uint64_t g) {
    while (g >= k.sb1) {
        ++k.b;
        k.sb = k.sb1;
        k.sb1 = seg[k.b + 1];
        if (OFFS) {
            k.ob = k.ob1;
            k.ob1 = offs[k.b + 1];
        }
    }
}

// Each wave takes a contiguous range of 64-segment chunks.  The bytes of the
// next D chunks (each one contiguous span of data) are in flight in registers
// while chunk c is computed (D-slot ring, fully unrolled so every slot lives in
// registers); they pass through LDS so each lane can take its own m bytes as
// packed words for v_dot4_u32_u8 (4 byte-products per instruction).
// PRE = dwords per lane per chunk: a chunk spans <= 64 m bytes + alignment,
// i.e. <= 16 m + 1 words: PRE 3 covers m <= 11 (DHash's 10), PRE 8 any m.
template <int PRE>
struct EncSlot {
    uint64_t segb, S, s, span;
    uint32_t off, words;
    int have;
    bool live;
    uint32_t pre[PRE];
};

template <int PRE, int D>
__global__ __launch_bounds__(256) void k_ida_encode(const uint8_t *data, const uint64_t *offs,
                                                    const uint64_t *seg, size_t blocks, int n,
                                                    int m, uint32_t p, float inv_p,
                                                    uint16_t *frags) {
    __shared__ __attribute__((aligned(16))) uint32_t Epk[IDA_MAX_N * IDA_EROW];
    __shared__ uint32_t stage[256 / 64][IDA_MAX_N * 16 + 12];  // a wave's bytes (<= 64 m)
    for (int t = threadIdx.x; t < n * 8; t += blockDim.x) {
        const int i = t >> 3, w = t & 7;
        uint32_t lo = 0, hi = 0, e = 1;
        for (int k = 0; k < 4 * w + 4; ++k) {  // e = (i+1)^k mod p
            if (k >= 4 * w && k < m) {
                lo |= (e & 0xFFu) << (8 * (k - 4 * w));
                hi |= (e >> 8) << (8 * (k - 4 * w));
            }
            e = (e * (uint32_t)(i + 1)) % p;
        }
        Epk[i * IDA_EROW + w] = lo;
        Epk[i * IDA_EROW + 8 + w] = hi;
    }
    __syncthreads();
    const bool hi_any = p > 256;
    const int nw = (m + 3) >> 2;
    const int lane = threadIdx.x & 63;
    uint32_t *st = stage[threadIdx.x >> 6];
    const uint64_t total = seg[blocks];
    const uint64_t nbytes = offs[blocks];
    const uint64_t chunks = (total + 63) / 64;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t cpw = (chunks + waves - 1) / waves;
    const uint64_t c0 = wave * cpw, c1 = c0 + cpw < chunks ? c0 + cpw : chunks;
    if (c0 >= c1) return;  // wave-uniform, after the only block barrier
    BlockCursor cur;
    cursor_init<true>(cur, seg, offs, seg_block(seg, blocks, c0 * 64));

    EncSlot<PRE> sl[D];
    // descriptor + loads of chunk c into slot x (chunks are issued in order,
    // so the per-lane block cursor only moves forward)
    auto issue = [&](EncSlot<PRE> &x, uint64_t c) {
        const uint64_t g = c * 64 + lane;
        x.live = g < total;
        cursor_advance<true>(cur, seg, offs, x.live ? g : total - 1);
        x.s = (x.live ? g : total - 1) - cur.sb;
        x.segb = cur.sb;
        x.S = cur.sb1 - cur.sb;
        const uint64_t my_lo = cur.ob + x.s * m;
        uint64_t my_hi = my_lo + m;
        if (my_hi > cur.ob1) my_hi = cur.ob1;
        x.span = __shfl(my_lo, 0) & ~3ull;
        const uint64_t span_hi = __shfl(my_hi, 63);
        x.words = (uint32_t)((span_hi - x.span + 3) >> 2);
        x.off = (uint32_t)(my_lo - x.span);
        x.have = (int)(my_hi - my_lo);
#pragma unroll
        for (int t = 0; t < PRE; ++t) {
            const uint32_t w = lane + 64 * t;
            const uint64_t at = x.span + 4ull * w;
            uint32_t v = 0;
            if (w < x.words) {
                if (at + 4 <= nbytes) {
                    v = *reinterpret_cast<const uint32_t *>(data + at);
                } else {
                    for (int k = 0; k < 4; ++k)
                        if (at + k < nbytes) v |= (uint32_t)data[at + k] << (8 * k);
                }
            }
            x.pre[t] = v;
        }
    };
#pragma unroll
    for (int k = 0; k < D; ++k)
        if (c0 + k < c1) issue(sl[k], c0 + k);
    for (uint64_t cb = c0; cb < c1; cb += D) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const uint64_t c = cb + k;
            if (c >= c1) break;  // wave-uniform
            // take over slot k, then refill it with chunk c + D
            const uint64_t segb = sl[k].segb, S = sl[k].S, sg = sl[k].s;
            const uint32_t off = sl[k].off, words = sl[k].words;
            const int have = sl[k].have;
            const bool live = sl[k].live;
#pragma unroll
            for (int t = 0; t < PRE; ++t)
                if (lane + 64 * t < (int)words) st[lane + 64 * t] = sl[k].pre[t];
            if (c + D < c1) issue(sl[k], c + D);  // loads overlap this chunk's math
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // this lane's segment as packed words W[0..nw), bytes past `have` zero
            const uint32_t bw = off >> 2, sh = off & 3;
            uint32_t W[8];
            uint32_t prev = st[bw];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (j < nw) {
                    const uint32_t nxt = st[bw + j + 1];
                    uint32_t x = __builtin_amdgcn_alignbyte(nxt, prev, sh);
                    const int valid = have - 4 * j;
                    x &= valid >= 4 ? 0xFFFFFFFFu
                                    : (valid <= 0 ? 0u : (1u << (8 * valid)) - 1u);
                    W[j] = x;
                    prev = nxt;
                } else {
                    W[j] = 0;
                }
            }
            if (live) {
                uint16_t *out = frags + (uint64_t)n * segb + sg;
                for (int i = 0; i < n; ++i) {
                    const uint4 *er = reinterpret_cast<const uint4 *>(Epk + i * IDA_EROW);
                    const uint4 l0 = er[0];
                    uint32_t acc = __builtin_amdgcn_udot4(l0.x, W[0], 0u, false);
                    if (nw > 1) acc = __builtin_amdgcn_udot4(l0.y, W[1], acc, false);
                    if (nw > 2) acc = __builtin_amdgcn_udot4(l0.z, W[2], acc, false);
                    if (nw > 3) acc = __builtin_amdgcn_udot4(l0.w, W[3], acc, false);
                    if (nw > 4) {
                        const uint4 l1 = er[1];
                        acc = __builtin_amdgcn_udot4(l1.x, W[4], acc, false);
                        if (nw > 5) acc = __builtin_amdgcn_udot4(l1.y, W[5], acc, false);
                        if (nw > 6) acc = __builtin_amdgcn_udot4(l1.z, W[6], acc, false);
                        if (nw > 7) acc = __builtin_amdgcn_udot4(l1.w, W[7], acc, false);
                    }
                    if (hi_any) {  // E >= 256: high bytes times 256
                        const uint4 h0 = er[2], h1 = er[3];
                        uint32_t ah = __builtin_amdgcn_udot4(h0.x, W[0], 0u, false);
                        ah = __builtin_amdgcn_udot4(h0.y, W[1], ah, false);
                        ah = __builtin_amdgcn_udot4(h0.z, W[2], ah, false);
                        ah = __builtin_amdgcn_udot4(h0.w, W[3], ah, false);
                        if (nw > 4) {
                            ah = __builtin_amdgcn_udot4(h1.x, W[4], ah, false);
                            ah = __builtin_amdgcn_udot4(h1.y, W[5], ah, false);
                            ah = __builtin_amdgcn_udot4(h1.z, W[6], ah, false);
                            ah = __builtin_amdgcn_udot4(h1.w, W[7], ah, false);
                        }
                        acc += ah << 8;  // total <= m (p-1) 255 < 2^29
                    }
                    out[(uint64_t)i * S] = (uint16_t)modp_f(acc, p, inv_p);
                }
            }
            __builtin_amdgcn_wave_barrier();  // stage reused by the next chunk
        }
    }
}

// One thread per run of blocks sharing an index list: the run's inverse
// Vandermonde (m x m, row-major as the reference returns it).  flag = 1 on
// success, 0 when a denominator has no inverse ("N is not invertible").
__device__ __forceinline__ int32_t cmod(int32_t x, int32_t p) { return (x % p + p) % p; }

__global__ void k_ida_inverse(const uint8_t *idx, const uint32_t *run_start, size_t runs,
                              size_t blocks, int m, int32_t p, int32_t *inv, uint8_t *okf,
                              uint32_t *err) {
    for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < runs;
         r += (size_t)gridDim.x * blockDim.x) {
        if (run_start[r] >= blocks) {  // bounds check (never taken on valid runs)
            atomicOr(err, IDA_ERR_RUN_START);
            okf[r] = 0;
            continue;
        }
        const uint8_t *b = idx + (size_t)run_start[r] * m;
        // elementary symmetric sums e_0..e_m of the basis, int32 wrap (uint32 ops)
        uint32_t e[IDA_MAX_N + 1];
        e[0] = 1;
        for (int j = 1; j <= m; ++j) e[j] = 0;
        for (int t = 0; t < m; ++t)
            for (int j = t + 1; j >= 1; --j) e[j] = e[j] + e[j - 1] * (uint32_t)b[t];
        int32_t *out = inv + r * (size_t)m * m;
        bool good = true;
        for (int i = 0; i < m; ++i) {
            const int32_t elt = b[i];
            int32_t prod = 1;
            for (int j = 0; j < m; ++j)
                if (j != i) prod = cmod(prod * (elt - (int32_t)b[j]), p);
            // ModInverse (matrix_math.cpp:66-86)
            int32_t t = 0, nt = 1, rr = p, nr = prod;
            while (nr) {
                const int32_t q = rr / nr;
                int32_t tmp = t;
                t = nt;
                nt = tmp - q * nt;
                tmp = rr;
                rr = nr;
                nr = tmp - q * nr;
            }
            if (rr > 1) {
                good = false;
                break;
            }
            if (t < 0) t += p;
            // numerators (built from the top), reversed, scaled; stored transposed
            int32_t row = 1, sign = -1;
            out[(size_t)(m - 1) * m + i] = cmod(row * t, p);
            for (int j = 1; j < m; ++j) {
                const int32_t a = cmod(row * elt, p);
                row = cmod((int32_t)((uint32_t)a + (uint32_t)sign * e[j]), p);
                out[(size_t)(m - 1 - j) * m + i] = cmod(row * t, p);
                sign = -sign;
            }
        }
        okf[r] = good ? 1 : 0;
    }
}

// Decode: each lane rebuilds one segment (m values) from its m fragment
// values.  When the wave's blocks share one inverse it is staged in LDS as
// u16 pairs and each output takes ceil(m/2) v_dot2_u32_u16 (sums fit 32 bits
// unless WIDE: m (p-1) 65535 >= 2^32, which takes a 64-bit path).
constexpr int IDA_AROW = 16;  // u16-pair words per staged inverse row

// Each wave takes a contiguous range of 64-segment chunks; the fragment values
// of the next D chunks are in flight in registers (D-slot ring, unrolled)
// while chunk c is computed.  FM >= m bounds the per-lane fragment registers.
template <int FM>
struct DecSlot {
    uint64_t s;
    size_t b;
    uint32_t r;
    bool live, ok;
    uint32_t f[FM];
};

template <bool WIDE, int FM, int D, int MF>
__global__ __launch_bounds__(256) void k_ida_decode(const uint16_t *frags, const uint64_t *seg,
                                                    size_t blocks, int m, uint32_t p,
                                                    float inv_p, const int32_t *inv,
                                                    const uint32_t *run_of, size_t runs,
                                                    const uint8_t *okf, uint16_t *out,
                                                    unsigned long long *out_len, uint32_t *err) {
    __shared__ __attribute__((aligned(16))) uint32_t Ainv[256 / 64][IDA_MAX_N * IDA_AROW];
    const int lane = threadIdx.x & 63;
    uint32_t *As = Ainv[threadIdx.x >> 6];
    if (MF) m = MF;  // fixed shape (DHash m = 10): rows unrolled, one-fix-up reduction
    const int nw = (m + 1) >> 1;
    const uint64_t total = seg[blocks];
    const uint64_t chunks = (total + 63) / 64;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t cpw = (chunks + waves - 1) / waves;
    const uint64_t c0 = wave * cpw, c1 = c0 + cpw < chunks ? c0 + cpw : chunks;
    if (c0 >= c1) return;
    size_t bl = seg_block(seg, blocks, c0 * 64);  // per-lane block cursor (moves forward)
    uint64_t bl1 = seg[bl + 1];
    uint32_t staged = 0xFFFFFFFFu;  // run whose inverse is in As
    DecSlot<FM> sl[D];
    auto issue = [&](DecSlot<FM> &x, uint64_t c) {
        const uint64_t g = c * 64 + lane;
        x.live = g < total;
        const uint64_t gl = x.live ? g : total - 1;
        while (bl1 <= gl && bl + 1 < blocks) bl1 = seg[++bl + 1];
        x.b = bl;
        const uint64_t sb = seg[bl];
        bool inb = sb <= gl && gl < bl1;  // the segment lies in the cursor's block
        x.r = run_of[bl];
        if (x.r >= runs) {
            inb = false;
            x.r = 0;
            atomicOr(err, IDA_ERR_RUN_OF);
        } else if (!inb) {
            atomicOr(err, IDA_ERR_CURSOR);
        }
        x.ok = x.live && inb && okf[x.r];
        x.s = gl - sb;
        const uint64_t S = bl1 - sb;
        const uint16_t *fr = frags + (uint64_t)m * sb + x.s;
#pragma unroll
        for (int k = 0; k < FM; ++k) x.f[k] = (x.ok && k < m) ? fr[(uint64_t)k * S] : 0u;
    };
#pragma unroll
    for (int k = 0; k < D; ++k)
        if (c0 + k < c1) issue(sl[k], c0 + k);
    for (uint64_t cb = c0; cb < c1; cb += D) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const uint64_t c = cb + k;
            if (c >= c1) break;  // wave-uniform
            const uint64_t g = c * 64 + lane;
            const size_t b = sl[k].b;
            const uint32_t r = sl[k].r;
            const bool ok = sl[k].ok;
            const uint64_t s = sl[k].s;
            uint32_t f[FM];
#pragma unroll
            for (int q = 0; q < FM; ++q) f[q] = sl[k].f[q];
            if (c + D < c1) issue(sl[k], c + D);  // loads overlap this chunk's math
            const uint32_t r0 = __shfl(r, 0);  // r < runs (checked at issue)
            const bool uniform = __ballot(r != r0) == 0;
            // stage the shared inverse (wave-uniform branch); a run whose
            // inverse failed ("N is not invertible") has rows k_ida_inverse
            // never wrote and no lane that would read them: not staged
            if (uniform && r0 != staged && okf[r0]) {
                __builtin_amdgcn_wave_barrier();  // previous readers of As are done
                const int32_t *A = inv + (size_t)r0 * m * m;
                for (int t = lane; t < m * IDA_AROW; t += 64) {
                    const int j = t / IDA_AROW, w = t - j * IDA_AROW;
                    const uint32_t a0 = 2 * w < m ? (uint32_t)A[j * m + 2 * w] : 0u;
                    const uint32_t a1 = 2 * w + 1 < m ? (uint32_t)A[j * m + 2 * w + 1] : 0u;
                    As[t] = a0 | (a1 << 16);
                }
                staged = r0;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            int last = -1;
            if (ok) {
                uint16_t *o = out + (uint64_t)m * g;  // = m seg[b] + s m
                if (!WIDE && uniform) {
                    uint32_t F[(FM + 1) / 2];
#pragma unroll
                    for (int w = 0; w < (FM + 1) / 2; ++w)
                        F[w] = f[2 * w] | (2 * w + 1 < FM ? f[2 * w + 1] << 16 : 0u);
                    uint32_t cprev = 0;
#pragma unroll
                    for (int j = 0; j < (MF ? MF : FM); ++j) {
                        if (!MF && j >= m) continue;  // uniform; MF: m == MF
                        const uint32_t *ar = As + j * IDA_AROW;
                        uint32_t acc = 0;
#pragma unroll
                        for (int w = 0; w < (FM + 1) / 2; ++w)
                            if (w < nw)
                                acc = __builtin_amdgcn_udot2(__builtin_bit_cast(cx_us2, ar[w]),
                                                             __builtin_bit_cast(cx_us2, F[w]),
                                                             acc, false);
                        // acc / p < m 65535 < 2^20 for m <= 12 (FM = 12)
                        const uint32_t cv = FM <= 12 ? modp_fast(acc, p, inv_p)
                                                     : modp_f(acc, p, inv_p);
                        if (cv) last = j;
                        if ((m & 1) == 0) {  // m even: 4-byte aligned pairs
                            if (j & 1)
                                reinterpret_cast<uint32_t *>(o)[j >> 1] = cprev | (cv << 16);
                            else
                                cprev = cv;
                        } else {
                            o[j] = (uint16_t)cv;
                        }
                    }
                } else {
                    const int32_t *A = inv + (size_t)r * m * m;
                    for (int j = 0; j < m; ++j) {
                        uint32_t cv;
                        if (WIDE) {
                            uint64_t acc = 0;
#pragma unroll
                            for (int q = 0; q < FM; ++q)
                                if (q < m) acc += (uint64_t)(uint32_t)A[j * m + q] * f[q];
                            cv = (uint32_t)(acc % p);
                        } else {
                            uint32_t acc = 0;
#pragma unroll
                            for (int q = 0; q < FM; ++q)
                                if (q < m) acc += (uint32_t)A[j * m + q] * f[q];
                            cv = modp_f(acc, p, inv_p);
                        }
                        o[j] = (uint16_t)cv;
                        if (cv) last = j;
                    }
                }
            }
            // kept length: per block, the highest lane holding a nonzero value
            const uint64_t nz = __ballot(last >= 0);
            const uint64_t above = lane == 63 ? 0ull : nz >> (lane + 1);
            const int nxt = above ? lane + 1 + __builtin_ctzll(above) : 64;
            const size_t bn = __shfl((unsigned long long)b, nxt & 63);
            if (last >= 0 && (nxt == 64 || bn != b))
                atomicMax(out_len + b, (unsigned long long)(s * m + last + 1));
        }
    }
}

// Marks the first block of each run of equal index lists.
__global__ void k_ida_runs(const uint8_t *idx, size_t blocks, int m, uint32_t *flag) {
    for (size_t b = blockIdx.x * (size_t)blockDim.x + threadIdx.x; b < blocks;
         b += (size_t)gridDim.x * blockDim.x) {
        uint32_t f = b == 0 ? 1u : 0u;
        if (b)
            for (int k = 0; k < m; ++k)
                if (idx[b * m + k] != idx[(b - 1) * m + k]) f = 1u;
        flag[b] = f;
    }
}

// run_of[b] = run index (inclusive scan - 1), run_start[run] = first block.
__global__ void k_ida_run_index(const uint32_t *flag_excl, const uint32_t *flag_raw, size_t blocks,
                                size_t runs, uint32_t *run_of, uint32_t *run_start,
                                uint32_t *err) {
    for (size_t b = blockIdx.x * (size_t)blockDim.x + threadIdx.x; b < blocks;
         b += (size_t)gridDim.x * blockDim.x) {
        const uint32_t r = flag_excl[b] + flag_raw[b] - 1;
        if (r >= runs) {
            atomicOr(err, IDA_ERR_RUN_INDEX);
            run_of[b] = 0;
            continue;
        }
        run_of[b] = r;
        if (flag_raw[b]) run_start[r] = (uint32_t)b;
    }
}

// Guard words after the inverse table: any overwrite is reported.
__global__ void k_ida_check_guard(const uint32_t *guard, int words, uint32_t *err) {
    for (int i = threadIdx.x; i < words; i += blockDim.x)
        if (guard[i] != IDA_GUARD_WORD) atomicOr(err, IDA_ERR_GUARD);
}

__global__ void k_ida_mark_failed(const uint32_t *run_of, const uint8_t *okf, size_t blocks,
                                  size_t runs, uint64_t *out_len, uint32_t *err) {
    for (size_t b = blockIdx.x * (size_t)blockDim.x + threadIdx.x; b < blocks;
         b += (size_t)gridDim.x * blockDim.x) {
        const uint32_t r = run_of[b];
        if (r >= runs) {
            atomicOr(err, IDA_ERR_RUN_OF);
            continue;
        }
        if (!okf[r]) out_len[b] = ~0ull;
    }
}

hipError_t ida_mark_failed(const uint32_t *run_of, const uint8_t *okf, size_t blocks,
                           size_t runs, uint64_t *out_len, uint32_t *err, hipStream_t s) {
    if (blocks == 0) return hipSuccess;
    k_ida_mark_failed<<<cx_grid(blocks, 256), 256, 0, s>>>(run_of, okf, blocks, runs, out_len,
                                                          err);
    return hipGetLastError();
}

hipError_t ida_check_guard(const uint32_t *guard, int words, uint32_t *err, hipStream_t s) {
    k_ida_check_guard<<<1, 256, 0, s>>>(guard, words, err);
    return hipGetLastError();
}

// Persistent grid (the segment count lives on the device): as many blocks as
// fit on the chip at once, from the occupancy API.
template <class K>
static unsigned resident_grid(K kernel, int block) {
    int dev = 0, cus = 256, per = 1;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, 0) != hipSuccess ||
        per < 1)
        per = 1;
    return (unsigned)(per * cus);
}
// Encoding rows for the fixed-shape kernel, passed by value as kernel
// arguments so the rows sit in SGPRs (v_dot4 takes them as scalar operands):
// lo[i][w] = low bytes of E[i][4w..4w+3], hi[i][w] the high bytes, and
// himask bit i = row i has an E >= 256 (for p = 257 only rows a = 2, 4, 8,
// where a^k = -1 for some k < 10).
struct IdaEncTab {
    uint32_t lo[IDA_MAX_N][4];
    uint32_t hi[IDA_MAX_N][4];
    uint32_t himask;
};

// Fixed-shape encode (N fragments, NW = ceil(m / 4) words per segment, DHash's
// (14, 10): N = 14, NW = 3): the same wave/chunk/LDS-staging scheme as
// k_ida_encode, with every row unrolled, E in SGPRs instead of LDS (no LDS
// round trip per row) and a one-fix-up reduction.  The generic kernel spent
// ~500 VALU + 5 serialised LDS reads per row-chunk; this one ~12 VALU per row.
template <int N, int NW, int D, bool P257>
__global__ __launch_bounds__(256) void k_ida_encode_fixed(const uint8_t *data,
                                                          const uint64_t *offs,
                                                          const uint64_t *seg, size_t blocks,
                                                          int m, uint32_t p, float inv_p,
                                                          uint16_t *frags, IdaEncTab tab) {
    constexpr int PRE = NW + 1 <= 3 ? 3 : NW + 1;  // chunk span <= 16 NW + 1 words
    __shared__ uint32_t stage[256 / 64][64 * PRE + 4];
    __shared__ uint32_t hi_s[N][NW];  // high-byte rows (rare: himask) stay in LDS
    for (int t = threadIdx.x; t < N * NW; t += blockDim.x) hi_s[t / NW][t % NW] = tab.hi[t / NW][t % NW];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    uint32_t *st = stage[threadIdx.x >> 6];
    const uint64_t total = seg[blocks];
    const uint64_t nbytes = offs[blocks];
    const uint64_t chunks = (total + 63) / 64;
    const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
    const uint64_t waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    const uint64_t cpw = (chunks + waves - 1) / waves;
    const uint64_t c0 = wave * cpw, c1 = c0 + cpw < chunks ? c0 + cpw : chunks;
    if (c0 >= c1) return;  // wave-uniform, after the only block barrier
    BlockCursor cur;
    cursor_init<true>(cur, seg, offs, seg_block(seg, blocks, c0 * 64));
    EncSlot<PRE> sl[D];
    auto issue = [&](EncSlot<PRE> &x, uint64_t c) {
        const uint64_t g = c * 64 + lane;
        x.live = g < total;
        cursor_advance<true>(cur, seg, offs, x.live ? g : total - 1);
        x.s = (x.live ? g : total - 1) - cur.sb;
        x.segb = cur.sb;
        x.S = cur.sb1 - cur.sb;
        const uint64_t my_lo = cur.ob + x.s * m;
        uint64_t my_hi = my_lo + m;
        if (my_hi > cur.ob1) my_hi = cur.ob1;
        x.span = __shfl(my_lo, 0) & ~3ull;
        const uint64_t span_hi = __shfl(my_hi, 63);
        x.words = (uint32_t)((span_hi - x.span + 3) >> 2);
        x.off = (uint32_t)(my_lo - x.span);
        x.have = (int)(my_hi - my_lo);
#pragma unroll
        for (int t = 0; t < PRE; ++t) {
            const uint32_t w = lane + 64 * t;
            const uint64_t at = x.span + 4ull * w;
            uint32_t v = 0;
            if (w < x.words) {
                if (at + 4 <= nbytes) {
                    v = *reinterpret_cast<const uint32_t *>(data + at);
                } else {
                    for (int k = 0; k < 4; ++k)
                        if (at + k < nbytes) v |= (uint32_t)data[at + k] << (8 * k);
                }
            }
            x.pre[t] = v;
        }
    };
#pragma unroll
    for (int k = 0; k < D; ++k)
        if (c0 + k < c1) issue(sl[k], c0 + k);
    for (uint64_t cb = c0; cb < c1; cb += D) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const uint64_t c = cb + k;
            if (c >= c1) break;  // wave-uniform
            const uint64_t segb = sl[k].segb, S = sl[k].S, sg = sl[k].s;
            const uint32_t off = sl[k].off, words = sl[k].words;
            const int have = sl[k].have;
            const bool live = sl[k].live;
#pragma unroll
            for (int t = 0; t < PRE; ++t)
                if (lane + 64 * t < (int)words) st[lane + 64 * t] = sl[k].pre[t];
            if (c + D < c1) issue(sl[k], c + D);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t bw = off >> 2, sh = off & 3;
            uint32_t W[NW];
            uint32_t prev = st[bw];
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                const uint32_t nxt = st[bw + j + 1];
                uint32_t x = __builtin_amdgcn_alignbyte(nxt, prev, sh);
                const int valid = have - 4 * j;
                x &= valid >= 4 ? 0xFFFFFFFFu : (valid <= 0 ? 0u : (1u << (8 * valid)) - 1u);
                W[j] = x;
                prev = nxt;
            }
            __builtin_amdgcn_wave_barrier();  // stage reused by the next chunk
            if (live) {
                uint16_t *o = frags + (uint64_t)N * segb + sg;
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    uint32_t acc = 0;
#pragma unroll
                    for (int j = 0; j < NW; ++j)
                        acc = __builtin_amdgcn_udot4(tab.lo[i][j], W[j], acc, false);
                    if (P257) {
                        // p = 257, 9 <= m <= 12: E >= 256 only where a^k = -1, i.e.
                        // E = 256 at (a, k) = (2, 8), (4, 4), (8, 8) (a = i + 1;
                        // 2 has order 16 mod 257): add 256 v_k directly
                        if (i == 1 || i == 7) acc += (W[2] & 0xFFu) << 8;
                        if (i == 3) acc += (W[1] & 0xFFu) << 8;
                    } else if ((tab.himask >> i) & 1) {  // scalar branch
                        uint32_t ah = 0;
#pragma unroll
                        for (int j = 0; j < NW; ++j)
                            ah = __builtin_amdgcn_udot4(hi_s[i][j], W[j], ah, false);
                        acc += ah << 8;  // <= m (p-1) 255 < 2^29
                    }
                    *o = (uint16_t)modp_fast(acc, p, inv_p);
                    o += S;
                }
            }
        }
    }
}

template <int PRE, int D>
static void ida_encode_launch(const uint8_t *data, const uint64_t *offs, const uint64_t *seg,
                              size_t blocks, int n, int m, int p, uint16_t *frags,
                              hipStream_t s) {
    static const unsigned grid = resident_grid(k_ida_encode<PRE, D>, 256);
    k_ida_encode<PRE, D><<<grid, 256, 0, s>>>(data, offs, seg, blocks, n, m, (uint32_t)p,
                                              1.0f / p, frags);
}

hipError_t ida_encode(const uint8_t *data, const uint64_t *offs, const uint64_t *seg,
                      size_t blocks, int n, int m, int p, uint16_t *frags, hipStream_t s) {
    if (blocks == 0) return hipSuccess;
    // pipeline depths (chunks in flight per wave): the measured best, 1 for the
    // fixed-shape kernel and 3 for the generic one (profiles/r02)
    if (n == 14 && m > 8 && m <= 12) {  // DHash (14, 10) and neighbours
        IdaEncTab tab = {};
        for (int i = 0; i < n; ++i) {
            uint32_t e = 1;
            for (int k = 0; k < m; ++k) {  // e = (i+1)^k mod p (ida.cpp:59-73)
                tab.lo[i][k >> 2] |= (e & 0xFFu) << (8 * (k & 3));
                tab.hi[i][k >> 2] |= (e >> 8) << (8 * (k & 3));
                if (e >> 8) tab.himask |= 1u << i;
                e = (uint32_t)(((uint64_t)e * (uint32_t)(i + 1)) % (uint32_t)p);
            }
        }
        // rows 1, 3, 7 hold the only E = 256 entries when p = 257 (see the kernel)
        const bool p257 = p == 257 && tab.himask == ((1u << 1) | (1u << 3) | (1u << 7));
        if (p257) {
            for (int i = 0; i < n; ++i)
                for (int w = 0; w < 4; ++w) tab.hi[i][w] = 0;
        }
#define CX_ENC_FIXED(DD, PP)                                                                 \
    do {                                                                                     \
        static const unsigned g = resident_grid(k_ida_encode_fixed<14, 3, DD, PP>, 256);     \
        k_ida_encode_fixed<14, 3, DD, PP><<<g, 256, 0, s>>>(data, offs, seg, blocks, m,      \
                                                            (uint32_t)p, 1.0f / p, frags,    \
                                                            tab);                            \
    } while (0)
        if (p257) CX_ENC_FIXED(1, true);
        else CX_ENC_FIXED(1, false);
#undef CX_ENC_FIXED
        return hipGetLastError();
    }
    if (16 * m + 1 > 64 * 3)
        ida_encode_launch<8, 2>(data, offs, seg, blocks, n, m, p, frags, s);
    else
        ida_encode_launch<3, 3>(data, offs, seg, blocks, n, m, p, frags, s);
    return hipGetLastError();
}

hipError_t ida_runs(const uint8_t *idx, size_t blocks, int m, uint32_t *flag, hipStream_t s) {
    if (blocks == 0) return hipSuccess;
    k_ida_runs<<<cx_grid(blocks, 256), 256, 0, s>>>(idx, blocks, m, flag);
    return hipGetLastError();
}

hipError_t ida_run_index(const uint32_t *flag_excl, const uint32_t *flag_raw, size_t blocks,
                         size_t runs, uint32_t *run_of, uint32_t *run_start, uint32_t *err,
                         hipStream_t s) {
    if (blocks == 0) return hipSuccess;
    k_ida_run_index<<<cx_grid(blocks, 256), 256, 0, s>>>(flag_excl, flag_raw, blocks, runs, run_of,
                                                        run_start, err);
    return hipGetLastError();
}

hipError_t ida_inverse(const uint8_t *idx, const uint32_t *run_start, size_t runs, size_t blocks,
                       int m, int p, int32_t *inv, uint8_t *okf, uint32_t *err, hipStream_t s) {
    if (runs == 0) return hipSuccess;
    k_ida_inverse<<<cx_grid(runs, 64), 64, 0, s>>>(idx, run_start, runs, blocks, m, p, inv, okf,
                                                   err);
    return hipGetLastError();
}

template <bool WIDE, int FM, int D, int MF = 0>
static void ida_decode_launch(const uint16_t *frags, const uint64_t *seg, size_t blocks, int m,
                              int p, const int32_t *inv, const uint32_t *run_of, size_t runs,
                              const uint8_t *okf, uint16_t *out, uint64_t *out_len,
                              uint32_t *err, hipStream_t s) {
    static const unsigned grid = resident_grid(k_ida_decode<WIDE, FM, D, MF>, 256);
    k_ida_decode<WIDE, FM, D, MF><<<grid, 256, 0, s>>>(
        frags, seg, blocks, m, (uint32_t)p, 1.0f / p, inv, run_of, runs, okf, out,
        reinterpret_cast<unsigned long long *>(out_len), err);
}

hipError_t ida_decode(const uint16_t *frags, const uint64_t *seg, size_t blocks, int m, int p,
                      const int32_t *inv, const uint32_t *run_of, size_t runs, const uint8_t *okf,
                      uint16_t *out, uint64_t *out_len, uint32_t *err, hipStream_t s) {
    if (blocks == 0) return hipSuccess;
    const bool wide = (uint64_t)m * (p - 1) * 65535ull >= (1ull << 32);
    // two chunks in flight per wave (the measured best, profiles/r02)
    if (wide)
        ida_decode_launch<true, IDA_MAX_N, 1>(frags, seg, blocks, m, p, inv, run_of, runs, okf, out,
                                              out_len, err, s);
    else if (m == 10)  // DHash (14, 10)
        ida_decode_launch<false, 12, 2, 10>(frags, seg, blocks, m, p, inv, run_of, runs, okf, out,
                                            out_len, err, s);
    else if (m > 12)
        ida_decode_launch<false, IDA_MAX_N, 1>(frags, seg, blocks, m, p, inv, run_of, runs, okf, out,
                                               out_len, err, s);
    else
        ida_decode_launch<false, 12, 2>(frags, seg, blocks, m, p, inv, run_of, runs, okf, out, out_len, err, s);
    return hipGetLastError();
}

// Validation of caller-supplied peer indices (finger uploads, preds):
// *d_bad = 1 if any entry is >= limit (CX_NONE allowed when allow_none).
__global__ void k_check_indices(const uint32_t *idx, size_t count, uint32_t limit,
                                int allow_none, uint32_t *bad) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint32_t v = idx[i];
        if (v >= limit && !(allow_none && v == CX_NONE)) atomicOr(bad, 1u);
    }
}

hipError_t check_indices(const uint32_t *idx, size_t count, uint32_t limit, bool allow_none,
                         uint32_t *d_bad, hipStream_t s) {
    if (count == 0) return hipSuccess;
    k_check_indices<<<cx_grid(count, 256), 256, 0, s>>>(idx, count, limit, allow_none ? 1 : 0,
                                                        d_bad);
    return hipGetLastError();
}

// ===========================================================================
// Request-rate probe: the walk's memory access pattern without the walk.
// Four lanes cooperate on one chain: each loads 16 B of a 64-B entry (one
// wave instruction, adjacent addresses), lane 0's data picks the next entry,
// so every step is one dependent random 64-B request.  Read only.
// ===========================================================================
__device__ __forceinline__ uint64_t probe_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_gather_probe(const uint4 *t, uint64_t slots, int hops,
                                                      unsigned long long *sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const int sub = threadIdx.x & 3;
    uint64_t x = probe_mix(tid / 4 + 777);
    for (int h = 0; h < hops; ++h) {
        const uint64_t slot = x % slots;
        // non-temporal, as the walk's table gathers
        typedef unsigned int v4n __attribute__((ext_vector_type(4)));
        const v4n a = __builtin_nontemporal_load(reinterpret_cast<const v4n *>(t) + slot * 4 + sub);
        uint64_t v = ((uint64_t)a.y << 32 | a.x) ^ a.z;
        v = __shfl(v, (threadIdx.x & 63) & ~3, 64);
        x = probe_mix(v + x);
    }
    if (x == 0x1234567ull) atomicAdd(sink, 1ull);  // keeps the chain live
}

hipError_t gather_probe(const void *table, size_t bytes, int lanes, int hops, double *rate,
                        hipStream_t s) {
    const uint64_t slots = bytes / 64;
    if (slots == 0 || lanes < 256 || hops < 1) return hipErrorInvalidValue;
    const unsigned blocks = (unsigned)(lanes / 256);
    const uint4 *t = static_cast<const uint4 *>(table);
    unsigned long long *sink = nullptr;
    hipEvent_t a = nullptr, b = nullptr;
    hipError_t e = hipMalloc(&sink, sizeof(*sink));
    if (e == hipSuccess) e = hipEventCreate(&a);
    if (e == hipSuccess) e = hipEventCreate(&b);
    if (e == hipSuccess) {
        k_gather_probe<<<blocks, 256, 0, s>>>(t, slots, 4, sink);  // warm-up
        e = hipEventRecord(a, s);
    }
    if (e == hipSuccess) {
        k_gather_probe<<<blocks, 256, 0, s>>>(t, slots, hops, sink);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(b, s);
    if (e == hipSuccess) e = hipEventSynchronize(b);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, a, b);
    if (e == hipSuccess) *rate = (double)(lanes / 4) * hops / (ms * 1e-3);
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    if (sink) (void)hipFree(sink);
    return e;
}

}  // namespace cxk
