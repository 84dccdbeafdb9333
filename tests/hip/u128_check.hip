// Test-only HIP kernels (libcxtest.so; never linked into libchordx.so).
//
// 1. Variable 128-bit shifts: `v << a` and `v >> a` for every amount 0..127,
//    with the amount per lane (VGPR), as a kernel argument (SGPR), and under a
//    lane-divergent branch, against host results (tests/test_gpu_u128.py).
//    Round-5 VERDICT "What's weak" #2: the round-5 fix of a nondeterministic
//    route-table word blamed the lowering of such shifts; this settles whether
//    the compiler is involved.
// 2. The round-5 gap-code encode (cz_encode_hi before commit 0a5da05, exact-ID
//    branch through `full >> gs`), standalone, over caller-given operands: the
//    same expression outside the build kernel.
// The u128 type and the 16-byte loads are the engine's own (cx_common.hpp).
#include "../../p2p-dhts_amd/csrc/cx_common.hpp"

namespace {

constexpr uint32_t CZ_NONE_T = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t expect_t(uint32_t n, int l) {
    const int sh = 128 - l;
    return sh > 40 ? 0u : (uint32_t)(((uint64_t)n + (1ull << (sh - 1))) >> sh);
}

// The encode as it stood at 0a5da05~1 (cx_kernels.hip:1724-1753 there).
__device__ __forceinline__ uint32_t encode_r5(uint32_t n, int gs, uint32_t par, uint64_t phi, int l,
                                              uint32_t x, uint64_t xhi, const cell128 *ring) {
    int d = (int)x - (int)par - (int)expect_t(n, l);
    const int h = (int)(n / 2);
    const int lo = h + 1 - (int)n > -32768 ? h + 1 - (int)n : -32768;
    const int hi = h < 32766 ? h : 32766;
    if ((uint32_t)(d - lo) > (uint32_t)(hi - lo)) {
        if (d < 0) d += (int)n;
        if (d < 0) d += (int)n;
        if (d > h) d -= (int)n;
    }
    const int sh = gs - 64;
    const uint64_t D = xhi - phi - (1ull << (l - 64));
    uint64_t code;
    if (D & ((1ull << sh) - 1)) {
        code = D >> sh;
    } else {
        const u128 full = ld128(ring + x) - ld128(ring + par) - ((u128)1 << l);
        code = (uint64_t)(full >> gs);
        if ((full >> gs) >> 64) code = ~0ull;
    }
    if (d < -32768 || d > 32766 || code >= 0xFFFF) return CZ_NONE_T;
    return ((uint32_t)code << 16) | (uint32_t)(d + 32768);
}

// The encode as it stands since 0a5da05 (cx_kernels.hip cz_encode_hi).
__device__ __forceinline__ uint32_t encode_r6(uint32_t n, int gs, uint32_t par, uint64_t phi, int l,
                                              uint32_t x, uint64_t xhi, const cell128 *ring) {
    int d = (int)x - (int)par - (int)expect_t(n, l);
    const int h = (int)(n / 2);
    const int lo = h + 1 - (int)n > -32768 ? h + 1 - (int)n : -32768;
    const int hi = h < 32766 ? h : 32766;
    if ((uint32_t)(d - lo) > (uint32_t)(hi - lo)) {
        if (d < 0) d += (int)n;
        if (d < 0) d += (int)n;
        if (d > h) d -= (int)n;
    }
    const int sh = gs - 64;
    const uint64_t D = xhi - phi - (1ull << (l - 64));
    uint64_t code;
    if (D & ((1ull << sh) - 1)) {
        code = D >> sh;
    } else {
        code = (D - (uint64_t)(ring[x].lo < ring[par].lo)) >> sh;
    }
    if (d < -32768 || d > 32766 || code >= 0xFFFF) return CZ_NONE_T;
    return ((uint32_t)code << 16) | (uint32_t)(d + 32768);
}

// The one-lane-per-entry route-table build (cx_kernels.hip k_cz_build, MODE 0
// = row-major fingers, MODE 1 = level planes; the chained path and the LDS
// staged stores as there), with the round-5 (R5) or the current encode: the
// build the round-5 nondeterminism was seen in, outside the engine.  Whole
// table: levels [l0, l0 + R), grid (rows / 256, 2 R).
template <int MODE, bool R5>
__global__ __launch_bounds__(256) void k_build_t(const uint32_t *F, size_t sl, int L,
                                                 const cell128 *ring, const uint64_t *rh,
                                                 uint32_t n, int l0, int gs, uint4 *cz,
                                                 uint32_t *esc) {
    __shared__ uint4 stage[256 * 4];
    const uint32_t plane = blockIdx.y;
    const uint32_t per = gridDim.x >> 3;
    const uint32_t lb = per ? (blockIdx.x & 7) * per + (blockIdx.x >> 3) : blockIdx.x;
    const int b = (int)(plane & 1);
    const int i = l0 + (int)(plane >> 1);
    auto fat = [&](uint32_t x, int l) -> uint32_t {
        if (MODE != 0) return F[(size_t)(l - L) * sl + x];
        return F[(size_t)x * CX_FINGERS + l];
    };
    auto enc = [&](uint32_t par, uint64_t ph, int l, uint32_t x, uint64_t xh) -> uint32_t {
        return R5 ? encode_r5(n, gs, par, ph, l, x, xh, ring) : encode_r6(n, gs, par, ph, l, x, xh, ring);
    };
    uint32_t bad = 0, oob = 0;
    const uint32_t j = lb * blockDim.x + threadIdx.x;
    uint32_t out[16];
    for (int v = 0; v < 16; ++v) out[v] = 0;
    if (j < n) {
        const uint32_t p = j;
        uint32_t node[8];
        uint64_t nh[8];
        const uint64_t ph = rh[p];
        uint32_t a = p;
        uint64_t ah = ph;
        int al = i;
        if (b) {
            uint32_t A = fat(p, i);
            if (A >= n) {
                A = 0;
                oob = 1;
            }
            const uint64_t Ah = rh[A];
            out[15] = enc(p, ph, i, A, Ah);
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
        out[0] = enc(a, ah, al, node[0], nh[0]);
#pragma unroll
        for (int v = 1; v < 16; ++v) {
            const int hb = 31 - __builtin_clz((unsigned)v);
            const int pv = v & ~(1 << hb);
            const int lv = i - 2 - hb;
            if (v == 15 && b) continue;
            uint32_t x = fat(node[pv], lv);
            if (x >= n) {
                x = 0;
                oob = 1;
            }
            const uint64_t xh = rh[x];
            out[v] = enc(node[pv], nh[pv], lv, x, xh);
            if (v < 8) {
                node[v] = x;
                nh[v] = xh;
            }
        }
#pragma unroll
        for (int v = 0; v < 16; ++v) bad += out[v] == CZ_NONE_T;
    }
    {
        const int lane = threadIdx.x & 63;
        uint4 *ws = stage + (threadIdx.x >> 6) * 256;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            ws[lane * 4 + k] = make_uint4(out[4 * k], out[4 * k + 1], out[4 * k + 2], out[4 * k + 3]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t j0 = lb * blockDim.x + (threadIdx.x & ~63u);
        const size_t t0 = (size_t)plane * n + j0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = k * 64 + lane;
            if (j0 + (c >> 2) < n) {
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                const uint4 u = ws[c];
                const v4u w = {u.x, u.y, u.z, u.w};
                __builtin_nontemporal_store(w, reinterpret_cast<v4u *>(cz + t0 * 4) + c);
            }
        }
    }
    if (oob) atomicOr(esc + 1, 1u);
    if (bad) atomicAdd(esc, bad);
}

// out[6 i + k]: k = 0 v << a, 1 v >> a (a = amt[i], per lane); 2 v << ua,
// 3 v >> ua (ua uniform); 4 / 5 the same per-lane shifts taken in a
// lane-divergent branch (odd lanes left, even lanes right, then swapped).
__global__ void k_shifts(const cell128 *x, const int *amt, int ua, cell128 *out, uint32_t q) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= q) return;
    const u128 v = ld128(x + i);
    const int a = amt[i];
    st128(out + 6 * (size_t)i + 0, v << a);
    st128(out + 6 * (size_t)i + 1, v >> a);
    st128(out + 6 * (size_t)i + 2, v << ua);
    st128(out + 6 * (size_t)i + 3, v >> ua);
    u128 p, r;
    if (i & 1) {
        p = v << a;
        r = v >> a;
    } else {
        r = v >> a;
        p = v << a;
    }
    st128(out + 6 * (size_t)i + 4, p);
    st128(out + 6 * (size_t)i + 5, r);
}

// out[i] = encode_r5 of operand set i; lvl < 0: level per lane from l[i],
// else the uniform level `lvl` (the build's levels are block-uniform).
__global__ void k_encode_r5(uint32_t n, int gs, const uint32_t *par, const uint32_t *x,
                            const int *l, int lvl, const cell128 *ring, const uint64_t *rh,
                            uint32_t *out, uint32_t q) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= q) return;
    const int li = lvl < 0 ? l[i] : lvl;
    out[i] = encode_r5(n, gs, par[i], rh[par[i]], li, x[i], rh[x[i]], ring);
}

template <class T>
hipError_t up(T **d, const T *h, size_t count) {
    hipError_t e = hipMalloc((void **)d, count * sizeof(T) + 16);
    if (e == hipSuccess && count) e = hipMemcpy(*d, h, count * sizeof(T), hipMemcpyHostToDevice);
    return e;
}

}  // namespace

extern "C" {

// Host arrays in and out; returns a hipError_t value (0 = success).
int cxt_shifts(const cx_u128 *x, const int *amt, int ua, cx_u128 *out, uint32_t q) {
    cell128 *dx = nullptr, *dout = nullptr;
    int *da = nullptr;
    hipError_t e = up(&dx, reinterpret_cast<const cell128 *>(x), q);
    if (e == hipSuccess) e = up(&da, amt, q);
    if (e == hipSuccess) e = hipMalloc((void **)&dout, 6 * (size_t)q * sizeof(cell128));
    if (e == hipSuccess && q) {
        k_shifts<<<(q + 255) / 256, 256>>>(dx, da, ua, dout, q);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess)
        e = hipMemcpy(out, dout, 6 * (size_t)q * sizeof(cell128), hipMemcpyDeviceToHost);
    hipFree(dx);
    hipFree(da);
    hipFree(dout);
    return (int)e;
}

int cxt_encode_r5(uint32_t n, int gs, const cx_u128 *ring, const uint32_t *par, const uint32_t *x,
                  const int *l, int lvl, uint32_t *out, uint32_t q) {
    cell128 *dr = nullptr;
    uint64_t *drh = nullptr;
    uint32_t *dp = nullptr, *dx = nullptr, *dout = nullptr;
    int *dl = nullptr;
    uint64_t *rh = new uint64_t[n ? n : 1];
    for (uint32_t p = 0; p < n; ++p) rh[p] = ring[p].hi;
    hipError_t e = up(&dr, reinterpret_cast<const cell128 *>(ring), n);
    if (e == hipSuccess) e = up(&drh, rh, n);
    if (e == hipSuccess) e = up(&dp, par, q);
    if (e == hipSuccess) e = up(&dx, x, q);
    if (e == hipSuccess) e = up(&dl, l, q);
    if (e == hipSuccess) e = hipMalloc((void **)&dout, (size_t)q * 4 + 16);
    for (uint32_t p = 0; e == hipSuccess && p < q; ++p)  // operands must index the ring
        if (par[p] >= n || x[p] >= n) e = hipErrorInvalidValue;
    if (e == hipSuccess && q) {
        k_encode_r5<<<(q + 255) / 256, 256>>>(n, gs, dp, dx, dl, lvl, dr, drh, dout, q);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)q * 4, hipMemcpyDeviceToHost);
    delete[] rh;
    hipFree(dr);
    hipFree(drh);
    hipFree(dp);
    hipFree(dx);
    hipFree(dl);
    hipFree(dout);
    return (int)e;
}

// Route table of a ring from its row-major finger table F[n][128] (host
// arrays): mode 0 reads the rows, mode 1 level planes transposed here; r5 = 1
// the round-5 encode.  out: R * 2 * n * 16 words; esc[0] = CZ_NONE words.
int cxt_cz_build(int mode, int r5, const cx_u128 *ring, const uint32_t *F, uint32_t n, int l0,
                 int R, int gs, uint32_t *out, uint32_t *esc) {
    const int L = l0 - 5, nl = CX_FINGERS - L;
    if (L < 64 || gs < 65 || n == 0 || n >= (1u << 30)) return (int)hipErrorInvalidValue;
    uint64_t *rh = new uint64_t[n];
    for (uint32_t p = 0; p < n; ++p) rh[p] = ring[p].hi;
    uint32_t *fh = nullptr;
    size_t fwords = (size_t)n * CX_FINGERS;
    if (mode == 1) {
        fwords = (size_t)nl * n;
        fh = new uint32_t[fwords];
        for (int c = 0; c < nl; ++c)
            for (uint32_t p = 0; p < n; ++p) fh[(size_t)c * n + p] = F[(size_t)p * CX_FINGERS + L + c];
    }
    cell128 *dr = nullptr;
    uint64_t *drh = nullptr;
    uint32_t *dF = nullptr, *desc = nullptr;
    uint4 *dcz = nullptr;
    const size_t words = (size_t)R * 2 * n * 16;
    hipError_t e = up(&dr, reinterpret_cast<const cell128 *>(ring), n);
    if (e == hipSuccess) e = up(&drh, rh, n);
    if (e == hipSuccess) e = up(&dF, mode == 1 ? fh : F, fwords);
    if (e == hipSuccess) e = hipMalloc((void **)&dcz, words * 4);
    if (e == hipSuccess) e = hipMalloc((void **)&desc, 8);
    if (e == hipSuccess) e = hipMemset(desc, 0, 8);
    if (e == hipSuccess) e = hipMemset(dcz, 0xA5, words * 4);
    if (e == hipSuccess) {
        dim3 grid((n + 255) / 256, (unsigned)(2 * R));
        if (grid.x % 8) grid.x += 8 - grid.x % 8;  // the XCD-aware block order needs 8 | grid.x
        const size_t sl = mode == 1 ? n : 1;
        if (mode == 1 && r5)
            k_build_t<1, true><<<grid, 256>>>(dF, sl, L, dr, drh, n, l0, gs, dcz, desc);
        else if (mode == 1)
            k_build_t<1, false><<<grid, 256>>>(dF, sl, L, dr, drh, n, l0, gs, dcz, desc);
        else if (r5)
            k_build_t<0, true><<<grid, 256>>>(dF, sl, L, dr, drh, n, l0, gs, dcz, desc);
        else
            k_build_t<0, false><<<grid, 256>>>(dF, sl, L, dr, drh, n, l0, gs, dcz, desc);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, dcz, words * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(esc, desc, 8, hipMemcpyDeviceToHost);
    delete[] rh;
    delete[] fh;
    hipFree(dr);
    hipFree(drh);
    hipFree(dF);
    hipFree(dcz);
    hipFree(desc);
    return (int)e;
}

}  // extern "C"
