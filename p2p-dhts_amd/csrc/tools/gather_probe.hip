// gather_probe.hip -- measures the random-gather ceiling of an MI355X, the
// bound that governs the finger-routed walk (one dependent gather per hop).
//
// Each lane runs `chains` independent pointer-chasing chains of `hops`
// dependent loads into a table of `bytes`; the next address is a hash of the
// loaded value, so every load is a random granule.  Reports dependent loads/s
// and the implied granule bandwidth.  Variants: load width (4/16/32 B), lanes
// in flight (grid size), chains per lane, table size.
//
// hipcc --offload-arch=gfx950 -O3 gather_probe.hip -o gather_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_fill(uint4 *t, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint64_t a = mix(i * 2 + 1), b = mix(i * 2 + 2);
        t[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
}

// WIDTH: 0 = 4 B, 1 = 16 B, 2 = 32 B (two dwordx4 from one 32-B slot),
// 3 = 20 B (dwordx4 + dword from one 32-B slot), 4 = 64 B (four dwordx4)
template <int WIDTH, int CHAINS>
__global__ __launch_bounds__(256) void k_chase(const uint4 *t, uint64_t slots, int hops,
                                               uint64_t *sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint64_t x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = mix(tid * CHAINS + c + 12345);
    for (int h = 0; h < hops; ++h) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) {
            const uint64_t slot = x[c] % slots;
            uint64_t v;
            if (WIDTH == 0) {
                v = reinterpret_cast<const uint32_t *>(t)[slot * 4];
            } else if (WIDTH == 1) {
                const uint4 a = t[slot];
                v = ((uint64_t)a.y << 32 | a.x) ^ a.z;
            } else if (WIDTH == 2) {
                const uint4 a = t[slot * 2], b = t[slot * 2 + 1];
                v = ((uint64_t)a.y << 32 | a.x) ^ a.z ^ b.x;
            } else if (WIDTH == 3) {
                const uint4 a = t[slot * 2];
                const uint32_t b = reinterpret_cast<const uint32_t *>(t + slot * 2 + 1)[0];
                v = ((uint64_t)a.y << 32 | a.x) ^ a.z ^ b;
            } else {
                const uint4 a = t[slot * 4], b = t[slot * 4 + 1], c = t[slot * 4 + 2],
                            d = t[slot * 4 + 3];
                v = ((uint64_t)a.y << 32 | a.x) ^ a.z ^ b.x ^ c.y ^ d.w;
            }
            x[c] = mix(v + x[c]);
        }
    }
    uint64_t r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) r ^= x[c];
    if (r == 0x1234567) sink[0] = r;
}

// G lanes cooperate on one chain: each loads 16 B of a G*16-byte slot (one
// wave instruction, adjacent addresses), lane 0's data picks the next slot.
template <int G>
__global__ __launch_bounds__(256) void k_chase_coop(const uint4 *t, uint64_t slots, int hops,
                                                    uint64_t *sink) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const int sub = threadIdx.x & (G - 1);
    uint64_t x = mix(tid / G + 777);
    for (int h = 0; h < hops; ++h) {
        const uint64_t slot = x % slots;
        const uint4 a = t[slot * G + sub];
        uint64_t v = ((uint64_t)a.y << 32 | a.x) ^ a.z;
        v = __shfl(v, (threadIdx.x & 63) & ~(G - 1), 64);  // lane 0 of the group
        x = mix(v + x);
    }
    if (x == 0x1234567) sink[0] = x;
}

template <int G>
double run_coop(const uint4 *t, size_t bytes, int lanes, int hops, uint64_t *sink) {
    const uint64_t slots = bytes / (16 * G);
    const int blocks = lanes / 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    k_chase_coop<G><<<blocks, 256>>>(t, slots, 4, sink);
    CK(hipEventRecord(a));
    k_chase_coop<G><<<blocks, 256>>>(t, slots, hops, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return (double)(lanes / G) * hops / (ms * 1e-3);  // chain steps (entries) per second
}

template <int WIDTH, int CHAINS>
double run(const uint4 *t, size_t bytes, int lanes, int hops, uint64_t *sink) {
    const uint64_t slots = WIDTH == 4 ? bytes / 64 : (WIDTH >= 2 ? bytes / 32 : bytes / 16);
    const int blocks = lanes / 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    k_chase<WIDTH, CHAINS><<<blocks, 256>>>(t, slots, 4, sink);
    CK(hipEventRecord(a));
    k_chase<WIDTH, CHAINS><<<blocks, 256>>>(t, slots, hops, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return (double)lanes * CHAINS * hops / (ms * 1e-3);
}

int main(int argc, char **argv) {
    const size_t max_bytes = argc > 1 ? strtoull(argv[1], 0, 0) : (16ull << 30);
    uint4 *t;
    uint64_t *sink;
    CK(hipMalloc(&t, max_bytes));
    CK(hipMalloc(&sink, 64));
    k_fill<<<4096, 256>>>(t, max_bytes / 16);
    CK(hipDeviceSynchronize());
    printf("{\"probe\":\"dependent random gathers\",\"rows\":[\n");
    bool first = true;
    auto row = [&](const char *w, int chains, size_t bytes, int lanes, double rate) {
        printf("%s{\"width\":\"%s\",\"chains\":%d,\"table_MiB\":%zu,\"lanes\":%d,"
               "\"Gloads_per_s\":%.2f,\"GBps_at_64B\":%.0f}",
               first ? "" : ",\n", w, chains, bytes >> 20, lanes, rate / 1e9, rate * 64 / 1e9);
        first = false;
        fflush(stdout);
    };
    const int full = 256 * 2048;  // 32 waves/CU x 256 CUs
    if (argc > 2 && !strcmp(argv[2], "calib")) {
        // one known workload for calibrating PMC FETCH_SIZE on this access
        // pattern (MI355X_MICROARCH.md: other widths than wide streams are
        // uncalibrated): a warm-up dispatch of 4 hops, then one of 64 hops, each
        // lane quad gathering one random 64-B entry per hop from the table
        const double rate = run_coop<4>(t, max_bytes, full, 64, sink);
        printf("{\"width\":\"64B/4lanes\",\"table_MiB\":%zu,\"entries_warmup\":%d,"
               "\"entries_timed\":%d,\"Gloads_per_s\":%.2f}]}\n",
               max_bytes >> 20, full / 4 * 4, full / 4 * 64, rate / 1e9);
        return 0;
    }
    if (argc > 2 && !strcmp(argv[2], "coop_sweep")) {
        // cooperative 64-B / 128-B entries against table size (TLB reach)
        for (size_t gb : {8ull, 16ull, 32ull, 64ull, 128ull, 192ull}) {
            const size_t bytes = gb << 30;
            if (bytes > max_bytes) continue;
            row("64B/4lanes", 1, bytes, full, run_coop<4>(t, bytes, full, 64, sink));
            row("128B/8lanes", 1, bytes, full, run_coop<8>(t, bytes, full, 64, sink));
        }
        printf("\n]}\n");
        return 0;
    }
    // table size sweep at full occupancy, 16-B loads
    for (size_t mb : {64ull, 256ull, 1024ull, 4096ull, 16384ull}) {
        size_t bytes = mb << 20;
        if (bytes > max_bytes) continue;
        row("16B", 1, bytes, full, run<1, 1>(t, bytes, full, 64, sink));
    }
    const size_t big = max_bytes;
    // width at full occupancy on the big table
    row("4B", 1, big, full, run<0, 1>(t, big, full, 64, sink));
    row("32B", 1, big, full, run<2, 1>(t, big, full, 64, sink));
    row("20B", 1, big, full, run<3, 1>(t, big, full, 64, sink));
    row("64B", 1, big, full, run<4, 1>(t, big, full, 64, sink));
    row("64B", 1, 1024ull << 20, full, run<4, 1>(t, 1024ull << 20, full, 64, sink));
    row("16B", 1, 2ull << 20, full, run<1, 1>(t, 2ull << 20, full, 64, sink));
    row("16B", 1, 32ull << 20, full, run<1, 1>(t, 32ull << 20, full, 64, sink));
    // cooperative wide entries: G lanes x 16 B = one entry
    row("32B/2lanes", 1, big, full, run_coop<2>(t, big, full, 64, sink));
    row("64B/4lanes", 1, big, full, run_coop<4>(t, big, full, 64, sink));
    row("128B/8lanes", 1, big, full, run_coop<8>(t, big, full, 64, sink));
    row("16B/1lane", 1, big, full, run_coop<1>(t, big, full, 64, sink));
    row("32B/2lanes", 1, 8192ull << 20, full, run_coop<2>(t, 8192ull << 20, full, 64, sink));
    row("64B/4lanes", 1, 8192ull << 20, full, run_coop<4>(t, 8192ull << 20, full, 64, sink));
    // lanes in flight
    for (int lanes : {full / 8, full / 4, full / 2}) row("16B", 1, big, lanes, run<1, 1>(t, big, lanes, 64, sink));
    // chains per lane (more MLP per lane)
    row("16B", 2, big, full, run<1, 2>(t, big, full, 32, sink));
    row("16B", 4, big, full, run<1, 4>(t, big, full, 16, sink));
    row("16B", 2, big, full / 2, run<1, 2>(t, big, full / 2, 32, sink));
    row("32B", 2, big, full, run<2, 2>(t, big, full, 32, sink));
    printf("\n]}\n");
    return 0;
}
