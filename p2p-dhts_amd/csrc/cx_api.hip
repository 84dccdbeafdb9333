// cx_api.hip -- C ABI of libchordx (include/chordx.h): ring handles, staging
// of host buffers, argument validation and error reporting.  All compute runs
// in the gfx950 kernels of cx_kernels.hip; there is no host compute path.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "cx_kernels.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define CX_HIP(expr)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(CX_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
    } while (0)

#define CX_CHECK(cond, code, msg)                                                         \
    do {                                                                                  \
        if (!(cond)) return fail((code), (msg));                                          \
    } while (0)

// RAII device allocation.
// ---------------------------------------------------------------------------
// Table pool.  A ring's large tables (finger table, route tables, arc planes:
// 72 GiB per 2^24-peer replica) and the builds' large temporaries (>= 64 KiB)
// are not returned to the driver
// when the ring is destroyed but kept, up to CX_POOL_CAP bytes per process,
// for the next ring that asks for the same size on the same device: after a
// membership change the new ring's tables reuse the old ring's HBM instead of
// paying ~0.6 s of fresh page mappings for 72 GiB.  A failed hipMalloc trims
// the pool and retries; cxi_pool_trim releases it.
// ---------------------------------------------------------------------------
namespace {
struct PoolEnt {
    int device;
    size_t bytes;
    void *p;
};
std::mutex g_pool_mu;
std::vector<PoolEnt> g_pool;
size_t g_pool_bytes = 0;
// Allocation-path counters (cumulative per process, under g_pool_mu; read by
// cxi_pool_stats): where each table / temporary came from -- fresh hipMalloc
// or a pooled block -- and how often an allocation had to trim the pool and
// retry (near the HBM limit).
struct PoolStats {
    uint64_t fresh_bytes = 0, fresh_allocs = 0;     // hipMalloc'd (new HBM pages)
    uint64_t reused_bytes = 0, reused_allocs = 0;   // handed back by the pool
    uint64_t trims = 0, trimmed_bytes = 0;          // idle blocks released to retry
    uint64_t retries = 0, failures = 0;             // first hipMalloc failed / both failed
} g_stats;
// Fault injection for tests (cxi_set_fault): bit 0 = the route-table build's
// finger-plane allocation fails (exercises the row-major fallback); bit 1 =
// the default build's overflow launches (cxk::cz2_set_cap).
std::atomic<int> g_fault{0};
// blocks from 64 KiB up: a churn's temporaries (2^17 joins: 0.5-3 MiB each)
// recur every epoch too, and each hipFree costs 0.1-0.3 ms
constexpr size_t POOL_MIN = (size_t)64 << 10;
// pool cap: CX_POOL_CAP_GIB (default 96; 0 disables pooling)
size_t pool_cap() {
    static const size_t cap = [] {
        const char *e = getenv("CX_POOL_CAP_GIB");
        const long v = e ? atol(e) : 96;
        return (size_t)(v < 0 ? 0 : v) << 30;
    }();
    return cap;
}

void pool_trim_locked(int device) {
    for (size_t k = 0; k < g_pool.size();) {
        if (device < 0 || g_pool[k].device == device) {
            ++g_stats.trims;
            g_stats.trimmed_bytes += g_pool[k].bytes;
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(g_pool[k].device);
            (void)hipFree(g_pool[k].p);
            (void)hipSetDevice(cur);
            g_pool_bytes -= g_pool[k].bytes;
            g_pool.erase(g_pool.begin() + k);
        } else {
            ++k;
        }
    }
}

// hipMalloc through the pool (current device).
hipError_t table_alloc(void **p, size_t bytes) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (bytes >= POOL_MIN) {
        std::lock_guard<std::mutex> g(g_pool_mu);
        for (size_t k = 0; k < g_pool.size(); ++k)
            if (g_pool[k].device == dev && g_pool[k].bytes == bytes) {
                *p = g_pool[k].p;
                g_pool_bytes -= bytes;
                g_pool.erase(g_pool.begin() + k);
                ++g_stats.reused_allocs;
                g_stats.reused_bytes += bytes;
                return hipSuccess;
            }
    }
    hipError_t e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        {
            std::lock_guard<std::mutex> g(g_pool_mu);
            ++g_stats.retries;
            pool_trim_locked(dev);
        }
        e = hipMalloc(p, bytes);
    }
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (e != hipSuccess) {
        *p = nullptr;
        ++g_stats.failures;
    } else {
        ++g_stats.fresh_allocs;
        g_stats.fresh_bytes += bytes;
    }
    return e;
}

// Returns a table to the pool (or frees it).  The caller has synchronised
// every stream that used it.
void table_free(int device, void *p, size_t bytes) {
    if (!p) return;
    if (bytes >= POOL_MIN) {
        std::lock_guard<std::mutex> g(g_pool_mu);
        while (g_pool_bytes + bytes > pool_cap() && !g_pool.empty()) {  // oldest first
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(g_pool.front().device);
            (void)hipFree(g_pool.front().p);
            (void)hipSetDevice(cur);
            g_pool_bytes -= g_pool.front().bytes;
            g_pool.erase(g_pool.begin());
        }
        if (g_pool_bytes + bytes <= pool_cap()) {
            g_pool.push_back(PoolEnt{device, bytes, p});
            g_pool_bytes += bytes;
            return;
        }
    }
    (void)hipFree(p);
}

// Plain hipMalloc that releases the idle pool blocks of the current device
// and retries once when HBM runs out (the pool must never be the reason an
// allocation outside it fails).
hipError_t dev_malloc(void **p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes);
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (e == hipSuccess) {
        ++g_stats.fresh_allocs;
        g_stats.fresh_bytes += bytes;
        return e;
    }
    (void)hipGetLastError();
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (g_pool.empty()) {
        ++g_stats.failures;
        return e;
    }
    ++g_stats.retries;
    pool_trim_locked(dev);
    e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
        *p = nullptr;
        ++g_stats.failures;
    } else {
        ++g_stats.fresh_allocs;
        g_stats.fresh_bytes += bytes;
    }
    return e;
}
bool cx_fault_planes() { return g_fault.load() & 1; }
template <class T>
hipError_t dev_malloc(T **p, size_t bytes) {
    return dev_malloc(reinterpret_cast<void **>(p), bytes);
}
}  // namespace

// Host-memory calls (CX_MEM_HOST) stage their inputs and outputs in device
// buffers.  A small process-wide cache keeps those buffers from call to call:
// a small batch's call otherwise spent more time in hipMalloc / hipFree (five
// of each for cx_route) than on the GPU.  Blocks are power-of-two sized, at
// most STAGE_MAX each (bigger staging is a plain hipMalloc, amortized by the
// batch), at most STAGE_HELD idle in the whole process (any number of calling
// threads: the cache is shared behind a mutex); a block returns to the cache
// only after the stream that used it has drained.  cx_pool_trim frees the idle
// blocks; the rest are left to process exit (the HIP runtime may already be
// gone when static destructors run).
constexpr size_t STAGE_MAX = (size_t)16 << 20;
constexpr size_t STAGE_HELD = (size_t)64 << 20;
struct StageBlk {
    void *p;
    size_t cap;
    int dev;
};
std::mutex g_stage_mu;
std::vector<StageBlk> *g_stage = new std::vector<StageBlk>();  // never destroyed
size_t g_stage_held = 0;

void stage_trim() {
    std::lock_guard<std::mutex> g(g_stage_mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (const StageBlk &b : *g_stage) {
        (void)hipSetDevice(b.dev);
        (void)hipFree(b.p);
    }
    (void)hipSetDevice(cur);
    g_stage->clear();
    g_stage_held = 0;
}

struct DBuf {
    void *p = nullptr;
    size_t pooled = 0;  // > 0: a table-pool block of this size (build temporaries >= 1 GiB)
    size_t staged = 0;  // > 0: a staging-cache block of this capacity (alloc_stage)
    int dev = 0;
    hipStream_t user = nullptr;  // stream whose work uses a pooled / staged block
    ~DBuf() { drop(); }
    void drop() {
        if (!p) return;
        if (staged) {
            (void)hipStreamSynchronize(user);
            bool kept = false;
            {
                std::lock_guard<std::mutex> g(g_stage_mu);
                if (g_stage_held + staged <= STAGE_HELD) {
                    g_stage->push_back(StageBlk{p, staged, dev});
                    g_stage_held += staged;
                    kept = true;
                }
            }
            if (!kept) (void)hipFree(p);
            p = nullptr;
            staged = 0;
            user = nullptr;
            return;
        }
        if (pooled) {
            // a pooled block goes back to the pool only after the work queued
            // on it has finished (hipFree would wait; the pool does not), so
            // another ring's build can never get it while kernels still use it
            // -- on the error paths too, where the caller returns early
            (void)hipStreamSynchronize(user);
            int dev = 0;
            (void)hipGetDevice(&dev);
            table_free(dev, p, pooled);
        } else {
            (void)hipFree(p);
        }
        p = nullptr;
        pooled = 0;
        user = nullptr;
    }
    hipError_t alloc(size_t bytes) {
        drop();
        return dev_malloc(&p, bytes ? bytes : 16);
    }
    // staging for a host-memory call on `stream` (the per-thread cache above)
    hipError_t alloc_stage(size_t bytes, hipStream_t stream) {
        drop();
        if (bytes > STAGE_MAX) return alloc(bytes);
        int d = 0;
        (void)hipGetDevice(&d);
        size_t cap = 4096;
        while (cap < bytes) cap <<= 1;
        {  // the smallest cached block of this device that fits
            std::lock_guard<std::mutex> g(g_stage_mu);
            std::vector<StageBlk> &c = *g_stage;
            size_t best = c.size();
            for (size_t k = 0; k < c.size(); ++k)
                if (c[k].dev == d && c[k].cap >= bytes && (best == c.size() || c[k].cap < c[best].cap))
                    best = k;
            if (best < c.size()) {
                p = c[best].p;
                cap = c[best].cap;
                c.erase(c.begin() + best);
                g_stage_held -= cap;
                staged = cap;
                dev = d;
                user = stream;
                return hipSuccess;
            }
        }
        hipError_t e = dev_malloc(&p, cap);
        if (e == hipSuccess) {
            staged = cap;
            dev = d;
            user = stream;
        }
        return e;
    }
    // through the table pool: build temporaries of the same size recur every
    // membership epoch; `stream` is the stream the block's users run on
    hipError_t alloc_pooled(size_t bytes, hipStream_t stream) {
        drop();
        hipError_t e = table_alloc(&p, bytes ? bytes : 16);
        if (e == hipSuccess) {
            pooled = bytes ? bytes : 16;
            user = stream;
        }
        return e;
    }
    template <class T>
    T *as() const {
        return static_cast<T *>(p);
    }
    void *release() {  // ownership to the caller (hipMalloc'd buffers only)
        void *r = p;
        p = nullptr;
        pooled = 0;
        return r;
    }
};

// IDA decode temporaries: a grow-only device arena per device and phase,
// reused across calls (calls on a device serialise on its mutex; growth
// hipFree-s the old block, which waits for the work still using it).  The
// arena is a performance measure only (per-call hipMalloc / hipFree cost
// 0.5 ms per call on 2^22 tiny blocks).  Pieces are packed tightly (8-B
// alignment, no padding), so an out-of-bounds index lands in a neighbouring
// piece instead of unmapped memory; the kernels bounds-check every index they
// derive (run_of, run_start, the block cursor) and a guard region after the
// inverse table is verified after each checked call ("IDA").
struct IdaArena {
    std::mutex mu;
    void *p[2] = {nullptr, nullptr};
    size_t cap[2] = {0, 0};
};
IdaArena &ida_arena(int device) {
    static IdaArena arenas[64];
    return arenas[device & 63];
}
// Carves tightly packed (8-B aligned) pieces of `sizes` bytes out of arena
// slot `slot`.
hipError_t arena_carve(IdaArena &a, int slot, std::initializer_list<size_t> sizes,
                       std::initializer_list<void **> outs) {
    size_t total = 0;
    for (size_t b : sizes) total += (b + 7) & ~(size_t)7;
    if (total > a.cap[slot]) {
        if (a.p[slot]) (void)hipFree(a.p[slot]);
        a.p[slot] = nullptr;
        a.cap[slot] = 0;
        hipError_t e = hipMalloc(&a.p[slot], total ? total : 256);
        if (e != hipSuccess) return e;
        a.cap[slot] = total ? total : 256;
    }
    char *c = static_cast<char *>(a.p[slot]);
    auto o = outs.begin();
    for (size_t b : sizes) {
        **o++ = c;
        c += (b + 7) & ~(size_t)7;
    }
    return hipSuccess;
}

}  // namespace

// The finger level planes a ring's route-table build read (kept with the
// ring: the next churn's finger repair remaps them).  Shared between a ring
// and the rings churned from it until their first finger build.
struct PlaneSet {
    int device = 0;
    uint32_t *p = nullptr;
    size_t bytes = 0, n = 0;
    int L = 0, nl = 0;
    ~PlaneSet() { table_free(device, p, bytes); }  // holders synchronise first
};

struct cx_ring {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    size_t n = 0;
    cell128 *d_ring = nullptr;     // sorted unique IDs [n]
    size_t ring_cap = 0;           // cells allocated for d_ring (>= n: before dedupe)
    cell128 *d_eyt = nullptr;      // Eytzinger copy [n+1]
    uint32_t *d_fingers = nullptr; // [n][128]
    bool fingers_converged = false;
    // converged, but the row-major table d_fingers is not written yet: the
    // default route (cz walk) needs only the level planes the finger build
    // hands to the route-table build, so cx_fingers_build without fingers_out
    // defers the 8 GiB of rows (2^24) to their first reader (ensure_fingers_rows)
    std::atomic<bool> rows_deferred{false};
    std::mutex rows_mu;  // first readers of deferred rows (ensure_fingers_rows)
    std::shared_ptr<PlaneSet> planes;         // level planes of the last finger build
    std::shared_ptr<PlaneSet> parent_planes;  // cx_churn: the parent's, until the first build
    // cxi_set_fingers_repair (A/B, default off): the repair is bit-identical
    // but slower than the streaming build (2^24, 1 %/1 % churn: 5.2 vs 1.7 ms
    // for the planes, profiles/r03/repair/); on, a ring keeps its planes
    // (2.3 GiB at 2^24) for the rings churned from it
    int fingers_repair = 0;
    int planes_repaired = 0;                  // last build: planes remapped from the parent
    uint64_t repair_searched = 0;             //   fingers searched exactly in that repair
    cell128 *d_ring_ext = nullptr; // [n+1] (pred, self) pairs
    int rt_l0 = 128, rt_R = 0;
    int depth_override = 0;        // cxi_set_route_depth (A/B): R levels instead of the default
    uint64_t *d_tree = nullptr;    // lookahead-tree table [n][rt_R][8] (variant 4)
    bool tree_valid = false;
    int pk_ib = 1;                 // index bits of a packed finger
    uint64_t *d_cz = nullptr;      // pattern-keyed window table [rt_R][2][n][8 x u64] (variant 5)
    int table_build = 0;           // route-table build input (cxi_set_table_build): 0 level + two-hop planes (roots),
                                   // 1 row-major fingers, 2 level planes only (A/B)
    bool cz_valid = false;
    uint64_t cz_escapes = 0;       // nodes the compressed format could not represent
    int route_variant = -1;        // 0: finger+ring gathers, 1: route table, 2: packed table,
                                   // 3: 2 + staging, 4: lookahead-tree table, 5: pattern-keyed
                                   // window table; -1: automatic (5 up to 2^24 peers, else 4)
    cell128 *d_min_keys = nullptr; // optional per-peer min_key_
    uint32_t *d_preds = nullptr;   // optional per-peer predecessor_
    uint8_t *d_alive = nullptr;    // optional per-peer liveness (cx_liveness_upload)
    uint32_t *d_succs = nullptr;   // optional successors_ lists [n][succ_ns]
    int succ_ns = 0;
    int fwd_rule = CX_FWD_CHORD;
    bool liveness = false;         // cx_liveness_upload called: literal walk
    uint32_t *d_scratch = nullptr; // small device scratch (counts/flags), 1 KiB
    unsigned long long *d_stats = nullptr;  // route gather counters (cxi_route_counters)
    bool counting = false;
    // arc mode (cx_arc_build): [replicated top planes | planes below arc_Lh for
    // the arc_M peers from arc_plo (the arc and its halo)] of the cz table
    uint64_t *d_arc_tree = nullptr;
    ArcBound *d_arc_bounds = nullptr;  // last peer ID of each non-empty arc
    int arc_world = 0, arc_rank = -1, arc_Lh = 128, arc_nb = 0;
    uint32_t arc_plo = 0, arc_M = 0;
    size_t arc_bytes = 0;          // d_arc_tree allocation

    uint4 *d_dir = nullptr;        // bucket directory [2^dir_k] (16 B entries)
    uint32_t *d_ring_key = nullptr; // ID slices [n] of the streaming finger build
    int dir_k = 1;
    int search_variant = 1;        // 0: Eytzinger (LDS top levels), 1: bucket directory
                                   // (successor / predecessor of large batches on rings that
                                   // fit LDS: the LDS slice table), 2: wave-cooperative 16-ary
                                   // tree, 3: wave-cooperative Eytzinger, 4: LDS slice table
                                   // whenever it fits, 5: directory only (1 without LDS)
    void *d_sltab = nullptr;       // LDS slice table (variants 1 / 4, lazy; cxk::slice_tab_*)
    int sl_b = 0, sl_steps = 0;
    bool sl_dev16 = false;         // offsets as int16 deviations (one more bucket bit)
    std::mutex sl_mu;              // first searches build it (const queries on many threads)
    std::atomic<bool> sl_ready{false};  // d_sltab / sl_b / sl_steps published
    cell128 *d_stree = nullptr;    // levels 1.. of the 16-ary tree (variant 2, lazy)
    uint32_t *d_eyt_rank = nullptr; // Eytzinger node -> sorted index (variant 3, lazy)
    int churn_variant = 1;         // 0: full re-sort, 1: merge of sorted joins (default)
    uint64_t serial = 0;           // process-unique handle number
    // cx_churn result: the parent's serial and the old_to_new it returned; the
    // churn directory (misplaced scan) is built from them on first use
    uint64_t churn_parent = 0;
    uint32_t *d_o2n_canon = nullptr;
    size_t o2n_canon_n = 0;
    uint4 *d_cdir = nullptr;       // [2^cdir_kb][2] (ChurnDir)
    int cdir_kb = 0;
    size_t cdir_bytes = 0;
    int misplaced_variant = 1;     // 0: two searches + old_to_new window, 1: churn directory

    EytView eyt() const {
        EytView v;
        v.E = d_eyt;
        v.n = (uint32_t)n;
        v.h = 63 - __builtin_clzll((unsigned long long)n);
        return v;
    }
    SearchView sv() const {
        SearchView v;
        v.ev = eyt();
        v.dir = (search_variant != 0) ? d_dir : nullptr;
        v.k = dir_k;
        v.ring = d_ring;
        return v;
    }
    bool literal() const { return !fingers_converged || d_min_keys || d_preds || liveness; }
    // hand-edited state (peer state or liveness uploads): only cx_route's
    // literal walk honours it
    bool edited() const { return d_min_keys || d_preds || liveness; }
    LitState lit() const {
        LitState l;
        l.alive = d_alive;
        l.succs = d_succs;
        l.ns = succ_ns;
        l.rule = fwd_rule;
        return l;
    }
    int variant() const {
        if (route_variant >= 0) return route_variant;
        return (pk_ib <= 24 && !cz_failed) ? 5 : 4;
    }
    bool cz_failed = false;        // automatic mode: no HBM for the variant-5 table
};

namespace {

int use_device(const cx_ring *r) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur == r->device) return CX_OK;
    CX_HIP(hipSetDevice(r->device));
    return CX_OK;
}

// Makes `count` elements of a caller buffer available on the device.
template <class T>
int stage_in(const T *src, size_t count, int memkind, DBuf &tmp, const T **dev, hipStream_t s) {
    if (count == 0) {
        *dev = src;
        return CX_OK;
    }
    CX_CHECK(src != nullptr, CX_E_INVALID, "null input buffer");
    if (memkind == CX_MEM_DEVICE) {
        *dev = src;
        return CX_OK;
    }
    CX_CHECK(memkind == CX_MEM_HOST, CX_E_INVALID, "bad memkind");
    CX_HIP(tmp.alloc_stage(count * sizeof(T), s));
    CX_HIP(hipMemcpyAsync(tmp.p, src, count * sizeof(T), hipMemcpyHostToDevice, s));
    *dev = tmp.as<T>();
    return CX_OK;
}

template <class T>
int stage_out(T *dst, size_t count, int memkind, DBuf &tmp, T **dev, hipStream_t s) {
    if (count == 0) {
        *dev = dst;
        return CX_OK;
    }
    CX_CHECK(dst != nullptr, CX_E_INVALID, "null output buffer");
    if (memkind == CX_MEM_DEVICE) {
        *dev = dst;
        return CX_OK;
    }
    CX_CHECK(memkind == CX_MEM_HOST, CX_E_INVALID, "bad memkind");
    CX_HIP(tmp.alloc_stage(count * sizeof(T), s));
    *dev = tmp.as<T>();
    return CX_OK;
}

template <class T>
int finish_out(T *dst, const T *dev, size_t count, int memkind, hipStream_t s) {
    if (memkind == CX_MEM_HOST && count) {
        CX_HIP(hipMemcpyAsync(dst, dev, count * sizeof(T), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
    }
    return CX_OK;
}

int sync_if_host(int memkind, hipStream_t s) {
    if (memkind == CX_MEM_HOST) CX_HIP(hipStreamSynchronize(s));
    return CX_OK;
}

// A ring handle's own stream and 1-KiB scratch word block are kept for the
// next handle on the device when a ring is destroyed (a membership epoch
// creates one ring and destroys one: hipStreamCreate + hipMalloc cost ~1 ms,
// hipStreamDestroy another).  Returned idle (the ring synchronised it).
struct RingRes {
    int device;
    hipStream_t stream;
    void *scratch;
};
std::mutex g_res_mu;
std::vector<RingRes> g_res;
constexpr size_t RES_KEEP = 16;  // per process

int alloc_ring(int device, cx_ring **out) {
    cx_ring *r = new cx_ring();
    r->device = device;
    {
        std::lock_guard<std::mutex> g(g_res_mu);
        for (size_t k = g_res.size(); k-- > 0;)
            if (g_res[k].device == device) {
                r->own_stream = g_res[k].stream;
                r->d_scratch = static_cast<uint32_t *>(g_res[k].scratch);
                g_res.erase(g_res.begin() + k);
                break;
            }
    }
    if (!r->own_stream) {
        hipError_t e = hipStreamCreateWithFlags(&r->own_stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete r;
            return fail(CX_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
        }
        e = dev_malloc(&r->d_scratch, 1024);
        if (e != hipSuccess) {
            (void)hipStreamDestroy(r->own_stream);
            delete r;
            return fail(CX_E_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
        }
    }
    r->stream = r->own_stream;
    static std::atomic<uint64_t> next_serial{1};
    r->serial = next_serial++;
    *out = r;
    return CX_OK;
}

void free_ring(cx_ring *r) {
    if (!r) return;
    (void)hipSetDevice(r->device);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    if (r->own_stream) (void)hipStreamSynchronize(r->own_stream);
    r->planes.reset();
    r->parent_planes.reset();
    // the ring's per-peer arrays recur at the same sizes every membership
    // epoch: through the pool like the tables (below 64 KiB: freed)
    table_free(r->device, r->d_ring, r->ring_cap * sizeof(cell128));
    (void)hipFree(r->d_eyt);
    table_free(r->device, r->d_dir, r->d_dir ? ((size_t)1 << r->dir_k) * sizeof(uint4) : 0);
    table_free(r->device, r->d_ring_key, r->n * sizeof(uint32_t));
    const size_t ent = r->n * (size_t)r->rt_R;
    table_free(r->device, r->d_fingers, r->n * CX_FINGERS * sizeof(uint32_t));
    table_free(r->device, r->d_tree, ent * 64);
    table_free(r->device, r->d_cz, ent * 128);
    (void)hipFree(r->d_stree);
    (void)hipFree(r->d_eyt_rank);
    (void)hipFree(r->d_sltab);
    table_free(r->device, r->d_ring_ext, (r->n + 1) * sizeof(cell128));
    (void)hipFree(r->d_min_keys);
    (void)hipFree(r->d_preds);
    (void)hipFree(r->d_alive);
    (void)hipFree(r->d_succs);
    table_free(r->device, r->d_arc_tree, r->arc_bytes);
    (void)hipFree(r->d_arc_bounds);
    (void)hipFree(r->d_stats);
    table_free(r->device, r->d_o2n_canon, r->o2n_canon_n * sizeof(uint32_t));
    table_free(r->device, r->d_cdir, r->cdir_bytes);
    if (r->own_stream) {
        // the own stream was synchronised above (r->stream may be a user stream:
        // then the own stream has seen no work since its last synchronisation)
        (void)hipStreamSynchronize(r->own_stream);
        std::lock_guard<std::mutex> g(g_res_mu);
        if (r->d_scratch && g_res.size() < RES_KEEP) {
            g_res.push_back(RingRes{r->device, r->own_stream, r->d_scratch});
        } else {
            (void)hipStreamDestroy(r->own_stream);
            (void)hipFree(r->d_scratch);
        }
    } else {
        (void)hipFree(r->d_scratch);
    }
    delete r;
}

// Eytzinger copy of r->d_ring: only the Eytzinger searches (variants 0 and 3)
// read it, so it is built when one of them is selected (256 MiB and 0.2 ms at
// 2^24 that a default ring -- and every churn epoch -- no longer pays).
int ensure_eyt(cx_ring *r, hipStream_t s) {
    if (r->d_eyt || !r->d_ring) return CX_OK;
    DBuf E;
    CX_HIP(E.alloc((r->n + 1) * sizeof(cell128)));
    CX_HIP(cxk::eyt_build(r->d_ring, r->n, E.as<cell128>(), s));
    CX_HIP(hipStreamSynchronize(s));
    r->d_eyt = E.as<cell128>();
    E.release();
    return CX_OK;
}

// Bucket directory (and, for the Eytzinger searches, the Eytzinger copy) of
// r->d_ring (r->n set).
int build_search(cx_ring *r, hipStream_t s) {
    const size_t m = r->n;
    if (r->search_variant == 0 || r->search_variant == 3) {
        int rc = ensure_eyt(r, s);
        if (rc) return rc;
    }
    // 2^k buckets, k = ceil(log2 n) + 1: a query's bucket entry resolves it
    // unless the bucket holds >= 2 peers and the key lies past the first; the
    // extra bit halves the load factor (fewer second gathers, 2x the bytes;
    // the measured best of 0..3 extra bits, round 1)
    constexpr int extra = 1;
    int k = 1;
    while (((size_t)1 << k) < m) ++k;
    k += extra;
    if (k > 29) k = 29;
    r->dir_k = k;
    DBuf lo, dir;
    CX_HIP(lo.alloc_pooled((((size_t)1 << k) + 1) * sizeof(uint32_t), s));
    CX_HIP(dir.alloc_pooled(((size_t)1 << k) * sizeof(uint4), s));
    CX_HIP(cxk::dir_build(r->d_ring, m, k, lo.as<uint32_t>(), dir.as<uint4>(), s));
    CX_HIP(hipStreamSynchronize(s));
    r->d_dir = dir.as<uint4>();
    dir.release();
    return CX_OK;
}

// Route-table levels [l0, 128): l0 = 128 - R, R = ceil(log2 n) + 8 rounded up
// to 4 (32 at 2^24; ib = index bits of a packed finger).  Below the table the
// walk takes exact hops: 0.004 per lookup at R = log2 n + 8, ~0.05 at + 4.
// Measured at 2^24 in the bench's ABBA leg: R = 32 routes
// 2.1 / 3.2 % faster per launch than R = 28 with either ring built first, for
// 8 GiB more table and ~2.8 ms more churn -> route-ready.
void route_geometry(cx_ring *r) {
    int lg = 0;
    while (((size_t)1 << lg) < r->n) ++lg;
    int R = ((lg + 8 + 3) / 4) * 4;
    // CX_ROUTE_R: table depth override (A/B of table size against exact hops)
    static const int r_env = [] {
        const char *e = getenv("CX_ROUTE_R");
        const int v = e ? atoi(e) : 0;
        if (e && (v < 16 || v > 59)) {
            fprintf(stderr, "cx: CX_ROUTE_R=%s ignored (must be in [16, 59])\n", e);
            return 0;
        }
        return v;
    }();
    if (r_env > 0) R = r_env;
    if (r->depth_override > 0) R = r->depth_override;
    if (R < 16) R = 16;
    if (R > 59) R = 59;
    r->rt_R = R;
    r->rt_l0 = 128 - R;
    r->pk_ib = lg < 1 ? 1 : lg;
}

// Finger access for a route-table build over levels [lo - 5, 128): level
// planes in `ft` when HBM allows (cxi_set_table_build(ring, 1) forces the
// row-major table, for A/B), else the row-major table itself.
hipError_t finger_planes(const cx_ring *r, int lo, DBuf &ft, cxk::FingerView &fv, DBuf &hi,
                         DBuf &c2, hipStream_t s, const uint32_t *ft_pre = nullptr) {
    fv = cxk::FingerView::rows(r->d_fingers);
    // gap codes of the root-centric build: 32-bit ID slices when every ring gap
    // is below 2^(gs + 17) (uniform rings by far), else the 64-bit high words
    // and the one-lane-per-entry build
    bool slices = false;
    const bool roots_build = r->table_build == 0;
    if (roots_build) {
        hipError_t e1 = hi.alloc_pooled(r->n * sizeof(uint32_t), s);
        uint32_t *d_wide = r->d_scratch + 100;
        if (e1 == hipSuccess)
            e1 = cxk::ring_codes(r->d_ring, r->n, r->pk_ib, hi.as<uint32_t>(), d_wide, s);
        uint32_t wide = 1;
        if (e1 == hipSuccess) e1 = hipMemcpyAsync(&wide, d_wide, sizeof(wide), hipMemcpyDeviceToHost, s);
        if (e1 == hipSuccess) e1 = hipStreamSynchronize(s);
        if (e1 != hipSuccess) return e1;
        slices = wide == 0;
    }
    if (!slices) {
        hipError_t e0 = hi.alloc_pooled(r->n * sizeof(uint64_t), s);
        if (e0 == hipSuccess) e0 = cxk::ring_hi(r->d_ring, r->n, hi.as<uint64_t>(), s);
        if (e0 != hipSuccess) return e0;
    }
    const int L = lo - 5 < 0 ? 0 : lo - 5, nl = (int)CX_FINGERS - L;
    hipError_t e = hipSuccess;
    bool have_planes = true;
    if (ft_pre && r->table_build != 1) {  // written by the finger build itself
        fv = cxk::FingerView::planes(ft_pre, r->n, L, nl);
    } else if (r->table_build == 1 || cx_fault_planes() ||
               ft.alloc_pooled((size_t)nl * r->n * sizeof(uint32_t), s) != hipSuccess) {
        // the row-major table (forced, or no HBM for the planes): no two-hop
        // planes and no root-centric build; the slice codes are replaced by
        // high words below
        (void)hipGetLastError();
        have_planes = false;
    } else {
        e = cxk::fingers_levels(r->d_fingers, r->n, L, nl, ft.as<uint32_t>(), s);
        if (e != hipSuccess) return e;
        fv = cxk::FingerView::planes(ft.as<uint32_t>(), r->n, L, nl);
    }
    if (have_planes && (roots_build || r->table_build == 3) &&
        c2.alloc_pooled((size_t)(nl - 1) * r->n * sizeof(uint32_t), s) == hipSuccess) {
        e = cxk::fingers_pairs(fv.F, r->n, nl, c2.as<uint32_t>(), s);
        if (e == hipSuccess) {
            fv.C2 = c2.as<uint32_t>();
            // 0: root-centric blocks sized by distinct roots; 3: one lane per entry
            fv.roots = roots_build ? 2 : 0;
        }
    }
    (void)hipGetLastError();
    if (slices) {
        if (fv.roots) {
            fv.rs = hi.as<uint32_t>();
        } else {  // no root-centric build after all: the others read high words
            hipError_t e0 = hi.alloc_pooled(r->n * sizeof(uint64_t), s);
            if (e0 == hipSuccess) e0 = cxk::ring_hi(r->d_ring, r->n, hi.as<uint64_t>(), s);
            if (e0 != hipSuccess) return e0;
        }
    }
    return e;
}

// Builds (once per finger build) the table the selected route variant reads.
// Without HBM for it the route falls back to variant 0 (finger + ring gathers).
int ensure_fingers_rows(cx_ring *ring, hipStream_t s);

int ensure_route_table(cx_ring *r, hipStream_t s, const uint32_t *ft_pre = nullptr) {
    if (!r->fingers_converged || !r->d_ring_ext) return CX_OK;

    const size_t ent = r->n * (size_t)r->rt_R;
    if (r->variant() == 5 && !r->cz_valid) {
        if (!r->d_cz && table_alloc((void **)&r->d_cz, ent * 128) != hipSuccess) {
            r->d_cz = nullptr;
            if (r->route_variant < 0) r->cz_failed = true;  // automatic: use variant 4
        }
        if (r->d_cz) {
            CX_HIP(hipMemsetAsync(r->d_scratch, 0, 2 * sizeof(uint32_t), s));
            DBuf ft, hi, c2;
            cxk::FingerView fv;
            if (!ft_pre || r->table_build == 1) {  // the planes come from the rows
                if (int rc = ensure_fingers_rows(r, s)) return rc;
            }
            CX_HIP(finger_planes(r, r->rt_l0, ft, fv, hi, c2, s, ft_pre));
            DBuf ws;  // the default build's overflow list
            if (fv.roots >= 2)
                CX_HIP(ws.alloc_pooled(cxk::cz_build_ws_words(r->n, r->rt_l0, r->rt_R, (uint32_t)r->n) *
                                           sizeof(uint32_t), s));
            CX_HIP(cxk::cz_build(fv, r->d_ring, hi.as<uint64_t>(), r->n, r->rt_l0, r->rt_R, r->pk_ib, r->d_cz,
                                 r->d_scratch, s, ws.as<uint32_t>()));
            uint32_t esc[2] = {0, 0};
            CX_HIP(hipMemcpyAsync(esc, r->d_scratch, sizeof(esc), hipMemcpyDeviceToHost, s));
            CX_HIP(hipStreamSynchronize(s));
            CX_CHECK(esc[1] == 0, CX_E_STATE, "route-table build met a finger out of range");
            r->cz_escapes = esc[0];
            r->cz_valid = true;
        }
    }
    if (r->variant() == 4 && !r->tree_valid) {
        if (!r->d_tree && table_alloc((void **)&r->d_tree, ent * 64) != hipSuccess)
            r->d_tree = nullptr;
        if (r->d_tree) {
            if (int rc = ensure_fingers_rows(r, s)) return rc;
            CX_HIP(cxk::tree_build(r->d_fingers, r->d_ring, r->n, r->rt_l0, r->rt_R, r->pk_ib, r->d_tree, s));
            r->tree_valid = true;
        }
    }
    return CX_OK;
}

// Merge-based churn: sorts the joins only; survivors keep their order (see
// cx_kernels.hip "Merge-based churn").  Fills r->n, r->d_ring and o2n.
int churn_merge(const cx_ring *old_ring, const cell128 *J0, size_t nj, const cell128 *L,
                size_t nl, cx_ring *r, DBuf &o2n, hipStream_t s) {
    const size_t n_old = old_ring->n;
    SearchView v = old_ring->sv();
    v.dir = old_ring->d_dir;
    // every temporary recurs at the same size each membership epoch: through
    // the pool (plain hipMalloc / hipFree cost ~0.7 ms per churn at 2^24)
    DBuf G, A, ws, jk0, jk1, jt0, jt1, pos, keep, ringbuf;
    // joins: bucket sort, and the radix sort when a bucket overflowed
    // (clustered joins)
    uint32_t *d_ovf = static_cast<uint32_t *>(r->d_scratch) + 64;
    uint32_t gone = 0, kept = 0, ovf = 0;
    const cell128 *J = J0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        const bool radix = attempt == 1;
        size_t sw = cxk::scan_workspace_words(n_old + 2 > nj + 1 ? n_old + 2 : nj + 1);
        const size_t rw = nj ? (radix ? cxk::sort_workspace_words(nj)
                                      : cxk::bucket_sort_workspace_words(nj)) : 0;
        if (rw > sw) sw = rw;
        CX_HIP(ws.alloc_pooled(sw * sizeof(uint32_t), s));
        CX_HIP(G.alloc_pooled((n_old + 1) * sizeof(uint32_t), s));
        CX_HIP(A.alloc_pooled((n_old + 2) * sizeof(uint32_t), s));
        CX_HIP(hipMemsetAsync(G.p, 0, (n_old + 1) * sizeof(uint32_t), s));
        CX_HIP(hipMemsetAsync(A.p, 0, (n_old + 2) * sizeof(uint32_t), s));
        CX_HIP(hipMemsetAsync(d_ovf, 0, sizeof(uint32_t), s));
        CX_HIP(cxk::merge_mark(v, old_ring->d_ring, L, nl, G.as<uint32_t>(), s));
        if (nj) {
            CX_HIP(jk0.alloc_pooled(nj * sizeof(cell128), s));
            if (radix) {
                CX_HIP(jk1.alloc_pooled(nj * sizeof(cell128), s));
                CX_HIP(jt0.alloc_pooled(nj * sizeof(uint32_t), s));
                CX_HIP(jt1.alloc_pooled(nj * sizeof(uint32_t), s));
                CX_HIP(cxk::copy_tagged(J0, nj, 0, jk0.as<cell128>(), jt0.as<uint32_t>(), s));
                CX_HIP(cxk::radix_sort(jk0.as<cell128>(), jt0.as<uint32_t>(), jk1.as<cell128>(),
                                       jt1.as<uint32_t>(), nj, ws.as<uint32_t>(), s));
            } else {
                CX_HIP(cxk::bucket_sort(J0, nj, jk0.as<cell128>(), ws.as<uint32_t>(), d_ovf, s));
            }
            J = jk0.as<cell128>();
            CX_HIP(pos.alloc_pooled(nj * sizeof(uint32_t), s));
            CX_HIP(keep.alloc_pooled((nj + 1) * sizeof(uint32_t), s));
            CX_HIP(hipMemsetAsync(keep.p, 0, (nj + 1) * sizeof(uint32_t), s));
            CX_HIP(cxk::merge_join_pos(v, old_ring->d_ring, n_old, G.as<uint32_t>(), J, nj,
                                       pos.as<uint32_t>(), keep.as<uint32_t>(), A.as<uint32_t>(),
                                       s));
            CX_HIP(cxk::exclusive_scan(keep.as<uint32_t>(), nj + 1, ws.as<uint32_t>(), s));
        }
        CX_HIP(cxk::exclusive_scan(G.as<uint32_t>(), n_old + 1, ws.as<uint32_t>(), s));
        CX_HIP(cxk::exclusive_scan(A.as<uint32_t>(), n_old + 2, ws.as<uint32_t>(), s));
        CX_HIP(hipMemcpyAsync(&gone, G.as<uint32_t>() + n_old, sizeof(gone),
                              hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(&kept, A.as<uint32_t>() + n_old + 1, sizeof(kept),
                              hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(&ovf, d_ovf, sizeof(ovf), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
        if (!ovf) break;  // else: clustered joins, sort again with the radix sort
    }
    const size_t m = n_old - gone + kept;
    CX_CHECK(m >= 1, CX_E_INVALID, "churn would leave an empty ring");
    CX_HIP(ringbuf.alloc_pooled(m * sizeof(cell128), s));
    CX_HIP(o2n.alloc_pooled(n_old * sizeof(uint32_t), s));
    CX_HIP(cxk::merge_scatter(old_ring->d_ring, n_old, G.as<uint32_t>(), A.as<uint32_t>(), J, nj,
                              pos.as<uint32_t>(), keep.as<uint32_t>(), ringbuf.as<cell128>(),
                              o2n.as<uint32_t>(), s));
    r->n = m;
    r->ring_cap = m;
    r->d_ring = ringbuf.as<cell128>();
    ringbuf.release();
    return CX_OK;
}

}  // namespace

// ===========================================================================
// ABI
// ===========================================================================
extern "C" {

int cx_version(void) { return CHORDX_VERSION; }

const char *cx_last_error(void) { return g_err.c_str(); }

int cx_device_count(int *count) {
    CX_CHECK(count != nullptr, CX_E_INVALID, "null count");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *count = c;
    return CX_OK;
}

int cx_ring_create(const cx_u128 *ids, size_t n, int memkind, int device, cx_ring **out) {
    CX_CHECK(out != nullptr, CX_E_INVALID, "null out");
    *out = nullptr;
    CX_CHECK(n >= 1, CX_E_INVALID, "a ring needs at least one peer");
    CX_CHECK(n < (size_t)CX_TAG_JOIN, CX_E_INVALID, "ring larger than 2^31 peers");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(CX_E_HIP, "no HIP device: chordx has no host compute path");
    CX_CHECK(device >= 0 && device < ndev, CX_E_INVALID, "bad device ordinal");
    CX_HIP(hipSetDevice(device));
    cx_ring *r = nullptr;
    int rc = alloc_ring(device, &r);
    if (rc) return rc;
    hipStream_t s = r->stream;
    DBuf k0, k1, t0, t1, stage;
    auto bail = [&](int code) {
        free_ring(r);
        return code;
    };
    if (k0.alloc(n * sizeof(cell128)) != hipSuccess || k1.alloc(n * sizeof(cell128)) ||
        t0.alloc(n * sizeof(uint32_t)) || t1.alloc(n * sizeof(uint32_t)))
        return bail(fail(CX_E_NOMEM, "hipMalloc failed for ring build"));
    const hipMemcpyKind kind =
        memkind == CX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (memkind != CX_MEM_DEVICE && memkind != CX_MEM_HOST)
        return bail(fail(CX_E_INVALID, "bad memkind"));
    if (!ids) return bail(fail(CX_E_INVALID, "null ids"));
    if (hipMemcpyAsync(k0.p, ids, n * sizeof(cell128), kind, s) != hipSuccess)
        return bail(fail(CX_E_HIP, "copying ids failed"));
    if (cxk::iota(t0.as<uint32_t>(), n, 0, s) != hipSuccess)
        return bail(fail(CX_E_HIP, "iota launch failed"));
    rc = [&]() -> int {
        DBuf ws, pos, ring;
        const size_t sw = cxk::sort_workspace_words(n), cw = cxk::scan_workspace_words(n);
        CX_HIP(ws.alloc((sw > cw ? sw : cw) * sizeof(uint32_t)));
        CX_HIP(pos.alloc(n * sizeof(uint32_t)));
        CX_HIP(cxk::radix_sort(k0.as<cell128>(), t0.as<uint32_t>(), k1.as<cell128>(),
                               t1.as<uint32_t>(), n, ws.as<uint32_t>(), s));
        CX_HIP(ring.alloc_pooled(n * sizeof(cell128), s));
        CX_HIP(cxk::unique_sorted(k0.as<cell128>(), t0.as<uint32_t>(), n, pos.as<uint32_t>(),
                                  ws.as<uint32_t>(), ring.as<cell128>(), nullptr,
                                  r->d_scratch, s));
        uint32_t m = 0;
        CX_HIP(hipMemcpyAsync(&m, r->d_scratch, sizeof(m), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
        CX_CHECK(m >= 1 && m <= n, CX_E_HIP, "ring build produced an invalid size");
        r->n = m;
        r->ring_cap = n;
        r->d_ring = ring.as<cell128>();
        ring.release();
        return build_search(r, s);
    }();
    if (rc) return bail(rc);
    *out = r;
    return CX_OK;
}

int cx_ring_destroy(cx_ring *ring) {
    free_ring(ring);
    return CX_OK;
}

int cx_ring_size(const cx_ring *ring, size_t *n) {
    CX_CHECK(ring && n, CX_E_INVALID, "null argument");
    *n = ring->n;
    return CX_OK;
}

int cx_ring_ids(const cx_ring *ring, cx_u128 *out, int memkind) {
    CX_CHECK(ring && out, CX_E_INVALID, "null argument");
    int rc = use_device(ring);
    if (rc) return rc;
    const hipMemcpyKind kind =
        memkind == CX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    CX_HIP(hipMemcpyAsync(out, ring->d_ring, ring->n * sizeof(cell128), kind, ring->stream));
    return sync_if_host(memkind, ring->stream);
}

int cx_ring_ids_device(const cx_ring *ring, const cx_u128 **ids) {
    CX_CHECK(ring && ids, CX_E_INVALID, "null argument");
    *ids = reinterpret_cast<const cx_u128 *>(ring->d_ring);
    return CX_OK;
}

int cx_ring_set_stream(cx_ring *ring, void *hip_stream) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    ring->stream = static_cast<hipStream_t>(hip_stream);
    return CX_OK;
}

int cx_ring_use_own_stream(cx_ring *ring) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    ring->stream = ring->own_stream;
    return CX_OK;
}

int cx_ring_sync(const cx_ring *ring) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    int rc = use_device(ring);
    if (rc) return rc;
    CX_HIP(hipStreamSynchronize(ring->stream));
    return CX_OK;
}

namespace {
// The 16-ary tree's levels (search variant 2), built on first use.
// BFS -> sorted index table of the Eytzinger copy (search variant 3), lazy.
int eyt_rank_view(cx_ring *r, hipStream_t s) {
    if (r->d_eyt_rank) return CX_OK;
    CX_HIP(dev_malloc(&r->d_eyt_rank, (r->n + 1) * sizeof(uint32_t)));
    CX_HIP(cxk::eyt_rank_build(r->n, r->d_eyt_rank, s));
    return CX_OK;
}

// The LDS slice table (cxk::slice_tab_*) of a ring that fits LDS, built on
// first use: b = ceil(log2 n) - 4 bucket bits (about 16 peers a bucket, 1 to
// 12; down to ceil(log2 n) - 7 when the table would not fit, ~79 000 peers at
// most), the search rounds from its largest bucket.  *ok = false when the ring
// does not fit (or has no HBM for it): the caller searches the directory.
// Built once under the ring's sl_mu (const queries may come from several
// threads) and published by sl_ready.
int slice_view(cx_ring *r, hipStream_t s, bool *ok) {
    *ok = r->sl_ready.load(std::memory_order_acquire);
    if (*ok) return CX_OK;
    std::lock_guard<std::mutex> g(r->sl_mu);
    *ok = r->sl_ready.load(std::memory_order_relaxed);
    if (*ok) return CX_OK;
    int lg = 0;
    while (((size_t)1 << lg) < r->n) ++lg;
    // first choice: b = ceil(log2 n) - 3 (~8 peers a bucket) with int16 offset
    // deviations, when they fit 16 bits (uniform rings) and the table fits LDS
    {
        const int b16 = lg - 3 < 1 ? 1 : (lg - 3 > 14 ? 14 : lg - 3);
        const size_t bytes16 = cxk::slice_tab_bytes(r->n, b16, true);
        const size_t tmp_bytes = cxk::slice_tab_bytes(r->n, b16);
        void *tmp = nullptr, *tab = nullptr;
        if (bytes16 <= cxk::SLICE_TAB_MAX && dev_malloc(&tmp, tmp_bytes) == hipSuccess) {
            const size_t nb = ((size_t)1 << b16) + 1;
            std::vector<uint32_t> off(nb);
            hipError_t e = cxk::slice_tab_build(r->d_ring, r->n, b16, tmp, s);
            if (e == hipSuccess)
                e = hipMemcpyAsync(off.data(), tmp, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) {
                (void)hipFree(tmp);
                return fail(CX_E_HIP, hipGetErrorString(e));
            }
            std::vector<int16_t> dev(nb);
            bool fits = true;
            uint32_t mx = 0;
            for (size_t t = 0; t < nb && fits; ++t) {
                const long long d = (long long)off[t] - (long long)((uint64_t)t * r->n >> b16);
                fits = d >= -32768 && d <= 32767;
                dev[t] = (int16_t)d;
                if (t + 1 < nb) mx = std::max(mx, off[t + 1] - off[t]);
            }
            const size_t off16 = (nb * 2 + 15) / 16 * 16, off32 = (nb * 4 + 15) / 16 * 16;
            if (fits && dev_malloc(&tab, bytes16) == hipSuccess) {
                e = hipMemsetAsync(tab, 0, bytes16, s);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(tab, dev.data(), nb * 2, hipMemcpyHostToDevice, s);
                if (e == hipSuccess)
                    e = hipMemcpyAsync(static_cast<char *>(tab) + off16,
                                       static_cast<char *>(tmp) + off32, r->n * 2,
                                       hipMemcpyDeviceToDevice, s);
                if (e == hipSuccess) e = hipStreamSynchronize(s);
                (void)hipFree(tmp);
                if (e != hipSuccess) {
                    (void)hipFree(tab);
                    return fail(CX_E_HIP, hipGetErrorString(e));
                }
                r->sl_steps = mx ? 32 - __builtin_clz(mx) : 0;
                r->sl_b = b16;
                r->sl_dev16 = true;
                r->d_sltab = tab;
                r->sl_ready.store(true, std::memory_order_release);
                *ok = true;
                return CX_OK;
            }
            (void)hipFree(tmp);
        }
    }
    int b = lg - 4 < 1 ? 1 : (lg - 4 > 12 ? 12 : lg - 4);
    const int bmin = lg - 7 < 1 ? 1 : lg - 7;  // buckets of <= ~128 peers (<= 8 rounds)
    while (b > bmin && cxk::slice_tab_bytes(r->n, b) > cxk::SLICE_TAB_MAX) --b;
    const size_t bytes = cxk::slice_tab_bytes(r->n, b);
    if (bytes > cxk::SLICE_TAB_MAX) return CX_OK;
    void *tab = nullptr;
    if (dev_malloc(&tab, bytes) != hipSuccess) return CX_OK;
    const size_t nb = ((size_t)1 << b) + 1;
    std::vector<uint32_t> off(nb);
    hipError_t e = cxk::slice_tab_build(r->d_ring, r->n, b, tab, s);
    if (e == hipSuccess)
        e = hipMemcpyAsync(off.data(), tab, nb * sizeof(uint32_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        (void)hipFree(tab);
        return fail(CX_E_HIP, hipGetErrorString(e));
    }
    uint32_t mx = 0;
    for (size_t t = 0; t + 1 < nb; ++t) mx = std::max(mx, off[t + 1] - off[t]);
    r->sl_steps = mx ? 32 - __builtin_clz(mx) : 0;
    r->sl_b = b;
    r->d_sltab = tab;
    r->sl_ready.store(true, std::memory_order_release);
    *ok = true;
    return CX_OK;
}

// Variant 1 takes the LDS table for batches of >= 2^16 keys and >= 4 n (each
// resident block stages the whole table once); variant 4 whenever it fits.
bool slice_wanted(const cx_ring *r, size_t q) {
    if (r->search_variant == 4) return true;
    return r->search_variant == 1 && q >= ((size_t)1 << 16) && q >= 4 * r->n &&
           r->n * 2 < cxk::SLICE_TAB_MAX;
}

int stree_view(cx_ring *r, cxk::STreeView &st, hipStream_t s) {
    st = cxk::stree_plan(r->d_ring, r->n, r->d_stree);
    if (!r->d_stree && st.words) {
        if (dev_malloc(&r->d_stree, st.words * sizeof(cell128)) != hipSuccess) {
            r->d_stree = nullptr;
            return fail(CX_E_NOMEM, "hipMalloc of the 16-ary search levels failed");
        }
        st = cxk::stree_plan(r->d_ring, r->n, r->d_stree);
        CX_HIP(cxk::stree_build(st, s));
    }
    return CX_OK;
}
}  // namespace

int cx_successor(const cx_ring *ring, const cx_u128 *keys, size_t q, uint32_t *owner,
                 int memkind) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    DBuf tk, to;
    const cx_u128 *dk;
    uint32_t *dout;
    if ((rc = stage_in(keys, q, memkind, tk, &dk, s))) return rc;
    if ((rc = stage_out(owner, q, memkind, to, &dout, s))) return rc;
    if (ring->search_variant == 2) {
        cxk::STreeView st;
        if ((rc = stree_view(const_cast<cx_ring *>(ring), st, s))) return rc;
        CX_HIP(cxk::successor_stree(st, reinterpret_cast<const cell128 *>(dk), q, dout, false, s));
    } else if (ring->search_variant == 3) {
        if ((rc = eyt_rank_view(const_cast<cx_ring *>(ring), s))) return rc;
        CX_HIP(cxk::successor_eyt16(ring->eyt(), ring->d_eyt_rank,
                                    reinterpret_cast<const cell128 *>(dk), q, dout, false, s));
    } else {
        bool lds = false;
        if (slice_wanted(ring, q) && (rc = slice_view(const_cast<cx_ring *>(ring), s, &lds)))
            return rc;
        if (lds)
            CX_HIP(cxk::successor_lds(ring->d_sltab, ring->sl_b, ring->sl_dev16, ring->sl_steps,
                                      ring->d_ring, ring->n,
                                      reinterpret_cast<const cell128 *>(dk), q, dout, false, s));
        else
            CX_HIP(cxk::successor(ring->sv(), reinterpret_cast<const cell128 *>(dk), q, dout, s));
    }
    return finish_out(owner, dout, q, memkind, s);
}

namespace {
// The converged n x 128 finger table into ring->d_fingers (allocated).
int build_fingers_table(cx_ring *ring, hipStream_t s, uint32_t *ft = nullptr, int ft_l = 0,
                        bool *ft_done = nullptr, bool rows = true) {
    // streaming per-block window build (needs the directory and the ID
    // slices); one search per entry without HBM for them
    SearchView fv = ring->sv();
    fv.dir = ring->d_dir;
    if (!ring->d_ring_key) {
        if (table_alloc((void **)&ring->d_ring_key, ring->n * sizeof(uint32_t)) == hipSuccess)
            CX_HIP(cxk::ring_slice_build(ring->d_ring, ring->n, cxk::finger_key_shift(ring->n),
                                         ring->d_ring_key, s));
        else
            ring->d_ring_key = nullptr;  // no HBM for it: one search per entry
    }
    DBuf fws;
    const bool streaming = ring->d_ring_key &&
                           fws.alloc_pooled(cxk::fingers_workspace_bytes(ring->n), s) == hipSuccess;
    // planes only (rows deferred) needs the streaming build with every plane a tile level
    if (!streaming || !ft || ft_l < cxk::FINGERS_TILE_L0 || ring->n < ((size_t)1 << 18)) rows = true;
    if (rows && !ring->d_fingers &&
        table_alloc((void **)&ring->d_fingers, ring->n * CX_FINGERS * sizeof(uint32_t)) != hipSuccess) {
        ring->d_fingers = nullptr;
        return fail(CX_E_NOMEM, "hipMalloc of the finger table failed");
    }
    CX_HIP(cxk::fingers_build(fv, ring->d_ring, streaming ? ring->d_ring_key : nullptr,
                              streaming ? fws.p : nullptr, rows ? ring->d_fingers : nullptr, s, ft,
                              ft_l, ft_done));
    ring->fingers_converged = true;
    ring->rows_deferred = !rows;
    ring->tree_valid = ring->cz_valid = false;
    return CX_OK;
}
}  // namespace

namespace {
// Writes the deferred row-major finger table (same kernels, rows instead of
// planes) before anything that reads d_fingers.
int ensure_fingers_rows(cx_ring *ring, hipStream_t s) {
    if (!ring->rows_deferred) return CX_OK;
    // readers on other threads / streams see rows_deferred cleared only once
    // the rows are complete (and pass no table to the cz walk until then)
    std::lock_guard<std::mutex> g(ring->rows_mu);
    if (!ring->rows_deferred) return CX_OK;
    if (!ring->d_fingers &&
        table_alloc((void **)&ring->d_fingers, ring->n * CX_FINGERS * sizeof(uint32_t)) != hipSuccess) {
        ring->d_fingers = nullptr;
        return fail(CX_E_NOMEM, "hipMalloc of the finger table failed");
    }
    SearchView fv = ring->sv();
    fv.dir = ring->d_dir;
    if (!ring->d_ring_key && ring->n >= ((size_t)1 << 18)) {  // a repaired ring has none yet
        if (table_alloc((void **)&ring->d_ring_key, ring->n * sizeof(uint32_t)) == hipSuccess)
            CX_HIP(cxk::ring_slice_build(ring->d_ring, ring->n, cxk::finger_key_shift(ring->n),
                                         ring->d_ring_key, s));
        else
            ring->d_ring_key = nullptr;
    }
    DBuf fws;
    const bool streaming = ring->d_ring_key &&
                           fws.alloc_pooled(cxk::fingers_workspace_bytes(ring->n), s) == hipSuccess;
    CX_HIP(cxk::fingers_build(fv, ring->d_ring, streaming ? ring->d_ring_key : nullptr,
                              streaming ? fws.p : nullptr, ring->d_fingers, s, nullptr, 0,
                              nullptr));
    CX_HIP(hipStreamSynchronize(s));
    ring->rows_deferred = false;
    return CX_OK;
}
}  // namespace

int cx_predecessor(const cx_ring *ring, const cx_u128 *keys, size_t q, uint32_t *pred,
                   int memkind) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    DBuf tk, to;
    const cx_u128 *dk;
    uint32_t *dout;
    if ((rc = stage_in(keys, q, memkind, tk, &dk, s))) return rc;
    if ((rc = stage_out(pred, q, memkind, to, &dout, s))) return rc;
    if (ring->search_variant == 2) {
        cxk::STreeView st;
        if ((rc = stree_view(const_cast<cx_ring *>(ring), st, s))) return rc;
        CX_HIP(cxk::successor_stree(st, reinterpret_cast<const cell128 *>(dk), q, dout, true, s));
    } else if (ring->search_variant == 3) {
        if ((rc = eyt_rank_view(const_cast<cx_ring *>(ring), s))) return rc;
        CX_HIP(cxk::successor_eyt16(ring->eyt(), ring->d_eyt_rank,
                                    reinterpret_cast<const cell128 *>(dk), q, dout, true, s));
    } else {
        bool lds = false;
        if (slice_wanted(ring, q) && (rc = slice_view(const_cast<cx_ring *>(ring), s, &lds)))
            return rc;
        if (lds)
            CX_HIP(cxk::successor_lds(ring->d_sltab, ring->sl_b, ring->sl_dev16, ring->sl_steps,
                                      ring->d_ring, ring->n,
                                      reinterpret_cast<const cell128 *>(dk), q, dout, true, s));
        else
            CX_HIP(cxk::predecessor(ring->sv(), reinterpret_cast<const cell128 *>(dk), q, dout, s));
    }
    return finish_out(pred, dout, q, memkind, s);
}

int cx_fingers_build(cx_ring *ring, uint32_t *fingers_out, int memkind) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    const size_t cnt = ring->n * CX_FINGERS;
    route_geometry(ring);
    // rows deferred (planes only) when nobody asked for them and the default
    // route reads planes from the streaming build
    const int ft_l = ring->rt_l0 - 5;
    const bool defer = !fingers_out && ring->variant() == 5 &&
                       (ring->table_build == 0 || ring->table_build == 3) && ft_l >= 64 &&
                       ring->n >= ((size_t)1 << 18) && ft_l >= cxk::FINGERS_TILE_L0;
    // the default route table reads the fingers as level planes: the streaming
    // finger build writes them alongside the rows (no transpose pass), and the
    // ring keeps them for the finger repair of the next churn
    std::shared_ptr<PlaneSet> ps;
    bool ft_done = false;
    if (ring->variant() == 5 && (ring->table_build == 0 || ring->table_build == 3) && ft_l >= 64) {
        const int nl = (int)CX_FINGERS - ft_l;
        const size_t bytes = (size_t)nl * ring->n * sizeof(uint32_t);
        void *pp = nullptr;
        if (table_alloc(&pp, bytes) == hipSuccess) {
            ps = std::make_shared<PlaneSet>();
            ps->device = ring->device;
            ps->p = static_cast<uint32_t *>(pp);
            ps->bytes = bytes;
            ps->n = ring->n;
            ps->L = ft_l;
            ps->nl = nl;
        } else {
            (void)hipGetLastError();
        }
    }
    // f2 finger repair: a churned ring remaps its parent's planes (cx_churn
    // handed them over with the old_to_new map) instead of searching every
    // finger; the rows stay deferred either way
    std::shared_ptr<PlaneSet> par = std::move(ring->parent_planes);
    ring->planes_repaired = 0;
    ring->repair_searched = 0;
    uint32_t searched = 0;
    const bool repair = ps && par && defer && ring->fingers_repair && par->device == ring->device &&
                        par->L == ps->L && par->nl == ps->nl && ring->d_o2n_canon &&
                        ring->o2n_canon_n == par->n && ring->d_dir;
    if (repair) {
        DBuf n2o;
        CX_HIP(n2o.alloc_pooled(ring->n * sizeof(uint32_t), s));
        uint32_t *d_cnt = ring->d_scratch + 96;
        CX_HIP(hipMemsetAsync(d_cnt, 0, sizeof(uint32_t), s));
        SearchView sv = ring->sv();
        sv.dir = ring->d_dir;
        CX_HIP(cxk::planes_repair(sv, ring->d_ring, ring->n, par->p, par->n, ring->d_o2n_canon,
                                  n2o.as<uint32_t>(), ps->L, ps->nl, ps->p, d_cnt, s));
        CX_HIP(hipMemcpyAsync(&searched, d_cnt, sizeof(searched), hipMemcpyDeviceToHost, s));
        ring->fingers_converged = true;
        ring->rows_deferred = true;
        ring->planes_repaired = 1;
        ft_done = true;
    } else if ((rc = build_fingers_table(ring, s, ps ? ps->p : nullptr, ft_l, &ft_done,
                                         !defer || !ps))) {
        return rc;
    }
    ring->tree_valid = ring->cz_valid = false;  // tables follow the fingers
    if (!ring->d_ring_ext &&
        table_alloc((void **)&ring->d_ring_ext, (ring->n + 1) * sizeof(cell128)) != hipSuccess)
        ring->d_ring_ext = nullptr;
    if (ring->d_ring_ext) CX_HIP(cxk::ring_ext_build(ring->d_ring, ring->n, ring->d_ring_ext, s));
    // the default route kernel's table is built now (outside any timed query)
    if (int rc2 = ensure_route_table(ring, s, ft_done ? ps->p : nullptr)) {
        (void)hipStreamSynchronize(s);  // before the planes go back to the pool
        return rc2;
    }
    if (fingers_out) {
        const hipMemcpyKind kind =
            memkind == CX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        CX_HIP(hipMemcpyAsync(fingers_out, ring->d_fingers, cnt * sizeof(uint32_t), kind, s));
    }
    if (repair || !ft_done) {
        // the repair read the parent's planes (and its count); unused planes
        // are dropped: both wait for the stream
        CX_HIP(hipStreamSynchronize(s));
        ring->repair_searched = searched;
    }
    ring->planes = (ft_done && ring->fingers_repair) ? ps : nullptr;
    return sync_if_host(memkind, s);
}

int cx_fingers_upload(cx_ring *ring, const uint32_t *fingers, int memkind) {
    CX_CHECK(ring && fingers, CX_E_INVALID, "null argument");
    int rc = use_device(ring);
    if (rc) return rc;
    CX_CHECK(memkind == CX_MEM_HOST || memkind == CX_MEM_DEVICE, CX_E_INVALID, "bad memkind");
    hipStream_t s = ring->stream;
    const size_t cnt = ring->n * CX_FINGERS;
    // validated in a staging buffer first: a rejected upload leaves the
    // ring's current table (and route state) untouched
    DBuf staged;
    if (staged.alloc(cnt * sizeof(uint32_t)) != hipSuccess)
        return fail(CX_E_NOMEM, "hipMalloc of the finger table failed");
    const hipMemcpyKind kind =
        memkind == CX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    CX_HIP(hipMemcpyAsync(staged.p, fingers, cnt * sizeof(uint32_t), kind, s));
    CX_HIP(hipMemsetAsync(ring->d_scratch, 0, sizeof(uint32_t), s));
    CX_HIP(cxk::check_indices(staged.as<uint32_t>(), cnt, (uint32_t)ring->n, true,
                              ring->d_scratch, s));
    uint32_t bad = 0;
    CX_HIP(hipMemcpyAsync(&bad, ring->d_scratch, sizeof(bad), hipMemcpyDeviceToHost, s));
    CX_HIP(hipStreamSynchronize(s));
    CX_CHECK(!bad, CX_E_INVALID, "finger entry is neither a ring index nor CX_NONE");
    table_free(ring->device, ring->d_fingers, cnt * sizeof(uint32_t));
    ring->d_fingers = staged.as<uint32_t>();
    staged.release();
    ring->fingers_converged = false;
    ring->rows_deferred = false;
    ring->tree_valid = ring->cz_valid = false;
    return CX_OK;
}

int cx_fingers_device(const cx_ring *ring, const uint32_t **fingers) {
    CX_CHECK(ring && fingers, CX_E_INVALID, "null argument");
    if (ring->rows_deferred) {  // materialised now, complete when this returns
        int rc = use_device(ring);
        if (rc) return rc;
        if ((rc = ensure_fingers_rows(const_cast<cx_ring *>(ring), ring->stream))) return rc;
    }
    *fingers = ring->d_fingers;
    return CX_OK;
}

int cx_peer_state_upload(cx_ring *ring, const cx_u128 *min_keys, const uint32_t *preds,
                         int memkind) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    int rc = use_device(ring);
    if (rc) return rc;
    CX_CHECK(memkind == CX_MEM_HOST || memkind == CX_MEM_DEVICE, CX_E_INVALID, "bad memkind");
    hipStream_t s = ring->stream;
    const hipMemcpyKind kind =
        memkind == CX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    // staged and validated first: a rejected upload leaves the current state
    DBuf mk, pr;
    if (min_keys) {
        CX_HIP(mk.alloc(ring->n * sizeof(cell128)));
        CX_HIP(hipMemcpyAsync(mk.p, min_keys, ring->n * sizeof(cell128), kind, s));
    }
    if (preds) {
        CX_HIP(pr.alloc(ring->n * sizeof(uint32_t)));
        CX_HIP(hipMemcpyAsync(pr.p, preds, ring->n * sizeof(uint32_t), kind, s));
        CX_HIP(hipMemsetAsync(ring->d_scratch, 0, sizeof(uint32_t), s));
        CX_HIP(cxk::check_indices(pr.as<uint32_t>(), ring->n, (uint32_t)ring->n, true,
                                  ring->d_scratch, s));
        uint32_t bad = 0;
        CX_HIP(hipMemcpyAsync(&bad, ring->d_scratch, sizeof(bad), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
        CX_CHECK(!bad, CX_E_INVALID, "predecessor is neither a ring index nor CX_NONE");
    }
    CX_HIP(hipStreamSynchronize(s));
    (void)hipFree(ring->d_min_keys);
    (void)hipFree(ring->d_preds);
    ring->d_min_keys = mk.as<cell128>();
    ring->d_preds = pr.as<uint32_t>();
    mk.release();
    pr.release();
    return CX_OK;
}

int cx_liveness_upload(cx_ring *ring, const uint8_t *alive, const uint32_t *succ_lists, int ns,
                       int forward_rule, int memkind) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(ns >= 0 && ns <= 64, CX_E_INVALID, "ns must be in [0, 64]");
    CX_CHECK(forward_rule == CX_FWD_CHORD || forward_rule == CX_FWD_DHASH, CX_E_INVALID,
             "forward_rule must be CX_FWD_CHORD or CX_FWD_DHASH");
    CX_CHECK(memkind == CX_MEM_HOST || memkind == CX_MEM_DEVICE, CX_E_INVALID, "bad memkind");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    if (!alive && !succ_lists) {
        // reset: every peer alive with the converged lists = the converged
        // walk again (the route table and the arc calls apply once more)
        CX_HIP(hipStreamSynchronize(s));
        (void)hipFree(ring->d_alive);
        (void)hipFree(ring->d_succs);
        ring->d_alive = nullptr;
        ring->d_succs = nullptr;
        ring->succ_ns = 0;
        ring->fwd_rule = CX_FWD_CHORD;
        ring->liveness = false;
        return CX_OK;
    }
    const hipMemcpyKind kind =
        memkind == CX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    DBuf al, sl;
    if (alive) {
        CX_HIP(al.alloc(ring->n));
        CX_HIP(hipMemcpyAsync(al.p, alive, ring->n, kind, s));
    }
    if (succ_lists && ns > 0) {
        const size_t cnt = ring->n * (size_t)ns;
        CX_HIP(sl.alloc(cnt * sizeof(uint32_t)));
        CX_HIP(hipMemcpyAsync(sl.p, succ_lists, cnt * sizeof(uint32_t), kind, s));
        CX_HIP(hipMemsetAsync(ring->d_scratch, 0, sizeof(uint32_t), s));
        CX_HIP(cxk::check_indices(sl.as<uint32_t>(), cnt, (uint32_t)ring->n, true,
                                  ring->d_scratch, s));
        uint32_t bad = 0;
        CX_HIP(hipMemcpyAsync(&bad, ring->d_scratch, sizeof(bad), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
        CX_CHECK(!bad, CX_E_INVALID, "successor entry is neither a ring index nor CX_NONE");
    }
    CX_HIP(hipStreamSynchronize(s));
    (void)hipFree(ring->d_alive);
    (void)hipFree(ring->d_succs);
    ring->d_alive = al.as<uint8_t>();
    ring->d_succs = sl.as<uint32_t>();
    al.release();
    sl.release();
    ring->succ_ns = ns;
    ring->fwd_rule = forward_rule;
    ring->liveness = true;
    return CX_OK;
}

int cx_route(const cx_ring *ring, const uint32_t *src, const cx_u128 *keys, size_t q,
             uint32_t *owner, uint8_t *hops, uint8_t *status, int memkind) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(ring->d_fingers != nullptr || ring->rows_deferred, CX_E_STATE,
             "finger table not built (cx_fingers_build / cx_fingers_upload)");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    DBuf ts, tk, to, th, tst;
    const uint32_t *dsrc;
    const cx_u128 *dk;
    uint32_t *dow;
    uint8_t *dh, *dst = nullptr;
    if ((rc = stage_in(src, q, memkind, ts, &dsrc, s))) return rc;
    if ((rc = stage_in(keys, q, memkind, tk, &dk, s))) return rc;
    if ((rc = stage_out(owner, q, memkind, to, &dow, s))) return rc;
    if ((rc = stage_out(hops, q, memkind, th, &dh, s))) return rc;
    if (status && (rc = stage_out(status, q, memkind, tst, &dst, s))) return rc;
    if (!ring->literal()) {
        int e2 = ensure_route_table(const_cast<cx_ring *>(ring), s);
        if (e2) return e2;
    }
    const int v = ring->literal() ? -1 : ring->variant();
    if (v != 5 || !ring->cz_valid) {
        // every other walk reads the row-major finger table
        int e2 = ensure_fingers_rows(const_cast<cx_ring *>(ring), s);
        if (e2) return e2;
    }
    SearchView dsv = ring->sv();
    dsv.dir = ring->d_dir;
    if (v == 5 && ring->cz_valid)
        CX_HIP(cxk::route_walk(ring->d_ring_ext, ring->d_ring, ring->n, ring->d_cz, ring->rt_l0,
                               ring->pk_ib, dsv, dsrc, reinterpret_cast<const cell128 *>(dk), q,
                               dow, dh, dst, ring->counting ? ring->d_stats : nullptr, s));
    else if (v == 4 && ring->tree_valid)
        CX_HIP(cxk::route_tree(ring->d_ring_ext, ring->d_ring, ring->n, ring->d_tree, ring->rt_l0,
                               ring->rt_R, ring->pk_ib, ring->d_fingers, dsrc,
                               reinterpret_cast<const cell128 *>(dk), q, dow, dh, dst, s));
    else
        CX_HIP(cxk::route(ring->d_ring, ring->n, ring->d_fingers, ring->d_min_keys,
                          ring->d_preds, ring->lit(), ring->literal(), dsrc,
                          reinterpret_cast<const cell128 *>(dk), q, dow, dh, dst, s));
    if (memkind == CX_MEM_HOST && q) {
        CX_HIP(hipMemcpyAsync(owner, dow, q * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(hops, dh, q, hipMemcpyDeviceToHost, s));
        if (status) CX_HIP(hipMemcpyAsync(status, dst, q, hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
    }
    return CX_OK;
}

int cx_nsucc(const cx_ring *ring, const cx_u128 *keys, size_t q, int n, uint32_t *lists,
             uint8_t *count, int memkind) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(n >= 1 && n <= CX_MAX_NSUCC, CX_E_INVALID, "n must be in [1, 16]");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    DBuf tk, tl, tc;
    const cx_u128 *dk;
    uint32_t *dl;
    uint8_t *dc;
    if ((rc = stage_in(keys, q, memkind, tk, &dk, s))) return rc;
    if ((rc = stage_out(lists, q * (size_t)n, memkind, tl, &dl, s))) return rc;
    if ((rc = stage_out(count, q, memkind, tc, &dc, s))) return rc;
    CX_HIP(cxk::nsucc(ring->sv(), reinterpret_cast<const cell128 *>(dk), q, n, dl, dc, s));
    if (memkind == CX_MEM_HOST && q) {
        CX_HIP(hipMemcpyAsync(lists, dl, q * (size_t)n * sizeof(uint32_t),
                              hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(count, dc, q, hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
    }
    return CX_OK;
}

int cx_dhash_check(const cx_ring *ring, int n, int m) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(n >= 1 && m >= 1, CX_E_INVALID, "n and m must be positive");
    const size_t got = ring->n < (size_t)n ? ring->n : (size_t)n;
    if (got < (size_t)m)
        return fail(CX_E_INSUFFICIENT, "Insufficient succs in list to complete request.");
    return CX_OK;
}

int cx_churn(const cx_ring *old_ring, const cx_u128 *joins, size_t nj, const cx_u128 *leaves,
             size_t nl, int memkind, cx_ring **new_ring, uint32_t *old_to_new) {
    CX_CHECK(old_ring && new_ring, CX_E_INVALID, "null argument");
    *new_ring = nullptr;
    int rc = use_device(old_ring);
    if (rc) return rc;
    const size_t n_old = old_ring->n;
    CX_CHECK(n_old + nj < (size_t)CX_TAG_JOIN, CX_E_INVALID, "ring larger than 2^31 peers");
    cx_ring *r = nullptr;
    if ((rc = alloc_ring(old_ring->device, &r))) return rc;
    hipStream_t s = r->stream;
    // order the new handle's work after anything pending on the old one
    rc = [&]() -> int {
        CX_HIP(hipStreamSynchronize(old_ring->stream));
        DBuf tj, tl, gone, k0, k1, t0, t1, ws, pos, o2n, ringbuf;
        const cx_u128 *dj, *dl;
        int e;
        if ((e = stage_in(joins, nj, memkind, tj, &dj, s))) return e;
        if ((e = stage_in(leaves, nl, memkind, tl, &dl, s))) return e;
        if (old_ring->churn_variant == 1) {
            e = churn_merge(old_ring, reinterpret_cast<const cell128 *>(dj), nj,
                            reinterpret_cast<const cell128 *>(dl), nl, r, o2n, s);
            if (e) return e;
            r->search_variant = old_ring->search_variant;
            r->churn_variant = old_ring->churn_variant;
            r->misplaced_variant = old_ring->misplaced_variant;
            if ((e = build_search(r, s))) return e;
            if (old_to_new) {
                const hipMemcpyKind kind =
                    memkind == CX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
                CX_HIP(hipMemcpyAsync(old_to_new, o2n.p, n_old * sizeof(uint32_t), kind, s));
            }
            CX_HIP(hipStreamSynchronize(s));
            r->churn_parent = old_ring->serial;
            r->o2n_canon_n = n_old;
            r->d_o2n_canon = o2n.as<uint32_t>();
            r->parent_planes = old_ring->planes;  // the finger repair's input
            r->fingers_repair = old_ring->fingers_repair;
            o2n.release();
            return CX_OK;
        }
        CX_HIP(gone.alloc(n_old));
        CX_HIP(hipMemsetAsync(gone.p, 0, n_old, s));
        CX_HIP(cxk::mark_leaves(old_ring->sv(), old_ring->d_ring,
                                reinterpret_cast<const cell128 *>(dl), nl, gone.as<uint8_t>(), s));
        const size_t cap = n_old + nj;
        CX_HIP(k0.alloc(cap * sizeof(cell128)));
        CX_HIP(k1.alloc(cap * sizeof(cell128)));
        CX_HIP(t0.alloc(cap * sizeof(uint32_t)));
        CX_HIP(t1.alloc(cap * sizeof(uint32_t)));
        CX_HIP(pos.alloc(cap * sizeof(uint32_t)));
        const size_t sw = cxk::sort_workspace_words(cap), cw = cxk::scan_workspace_words(cap);
        CX_HIP(ws.alloc((sw > cw ? sw : cw) * sizeof(uint32_t)));
        CX_HIP(cxk::compact_survivors(old_ring->d_ring, gone.as<uint8_t>(), n_old,
                                      pos.as<uint32_t>(), ws.as<uint32_t>(), k0.as<cell128>(),
                                      t0.as<uint32_t>(), r->d_scratch, s));
        uint32_t ns = 0;
        CX_HIP(hipMemcpyAsync(&ns, r->d_scratch, sizeof(ns), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
        const size_t total = ns + nj;
        CX_CHECK(total >= 1, CX_E_INVALID, "churn would leave an empty ring");
        CX_HIP(cxk::copy_tagged(reinterpret_cast<const cell128 *>(dj), nj, CX_TAG_JOIN,
                                k0.as<cell128>() + ns, t0.as<uint32_t>() + ns, s));
        CX_HIP(cxk::radix_sort(k0.as<cell128>(), t0.as<uint32_t>(), k1.as<cell128>(),
                               t1.as<uint32_t>(), total, ws.as<uint32_t>(), s));
        CX_HIP(o2n.alloc(n_old * sizeof(uint32_t)));
        CX_HIP(cxk::fill_u32(o2n.as<uint32_t>(), n_old, CX_NONE, s));
        CX_HIP(ringbuf.alloc(total * sizeof(cell128)));
        CX_HIP(cxk::unique_sorted(k0.as<cell128>(), t0.as<uint32_t>(), total,
                                  pos.as<uint32_t>(), ws.as<uint32_t>(),
                                  ringbuf.as<cell128>(), o2n.as<uint32_t>(), r->d_scratch, s));
        uint32_t m = 0;
        CX_HIP(hipMemcpyAsync(&m, r->d_scratch, sizeof(m), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
        CX_CHECK(m >= 1 && m <= total, CX_E_HIP, "churn produced an invalid ring size");
        r->n = m;
        r->ring_cap = total;
        r->d_ring = ringbuf.as<cell128>();
        ringbuf.release();
        r->search_variant = old_ring->search_variant;
        r->churn_variant = old_ring->churn_variant;
        r->misplaced_variant = old_ring->misplaced_variant;
        {
            int e2 = build_search(r, s);
            if (e2) return e2;
        }
        if (old_to_new) {
            const hipMemcpyKind kind =
                memkind == CX_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
            CX_HIP(hipMemcpyAsync(old_to_new, o2n.p, n_old * sizeof(uint32_t), kind, s));
        }
        CX_HIP(hipStreamSynchronize(s));
        r->churn_parent = old_ring->serial;
        r->o2n_canon_n = n_old;
        r->d_o2n_canon = o2n.as<uint32_t>();
        r->parent_planes = old_ring->planes;  // the finger repair's input
        r->fingers_repair = old_ring->fingers_repair;
        o2n.release();
        return CX_OK;
    }();
    if (rc) {
        free_ring(r);
        return rc;
    }
    *new_ring = r;
    return CX_OK;
}

// cx_misplaced, and with old_lists / old_count the fused cx_dhash_maintenance
static int misplaced_impl(const cx_ring *old_ring, const cx_ring *new_ring,
                          const uint32_t *old_to_new, const cx_u128 *keys, size_t q, int n,
                          uint32_t *old_lists, uint8_t *old_count, uint32_t *new_lists,
                          uint8_t *count, uint16_t *mask, uint8_t *target, int memkind) {
    CX_CHECK(old_ring && new_ring, CX_E_INVALID, "null ring");
    CX_CHECK(old_ring->device == new_ring->device, CX_E_INVALID, "rings on different devices");
    CX_CHECK(n >= 1 && n <= CX_MAX_NSUCC, CX_E_INVALID, "n must be in [1, 16]");
    int rc = use_device(new_ring);
    if (rc) return rc;
    hipStream_t s = new_ring->stream;
    // misplaced_churn searches both rings with the Eytzinger copy when either
    // ring's directory is off (search variant 0): make sure both have one
    if (!old_ring->sv().dir || !new_ring->sv().dir) {
        if ((rc = ensure_eyt(const_cast<cx_ring *>(old_ring), s))) return rc;
        if ((rc = ensure_eyt(const_cast<cx_ring *>(new_ring), s))) return rc;
    }
    DBuf to2n, tk, tl, tc, tm, tt, tol, toc;
    const uint32_t *d_o2n;
    const cx_u128 *dk;
    uint32_t *dl, *dol = nullptr;
    uint8_t *dc, *dt, *doc = nullptr;
    uint16_t *dm;
    const bool fused = old_lists != nullptr;
    if ((rc = stage_in(old_to_new, old_ring->n, memkind, to2n, &d_o2n, s))) return rc;
    if ((rc = stage_in(keys, q, memkind, tk, &dk, s))) return rc;
    if ((rc = stage_out(new_lists, q * (size_t)n, memkind, tl, &dl, s))) return rc;
    if ((rc = stage_out(count, q, memkind, tc, &dc, s))) return rc;
    if ((rc = stage_out(mask, q, memkind, tm, &dm, s))) return rc;
    if ((rc = stage_out(target, q * (size_t)n, memkind, tt, &dt, s))) return rc;
    if (fused) {
        if ((rc = stage_out(old_lists, q * (size_t)n, memkind, tol, &dol, s))) return rc;
        if ((rc = stage_out(old_count, q, memkind, toc, &doc, s))) return rc;
    }
    // churn directory: the new ring came from cx_churn(old_ring) and the
    // caller's mapping equals the one it returned (checked on the device)
    cxk::ChurnDirArgs cda{};
    const bool cd_ok = q && new_ring->misplaced_variant == 1 &&
                       new_ring->churn_parent == old_ring->serial && new_ring->d_o2n_canon &&
                       new_ring->o2n_canon_n == old_ring->n && old_ring->n >= 32 &&
                       new_ring->n >= 32 && old_ring->d_dir && new_ring->d_dir &&
                       old_ring->search_variant != 0 && new_ring->search_variant != 0;
    if (cd_ok) {
        cx_ring *nr = const_cast<cx_ring *>(new_ring);
        if (!nr->d_cdir) {
            const size_t Mmax = old_ring->n + new_ring->n;
            int kb = 1;
            // load factor <= 1/4: a key whose bucket holds a third entry before
            // it takes the two-search path, and at 1/2 (~0.8 % of keys) nearly half
            // the waves waited for one (3.29 vs 3.03 ms at C5, profiles/r05/c5_cdkb/)
            while (((size_t)1 << kb) < 2 * Mmax) ++kb;
            const size_t bytes = ((size_t)1 << kb) * 32;
            DBuf ws, lo, sw;
            CX_HIP(ws.alloc_pooled(cxk::churn_dir_workspace_bytes(old_ring->n, new_ring->n), s));
            CX_HIP(lo.alloc((((size_t)1 << kb) + 1) * sizeof(uint32_t)));
            CX_HIP(sw.alloc(cxk::scan_workspace_words(Mmax + 1) * sizeof(uint32_t)));
            void *cdp = nullptr;
            CX_CHECK(table_alloc(&cdp, bytes) == hipSuccess, CX_E_NOMEM,
                     "hipMalloc of the churn directory failed");
            uint32_t M = 0;
            hipError_t e = cxk::churn_dir_build(old_ring->sv(), new_ring->sv(), nr->d_o2n_canon,
                                                kb, ws.p, lo.as<uint32_t>(),
                                                static_cast<uint4 *>(cdp), sw.as<uint32_t>(), &M,
                                                s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e != hipSuccess) {
                table_free(nr->device, cdp, bytes);
                return fail(CX_E_HIP, std::string("churn directory: ") + hipGetErrorString(e));
            }
            nr->d_cdir = static_cast<uint4 *>(cdp);
            nr->cdir_kb = kb;
            nr->cdir_bytes = bytes;
        }
        uint32_t *ok = new_ring->d_scratch + 250;
        CX_HIP(cxk::churn_dir_same(d_o2n, new_ring->d_o2n_canon, old_ring->n, ok, s));
        cda = cxk::ChurnDirArgs{new_ring->d_cdir, new_ring->cdir_kb, ok};
    }
    CX_HIP(cxk::misplaced_churn(old_ring->sv(), new_ring->sv(), d_o2n,
                                reinterpret_cast<const cell128 *>(dk), q, n, dl, dc, dm, dt,
                                cd_ok ? &cda : nullptr, s, dol, doc));
    if (memkind == CX_MEM_HOST && q) {
        CX_HIP(hipMemcpyAsync(new_lists, dl, q * (size_t)n * 4, hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(count, dc, q, hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(mask, dm, q * 2, hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(target, dt, q * (size_t)n, hipMemcpyDeviceToHost, s));
        if (fused) {
            CX_HIP(hipMemcpyAsync(old_lists, dol, q * (size_t)n * 4, hipMemcpyDeviceToHost, s));
            CX_HIP(hipMemcpyAsync(old_count, doc, q, hipMemcpyDeviceToHost, s));
        }
        CX_HIP(hipStreamSynchronize(s));
    }
    return CX_OK;
}

int cx_misplaced(const cx_ring *old_ring, const cx_ring *new_ring, const uint32_t *old_to_new,
                 const cx_u128 *keys, size_t q, int n, uint32_t *new_lists, uint8_t *count,
                 uint16_t *mask, uint8_t *target, int memkind) {
    return misplaced_impl(old_ring, new_ring, old_to_new, keys, q, n, nullptr, nullptr, new_lists,
                          count, mask, target, memkind);
}

int cx_dhash_maintenance(const cx_ring *old_ring, const cx_ring *new_ring,
                         const uint32_t *old_to_new, const cx_u128 *keys, size_t q, int n,
                         uint32_t *old_lists, uint8_t *old_count, uint32_t *new_lists,
                         uint8_t *count, uint16_t *mask, uint8_t *target, int memkind) {
    CX_CHECK(old_lists && old_count, CX_E_INVALID, "null old_lists / old_count");
    return misplaced_impl(old_ring, new_ring, old_to_new, keys, q, n, old_lists, old_count,
                          new_lists, count, mask, target, memkind);
}

int cx_misplaced_holders(const cx_ring *ring, const cx_u128 *keys, size_t q,
                         const uint32_t *holders, int nh, int n, uint32_t *new_lists,
                         uint8_t *count, uint16_t *mask, uint8_t *target, int memkind) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(n >= 1 && n <= CX_MAX_NSUCC, CX_E_INVALID, "n must be in [1, 16]");
    CX_CHECK(nh >= 1 && nh <= CX_MAX_NSUCC, CX_E_INVALID, "nh must be in [1, 16]");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    DBuf th, tk, tl, tc, tm, tt;
    const uint32_t *dh;
    const cx_u128 *dk;
    uint32_t *dl;
    uint8_t *dc, *dt;
    uint16_t *dm;
    if ((rc = stage_in(holders, q * (size_t)nh, memkind, th, &dh, s))) return rc;
    if ((rc = stage_in(keys, q, memkind, tk, &dk, s))) return rc;
    if ((rc = stage_out(new_lists, q * (size_t)n, memkind, tl, &dl, s))) return rc;
    if ((rc = stage_out(count, q, memkind, tc, &dc, s))) return rc;
    if ((rc = stage_out(mask, q, memkind, tm, &dm, s))) return rc;
    if ((rc = stage_out(target, q * (size_t)nh, memkind, tt, &dt, s))) return rc;
    CX_HIP(cxk::misplaced_holders(ring->sv(), dh, nh, reinterpret_cast<const cell128 *>(dk), q,
                                  n, dl, dc, dm, dt, s));
    if (memkind == CX_MEM_HOST && q) {
        CX_HIP(hipMemcpyAsync(new_lists, dl, q * (size_t)n * 4, hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(count, dc, q, hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(mask, dm, q * 2, hipMemcpyDeviceToHost, s));
        CX_HIP(hipMemcpyAsync(target, dt, q * (size_t)nh, hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
    }
    return CX_OK;
}

int cx_in_between(const cx_u256 *v, const cx_u256 *lb, const cx_u256 *ub, size_t q,
                  int inclusive, uint8_t *out, int memkind) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(CX_E_HIP, "no HIP device: chordx has no host compute path");
    hipStream_t s = nullptr;  // default stream of the current device
    DBuf tv, tl, tu, to;
    const cx_u256 *dv, *dl, *du;
    uint8_t *dout;
    int rc;
    if ((rc = stage_in(v, q, memkind, tv, &dv, s))) return rc;
    if ((rc = stage_in(lb, q, memkind, tl, &dl, s))) return rc;
    if ((rc = stage_in(ub, q, memkind, tu, &du, s))) return rc;
    if ((rc = stage_out(out, q, memkind, to, &dout, s))) return rc;
    CX_HIP(cxk::in_between(dv, dl, du, q, inclusive, dout, s));
    if (memkind == CX_MEM_HOST && q) {
        CX_HIP(hipMemcpyAsync(out, dout, q, hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
    }
    return CX_OK;
}

int cx_uuid5_dns(const uint8_t *bytes, const uint64_t *offsets, size_t count, cx_u128 *out,
                 int memkind, int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(CX_E_HIP, "no HIP device: chordx has no host compute path");
    CX_CHECK(device >= 0 && device < ndev, CX_E_INVALID, "bad device ordinal");
    if (count == 0) return CX_OK;
    CX_CHECK(offsets != nullptr && out != nullptr, CX_E_INVALID, "null argument");
    CX_HIP(hipSetDevice(device));
    hipStream_t s = nullptr;
    DBuf to, tb, tout;
    const uint64_t *doff;
    const uint8_t *dbytes;
    cx_u128 *dout;
    int rc;
    if ((rc = stage_in(offsets, count + 1, memkind, to, &doff, s))) return rc;
    uint64_t nbytes = 0;
    if (memkind == CX_MEM_HOST) {
        nbytes = offsets[count];
        CX_CHECK(offsets[0] == 0, CX_E_INVALID, "offsets[0] must be 0");
        for (size_t i = 0; i < count; ++i)
            CX_CHECK(offsets[i] <= offsets[i + 1], CX_E_INVALID, "offsets not ascending");
    } else {
        CX_HIP(hipMemcpy(&nbytes, offsets + count, sizeof(nbytes), hipMemcpyDeviceToHost));
    }
    if ((rc = stage_in(bytes, (size_t)nbytes, memkind, tb, &dbytes, s))) return rc;
    if ((rc = stage_out(out, count, memkind, tout, &dout, s))) return rc;
    CX_HIP(cxk::uuid5(dbytes, doff, count, reinterpret_cast<cell128 *>(dout), s));
    return finish_out(out, dout, count, memkind, s);
}

int cx_fill_splitmix(cx_u128 *out_device, size_t count, uint64_t seed, uint64_t offset,
                     int device, void *hip_stream) {
    CX_CHECK(out_device || count == 0, CX_E_INVALID, "null output");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(CX_E_HIP, "no HIP device: chordx has no host compute path");
    CX_HIP(hipSetDevice(device));
    CX_HIP(cxk::fill_splitmix(reinterpret_cast<cell128 *>(out_device), count, seed, offset,
                              static_cast<hipStream_t>(hip_stream)));
    return CX_OK;
}

int cx_hex_parse(const uint8_t *bytes, const uint64_t *offsets, size_t count, cx_u128 *out,
                 uint8_t *ok, int memkind, int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(CX_E_HIP, "no HIP device: chordx has no host compute path");
    CX_CHECK(device >= 0 && device < ndev, CX_E_INVALID, "bad device ordinal");
    if (count == 0) return CX_OK;
    CX_CHECK(offsets && out && ok, CX_E_INVALID, "null argument");
    CX_HIP(hipSetDevice(device));
    hipStream_t s = nullptr;
    DBuf to, tb, tout, tok;
    const uint64_t *doff;
    const uint8_t *dbytes;
    cx_u128 *dout;
    uint8_t *dok;
    int rc;
    if ((rc = stage_in(offsets, count + 1, memkind, to, &doff, s))) return rc;
    uint64_t nbytes = 0;
    if (memkind == CX_MEM_HOST) {
        nbytes = offsets[count];
        CX_CHECK(offsets[0] == 0, CX_E_INVALID, "offsets[0] must be 0");
        for (size_t i = 0; i < count; ++i)
            CX_CHECK(offsets[i] <= offsets[i + 1], CX_E_INVALID, "offsets not ascending");
    } else {
        CX_HIP(hipMemcpy(&nbytes, offsets + count, sizeof(nbytes), hipMemcpyDeviceToHost));
    }
    if ((rc = stage_in(bytes, (size_t)nbytes, memkind, tb, &dbytes, s))) return rc;
    if ((rc = stage_out(out, count, memkind, tout, &dout, s))) return rc;
    if ((rc = stage_out(ok, count, memkind, tok, &dok, s))) return rc;
    CX_HIP(cxk::hex_parse(dbytes, doff, count, reinterpret_cast<cell128 *>(dout), dok, s));
    if ((rc = finish_out(ok, dok, count, memkind, s))) return rc;
    return finish_out(out, dout, count, memkind, s);
}

int cx_hex_format(const cx_u128 *keys, size_t count, char *out, uint8_t *len, int memkind,
                  int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(CX_E_HIP, "no HIP device: chordx has no host compute path");
    CX_CHECK(device >= 0 && device < ndev, CX_E_INVALID, "bad device ordinal");
    if (count == 0) return CX_OK;
    CX_CHECK(keys && out && len, CX_E_INVALID, "null argument");
    CX_HIP(hipSetDevice(device));
    hipStream_t s = nullptr;
    DBuf tk, tout, tlen;
    const cx_u128 *dk;
    char *dout;
    uint8_t *dlen;
    int rc;
    if ((rc = stage_in(keys, count, memkind, tk, &dk, s))) return rc;
    if ((rc = stage_out(out, count * 32, memkind, tout, &dout, s))) return rc;
    if ((rc = stage_out(len, count, memkind, tlen, &dlen, s))) return rc;
    CX_HIP(cxk::hex_format(reinterpret_cast<const cell128 *>(dk), count, dout, dlen, s));
    if ((rc = finish_out(len, dlen, count, memkind, s))) return rc;
    return finish_out(out, dout, count * 32, memkind, s);
}

// ---- Rabin IDA --------------------------------------------------------------
namespace {
int ida_check(int n, int m, int p) {
    CX_CHECK(m >= 1 && n > m && n <= 32, CX_E_INVALID, "IDA needs 1 <= m < n <= 32");
    CX_CHECK(p > n && p <= 46340, CX_E_INVALID, "IDA needs n < p <= 46340");  // ida.cpp:54-56
    return CX_OK;
}

int device_ok(int device) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(CX_E_HIP, "no HIP device: chordx has no host compute path");
    CX_CHECK(device >= 0 && device < ndev, CX_E_INVALID, "bad device ordinal");
    CX_HIP(hipSetDevice(device));
    return CX_OK;
}

// Host copy of a (blocks + 1) offset array given in either memory kind.
int host_offsets(const uint64_t *offs, size_t blocks, int memkind, std::vector<uint64_t> &h) {
    h.resize(blocks + 1);
    if (memkind == CX_MEM_DEVICE)
        CX_HIP(hipMemcpy(h.data(), offs, (blocks + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost));
    else
        std::memcpy(h.data(), offs, (blocks + 1) * sizeof(uint64_t));
    CX_CHECK(h[0] == 0, CX_E_INVALID, "offsets[0] must be 0");
    for (size_t b = 0; b < blocks; ++b)
        CX_CHECK(h[b] <= h[b + 1], CX_E_INVALID, "offsets not ascending");
    return CX_OK;
}
}  // namespace

int cx_ida_segments(const uint64_t *offsets, size_t blocks, int m, uint64_t *seg_offsets) {
    CX_CHECK(offsets && seg_offsets && m >= 1, CX_E_INVALID, "bad argument");
    seg_offsets[0] = 0;
    for (size_t b = 0; b < blocks; ++b) {
        CX_CHECK(offsets[b] <= offsets[b + 1], CX_E_INVALID, "offsets not ascending");
        seg_offsets[b + 1] = seg_offsets[b] + (offsets[b + 1] - offsets[b] + m - 1) / m;
    }
    return CX_OK;
}

int cx_ida_encode(const uint8_t *data, const uint64_t *offsets, const uint64_t *seg_offsets,
                  size_t blocks, int n, int m, int p, uint16_t *frags, int memkind,
                  int device) {
    int rc;
    if ((rc = ida_check(n, m, p))) return rc;
    if ((rc = device_ok(device))) return rc;
    if (blocks == 0) return CX_OK;
    CX_CHECK(offsets && seg_offsets, CX_E_INVALID, "null argument");
    hipStream_t s = nullptr;
    if (memkind == CX_MEM_DEVICE) {  // device-resident: no host round trip
        CX_CHECK(frags != nullptr, CX_E_INVALID, "null argument");
        CX_HIP(cxk::ida_encode(data, offsets, seg_offsets, blocks, n, m, p, frags, s));
        return CX_OK;
    }
    CX_CHECK(memkind == CX_MEM_HOST, CX_E_INVALID, "bad memkind");
    std::vector<uint64_t> ho, hs;
    if ((rc = host_offsets(offsets, blocks, memkind, ho))) return rc;
    if ((rc = host_offsets(seg_offsets, blocks, memkind, hs))) return rc;
    for (size_t b = 0; b < blocks; ++b)
        CX_CHECK(hs[b + 1] - hs[b] == (ho[b + 1] - ho[b] + m - 1) / m, CX_E_INVALID,
                 "seg_offsets do not match offsets (cx_ida_segments)");
    const uint64_t segs = hs[blocks], nbytes = ho[blocks];
    DBuf td, to, tseg, tf;
    const uint8_t *dd;
    const uint64_t *doff, *dseg;
    uint16_t *df;
    if ((rc = stage_in(data, (size_t)nbytes, memkind, td, &dd, s))) return rc;
    if ((rc = stage_in(offsets, blocks + 1, memkind, to, &doff, s))) return rc;
    if ((rc = stage_in(seg_offsets, blocks + 1, memkind, tseg, &dseg, s))) return rc;
    if ((rc = stage_out(frags, (size_t)(segs * n), memkind, tf, &df, s))) return rc;
    CX_HIP(cxk::ida_encode(dd, doff, dseg, blocks, n, m, p, df, s));
    return finish_out(frags, df, (size_t)(segs * n), memkind, s);
}

int cx_ida_decode(const uint16_t *frags, const uint64_t *seg_offsets, const uint8_t *indices,
                  size_t blocks, int m, int p, uint16_t *out, uint64_t *out_len, int memkind,
                  int device) {
    int rc;
    CX_CHECK(m >= 1 && m < 32 && p > m + 1 && p <= 46340, CX_E_INVALID,
             "IDA needs 1 <= m < 32, m + 1 < p <= 46340");
    if ((rc = device_ok(device))) return rc;
    if (blocks == 0) return CX_OK;
    CX_CHECK(seg_offsets && indices && out_len, CX_E_INVALID, "null argument");
    CX_CHECK(blocks < (1ull << 32), CX_E_INVALID, "too many blocks");
    CX_CHECK(memkind == CX_MEM_HOST || memkind == CX_MEM_DEVICE, CX_E_INVALID, "bad memkind");
    hipStream_t s = nullptr;
    uint64_t segs = 0;
    if (memkind == CX_MEM_HOST) {
        std::vector<uint64_t> hs;
        if ((rc = host_offsets(seg_offsets, blocks, memkind, hs))) return rc;
        segs = hs[blocks];
        CX_CHECK(segs == 0 || (frags && out), CX_E_INVALID, "null argument");
    }
    DBuf tf, tsg, ti, tout, tlen;
    const uint16_t *dfr = frags;
    const uint64_t *dseg = seg_offsets;
    const uint8_t *didx = indices;
    uint16_t *dout = out;
    uint64_t *dlen = out_len;
    if (memkind == CX_MEM_HOST) {
        if ((rc = stage_in(frags, (size_t)(segs * m), memkind, tf, &dfr, s))) return rc;
        if ((rc = stage_in(seg_offsets, blocks + 1, memkind, tsg, &dseg, s))) return rc;
        if ((rc = stage_in(indices, blocks * (size_t)m, memkind, ti, &didx, s))) return rc;
        if ((rc = stage_out(out, (size_t)(segs * m), memkind, tout, &dout, s))) return rc;
        if ((rc = stage_out(out_len, blocks, memkind, tlen, &dlen, s))) return rc;
    }
    // runs of equal index lists share one inverse
    IdaArena &arena = ida_arena(device);
    std::lock_guard<std::mutex> lock(arena.mu);
    uint32_t *flag, *flag2, *ws, *run_of, *run_start, *guard, *err;
    int32_t *inv;
    uint8_t *okf;
    CX_HIP(arena_carve(arena, 0,
                       {sizeof(uint32_t), blocks * sizeof(uint32_t), blocks * sizeof(uint32_t),
                        cxk::scan_workspace_words(blocks) * sizeof(uint32_t)},
                       {(void **)&err, (void **)&flag, (void **)&flag2, (void **)&ws}));
    CX_HIP(hipMemsetAsync(err, 0, sizeof(uint32_t), s));
    CX_HIP(cxk::ida_runs(didx, blocks, m, flag, s));
    CX_HIP(hipMemcpyAsync(flag2, flag, blocks * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
    CX_HIP(cxk::exclusive_scan(flag2, blocks, ws, s));
    uint32_t last[2] = {0, 0};
    CX_HIP(hipMemcpyAsync(&last[0], flag2 + blocks - 1, 4, hipMemcpyDeviceToHost, s));
    CX_HIP(hipMemcpyAsync(&last[1], flag + blocks - 1, 4, hipMemcpyDeviceToHost, s));
    CX_HIP(hipStreamSynchronize(s));
    const size_t runs = (size_t)last[0] + last[1];
    CX_CHECK(runs >= 1 && runs <= blocks, CX_E_HIP, "IDA decode: invalid run count");
    CX_HIP(arena_carve(arena, 1,
                       {blocks * sizeof(uint32_t), runs * sizeof(uint32_t),
                        runs * (size_t)m * m * sizeof(int32_t),
                        IDA_GUARD_WORDS * sizeof(uint32_t), runs},
                       {(void **)&run_of, (void **)&run_start, (void **)&inv, (void **)&guard,
                        (void **)&okf}));
    CX_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(guard), IDA_GUARD_WORD,
                             IDA_GUARD_WORDS, s));
    CX_HIP(cxk::ida_run_index(flag2, flag, blocks, runs, run_of, run_start, err, s));
    CX_HIP(cxk::ida_inverse(didx, run_start, runs, blocks, m, p, inv, okf, err, s));
    CX_HIP(hipMemsetAsync(dlen, 0, blocks * sizeof(uint64_t), s));
    CX_HIP(cxk::ida_decode(dfr, dseg, blocks, m, p, inv, run_of, runs, okf, dout, dlen, err, s));
    CX_HIP(cxk::ida_mark_failed(run_of, okf, blocks, runs, dlen, err, s));
    CX_HIP(cxk::ida_check_guard(guard, IDA_GUARD_WORDS, err, s));
    if (memkind == CX_MEM_HOST) {
        if ((rc = finish_out(out_len, dlen, blocks, memkind, s))) return rc;
        if ((rc = finish_out(out, dout, (size_t)(segs * m), memkind, s))) return rc;
    }
    // the bounds / guard word, on both memory kinds (4 B and one wait on the
    // null stream; the next call clears it, so it is read before returning)
    uint32_t e = 0;
    CX_HIP(hipMemcpyAsync(&e, err, sizeof(e), hipMemcpyDeviceToHost, s));
    CX_HIP(hipStreamSynchronize(s));
    CX_CHECK(e == 0, CX_E_HIP,
             "IDA decode: index bounds check failed (flags " + std::to_string(e) + ")");
    return CX_OK;
}

// ---- arc-sharded routing --------------------------------------------------
int cx_arc_build(cx_ring *ring, int world, int rank, int top_levels) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(world >= 1 && world <= CX_ARC_MAX_RANKS, CX_E_INVALID, "world must be in [1, 64]");
    CX_CHECK(rank >= 0 && rank < world, CX_E_INVALID, "rank out of range");
    CX_CHECK(top_levels >= 0 && top_levels <= (int)CX_FINGERS, CX_E_INVALID,
             "top_levels must be in [0, 128]");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    const size_t n = ring->n;
    // the converged finger table (streaming build; no route table); one built
    // here only to derive the planes is released afterwards (the walk finds
    // exact below-table fingers by directory search)
    // arc routing walks the converged table: refuse state it would ignore
    CX_CHECK(!ring->edited(), CX_E_STATE,
             "arc routing walks the converged ring; peer-state / liveness uploads need cx_route");
    CX_CHECK(!ring->d_fingers || ring->fingers_converged, CX_E_STATE,
             "arc routing walks the converged ring; uploaded fingers need cx_route");
    if ((rc = ensure_fingers_rows(ring, s))) return rc;  // deferred rows: written now
    const bool own_fingers = !ring->d_fingers;
    if (own_fingers) {
        if (!ring->d_fingers &&
            table_alloc((void **)&ring->d_fingers, n * CX_FINGERS * sizeof(uint32_t)) != hipSuccess) {
            ring->d_fingers = nullptr;
            return fail(CX_E_NOMEM, "hipMalloc of the finger table failed");
        }
        if ((rc = build_fingers_table(ring, s))) return rc;
    }
    route_geometry(ring);
    if (!ring->d_ring_ext) {
        CX_HIP(dev_malloc(&ring->d_ring_ext, (n + 1) * sizeof(cell128)));
        CX_HIP(cxk::ring_ext_build(ring->d_ring, n, ring->d_ring_ext, s));
    }
    const int l0 = ring->rt_l0;
    int Lh = (int)CX_FINGERS - (top_levels ? top_levels : CX_ARC_TOP_LEVELS);
    if (Lh < l0) Lh = l0;
    const uint32_t lo = (uint32_t)((uint64_t)rank * n / world);
    const uint32_t hi = (uint32_t)((uint64_t)(rank + 1) * n / world);
    // local rows: the arc and the peers with IDs within 2^Lh before its first
    // (a walk that needs a row below Lh is within 2^Lh of its key)
    uint32_t plo = lo, M = hi - lo;
    if (world == 1) {
        plo = 0;
        M = (uint32_t)n;
    } else if (hi > lo) {
        cell128 prev;
        CX_HIP(hipMemcpy(&prev, ring->d_ring + (lo == 0 ? n - 1 : lo - 1), sizeof(prev),
                         hipMemcpyDeviceToHost));
        const cell128 start = to_cell(to_u128(prev) - ((u128)1 << Lh) + 1);
        cell128 *dk = reinterpret_cast<cell128 *>(ring->d_scratch + 192);
        uint32_t *dout = ring->d_scratch + 188;
        CX_HIP(hipMemcpyAsync(dk, &start, sizeof(start), hipMemcpyHostToDevice, s));
        SearchView v = ring->sv();
        v.dir = ring->d_dir;
        CX_HIP(cxk::successor(v, dk, 1, dout, s));
        CX_HIP(hipMemcpyAsync(&plo, dout, sizeof(plo), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
        const uint64_t halo = ((uint64_t)lo + n - plo) % n;
        if (halo + (hi - lo) >= n) {
            plo = 0;
            M = (uint32_t)n;
        } else {
            M = (uint32_t)(halo + (hi - lo));
        }
    }
    (void)hipStreamSynchronize(s);
    table_free(ring->device, ring->d_arc_tree, ring->arc_bytes);
    ring->d_arc_tree = nullptr;
    ring->arc_bytes = 0;
    ring->arc_world = 0;
    const size_t top_ent = (size_t)((int)CX_FINGERS - Lh) * 2 * n;
    const size_t low_ent = (size_t)(Lh - l0) * 2 * M;
    if (table_alloc((void **)&ring->d_arc_tree, (top_ent + low_ent) * 64 + 64) != hipSuccess) {
        ring->d_arc_tree = nullptr;
        return fail(CX_E_NOMEM, "hipMalloc of the arc route planes failed");
    }
    ring->arc_bytes = (top_ent + low_ent) * 64 + 64;
    CX_HIP(hipMemsetAsync(ring->d_scratch, 0, 2 * sizeof(uint32_t), s));
    {
        DBuf ft, hi, c2;
        cxk::FingerView fv;
        CX_HIP(finger_planes(ring, l0, ft, fv, hi, c2, s, nullptr));
        DBuf ws;  // the default build's overflow list (sized for the larger part)
        if (fv.roots >= 2) {
            const size_t w0 = cxk::cz_build_ws_words(n, Lh, (int)CX_FINGERS - Lh, (uint32_t)n);
            const size_t w1 = cxk::cz_build_ws_words(n, l0, Lh - l0, M);
            CX_HIP(ws.alloc_pooled((w0 > w1 ? w0 : w1) * sizeof(uint32_t), s));
        }
        CX_HIP(cxk::cz_build_part(fv, ring->d_ring, hi.as<uint64_t>(), n, Lh, (int)CX_FINGERS - Lh, 0, (uint32_t)n,
                                  ring->pk_ib, ring->d_arc_tree, ring->d_scratch, s, ws.as<uint32_t>()));
        CX_HIP(cxk::cz_build_part(fv, ring->d_ring, hi.as<uint64_t>(), n, l0, Lh - l0, plo, M, ring->pk_ib,
                                  ring->d_arc_tree + top_ent * 8, ring->d_scratch, s, ws.as<uint32_t>()));
        uint32_t esc[2] = {0, 0};
        CX_HIP(hipMemcpyAsync(esc, ring->d_scratch, sizeof(esc), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));  // ft and hi are freed at scope end
        CX_CHECK(esc[1] == 0, CX_E_STATE, "route-table build met a finger out of range");
    }
    // WALK destinations: the last peer ID of every non-empty arc, ascending
    std::vector<ArcBound> b;
    for (int g = 0; g < world; ++g) {
        const uint64_t glo = (uint64_t)g * n / world, ghi = (uint64_t)(g + 1) * n / world;
        if (ghi <= glo) continue;
        cell128 id;
        CX_HIP(hipMemcpy(&id, ring->d_ring + ghi - 1, sizeof(id), hipMemcpyDeviceToHost));
        b.push_back(ArcBound{id.lo, id.hi, (uint32_t)g, 0});
    }
    (void)hipFree(ring->d_arc_bounds);
    ring->d_arc_bounds = nullptr;
    CX_HIP(dev_malloc(&ring->d_arc_bounds, b.size() * sizeof(ArcBound)));
    CX_HIP(hipMemcpy(ring->d_arc_bounds, b.data(), b.size() * sizeof(ArcBound),
                     hipMemcpyHostToDevice));
    CX_HIP(hipStreamSynchronize(s));
    if (own_fingers) {
        table_free(ring->device, ring->d_fingers, ring->n * CX_FINGERS * sizeof(uint32_t));
        ring->d_fingers = nullptr;
        ring->fingers_converged = false;
    }
    ring->arc_world = world;
    ring->arc_rank = rank;
    ring->arc_Lh = Lh;
    ring->arc_plo = plo;
    ring->arc_M = M;
    ring->arc_nb = (int)b.size();
    return CX_OK;
}

int cx_arc_info(const cx_ring *ring, int *top_levels, uint64_t *local_rows,
                uint64_t *table_bytes) {
    CX_CHECK(ring && top_levels && local_rows && table_bytes, CX_E_INVALID, "null argument");
    CX_CHECK(ring->arc_world > 0, CX_E_STATE, "arc not built (cx_arc_build)");
    *top_levels = (int)CX_FINGERS - ring->arc_Lh;
    *local_rows = ring->arc_M;
    *table_bytes = ((uint64_t)((int)CX_FINGERS - ring->arc_Lh) * 2 * ring->n +
                    (uint64_t)(ring->arc_Lh - ring->rt_l0) * 2 * ring->arc_M) * 64;
    return CX_OK;
}

int cx_arc_seed(const cx_ring *ring, int rank, const uint32_t *src, const cx_u128 *keys,
                size_t q, cx_arc_rec *out) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(rank >= 0 && rank < CX_ARC_MAX_RANKS, CX_E_INVALID, "rank out of range");
    CX_CHECK(q < (1ull << ARC_ORIGIN_SHIFT), CX_E_INVALID, "too many lookups for one rank");
    CX_CHECK(q == 0 || (src && keys && out), CX_E_INVALID, "null buffer");
    int rc = use_device(ring);
    if (rc) return rc;
    CX_HIP(cxk::arc_seed(src, reinterpret_cast<const cell128 *>(keys), q, rank,
                         reinterpret_cast<ArcRec *>(out), ring->stream));
    return CX_OK;
}

int cx_arc_step(const cx_ring *ring, int rank, const cx_arc_rec *in, size_t q, cx_arc_rec *out,
                uint32_t *owner, uint8_t *hops, uint8_t *status) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(ring->arc_world > 0 && ring->d_arc_tree, CX_E_STATE, "arc not built (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    CX_CHECK(rank == ring->arc_rank, CX_E_INVALID, "rank differs from the one cx_arc_build used");
    CX_CHECK(rank >= 0 && rank < CX_ARC_MAX_RANKS, CX_E_INVALID, "rank out of range");
    CX_CHECK(q == 0 || (in && out && owner && hops), CX_E_INVALID, "null buffer");
    int rc = use_device(ring);
    if (rc) return rc;
    SearchView v = ring->sv();
    v.dir = ring->d_dir;  // exact below-table fingers by directory search
    CX_HIP(cxk::route_arc(ring->d_ring_ext, ring->d_ring, ring->n, ring->d_arc_tree, ring->rt_l0,
                          ring->rt_R, ring->pk_ib, v, ring->arc_Lh, ring->arc_plo,
                          ring->arc_M, rank, reinterpret_cast<const ArcRec *>(in), nullptr,
                          nullptr, q, reinterpret_cast<ArcRec *>(out), owner, hops, status,
                          ring->stream));
    return CX_OK;
}

int cx_arc_start(const cx_ring *ring, int rank, const uint32_t *src, const cx_u128 *keys,
                 size_t q, cx_arc_rec *out, uint32_t *owner, uint8_t *hops, uint8_t *status) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(ring->arc_world > 0 && ring->d_arc_tree, CX_E_STATE, "arc not built (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    CX_CHECK(rank == ring->arc_rank, CX_E_INVALID, "rank differs from the one cx_arc_build used");
    CX_CHECK(q < (1ull << ARC_ORIGIN_SHIFT), CX_E_INVALID, "too many lookups for one rank");
    CX_CHECK(q == 0 || (src && keys && out && owner && hops), CX_E_INVALID, "null buffer");
    int rc = use_device(ring);
    if (rc) return rc;
    SearchView v = ring->sv();
    v.dir = ring->d_dir;
    CX_HIP(cxk::route_arc(ring->d_ring_ext, ring->d_ring, ring->n, ring->d_arc_tree, ring->rt_l0,
                          ring->rt_R, ring->pk_ib, v, ring->arc_Lh, ring->arc_plo, ring->arc_M,
                          rank, nullptr, src, reinterpret_cast<const cell128 *>(keys), q,
                          reinterpret_cast<ArcRec *>(out), owner, hops, status, ring->stream));
    return CX_OK;
}

int cx_arc_bucket(const cx_ring *ring, int world, const cx_arc_rec *recs, size_t q,
                  cx_arc_rec *send, uint64_t *counts) {
    CX_CHECK(ring && counts, CX_E_INVALID, "null argument");
    CX_CHECK(world >= 1 && world <= CX_ARC_MAX_RANKS, CX_E_INVALID, "world must be in [1, 64]");
    CX_CHECK(q == 0 || (recs && send), CX_E_INVALID, "null buffer");
    CX_CHECK(q < (1ull << 32), CX_E_INVALID, "too many records for one step");
    CX_CHECK(ring->arc_world == world && ring->d_arc_bounds, CX_E_STATE,
             "arc not built for this world size (cx_arc_build)");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    uint32_t *dcnt = ring->d_scratch, *dcur = ring->d_scratch + CX_ARC_MAX_RANKS;
    CX_HIP(hipMemsetAsync(dcnt, 0, CX_ARC_MAX_RANKS * sizeof(uint32_t), s));
    // count -> device-side cursors -> scatter, one host synchronisation (the
    // counts the caller needs for the exchange)
    CX_HIP(cxk::arc_bucket(reinterpret_cast<const ArcRec *>(recs), q, ring->d_arc_bounds,
                           ring->arc_nb, world, dcnt, dcur, nullptr, s, false));
    CX_HIP(cxk::arc_bucket(reinterpret_cast<const ArcRec *>(recs), q, ring->d_arc_bounds,
                           ring->arc_nb, world, nullptr, dcur, reinterpret_cast<ArcRec *>(send), s,
                           true));
    uint32_t hc[CX_ARC_MAX_RANKS];
    CX_HIP(hipMemcpyAsync(hc, dcnt, world * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    CX_HIP(hipStreamSynchronize(s));
    for (int g = 0; g < world; ++g) counts[g] = hc[g];
    return CX_OK;
}

int cx_arc_send_ahead(const cx_ring *ring, int world, int rank, const uint32_t *src,
                      const cx_u128 *keys, size_t q, cx_arc_rec *send, uint64_t *counts) {
    CX_CHECK(ring && counts, CX_E_INVALID, "null argument");
    CX_CHECK(world >= 1 && world <= CX_ARC_MAX_RANKS, CX_E_INVALID, "world must be in [1, 64]");
    CX_CHECK(rank >= 0 && rank < world, CX_E_INVALID, "rank out of range");
    CX_CHECK(q == 0 || (src && keys && send), CX_E_INVALID, "null buffer");
    CX_CHECK(q < (1ull << ARC_ORIGIN_SHIFT), CX_E_INVALID, "too many lookups for one rank");
    CX_CHECK(ring->arc_world == world && ring->d_arc_bounds, CX_E_STATE,
             "arc not built for this world size (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    uint32_t *dcnt = ring->d_scratch, *dcur = ring->d_scratch + CX_ARC_MAX_RANKS;
    const cell128 *k = reinterpret_cast<const cell128 *>(keys);
    CX_HIP(hipMemsetAsync(dcnt, 0, CX_ARC_MAX_RANKS * sizeof(uint32_t), s));
    CX_HIP(cxk::arc_bucket_seed(src, k, rank, q, ring->d_arc_bounds, ring->arc_nb, world, dcnt,
                                dcur, nullptr, s, false));
    CX_HIP(cxk::arc_bucket_seed(src, k, rank, q, ring->d_arc_bounds, ring->arc_nb, world,
                                nullptr, dcur, reinterpret_cast<ArcRec *>(send), s, true));
    uint32_t hc[CX_ARC_MAX_RANKS];
    CX_HIP(hipMemcpyAsync(hc, dcnt, world * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    CX_HIP(hipStreamSynchronize(s));
    for (int g = 0; g < world; ++g) counts[g] = hc[g];
    return CX_OK;
}

int cx_arc_partition(const cx_ring *ring, int world, const uint32_t *src, const cx_u128 *keys,
                     size_t q, cx_u128 *send_keys, uint32_t *send_src, uint32_t *perm,
                     uint64_t *counts) {
    CX_CHECK(ring && counts, CX_E_INVALID, "null argument");
    CX_CHECK(world >= 1 && world <= CX_ARC_MAX_RANKS, CX_E_INVALID, "world must be in [1, 64]");
    CX_CHECK(q == 0 || (src && keys && send_keys && send_src && perm), CX_E_INVALID,
             "null buffer");
    CX_CHECK(q < (1ull << 32), CX_E_INVALID, "too many lookups for one rank");
    CX_CHECK(ring->arc_world == world && ring->d_arc_bounds, CX_E_STATE,
             "arc not built for this world size (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    uint32_t *dcnt = ring->d_scratch, *dcur = ring->d_scratch + CX_ARC_MAX_RANKS;
    CX_HIP(hipMemsetAsync(dcnt, 0, CX_ARC_MAX_RANKS * sizeof(uint32_t), s));
    CX_HIP(cxk::arc_partition(src, reinterpret_cast<const cell128 *>(keys), q, ring->d_arc_bounds,
                              ring->arc_nb, world, dcnt, dcur,
                              reinterpret_cast<cell128 *>(send_keys), send_src, perm, s));
    uint32_t hc[CX_ARC_MAX_RANKS];
    CX_HIP(hipMemcpyAsync(hc, dcnt, world * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    CX_HIP(hipStreamSynchronize(s));
    for (int g = 0; g < world; ++g) counts[g] = hc[g];
    return CX_OK;
}

int cx_arc_partition_regions(const cx_ring *ring, int world, const uint32_t *src,
                             const cx_u128 *keys, size_t q, uint64_t cap, cx_u128 *send_keys,
                             uint32_t *send_src, uint64_t *send_hint, uint32_t *perm,
                             uint64_t *counts) {
    CX_CHECK(ring && counts, CX_E_INVALID, "null argument");
    CX_CHECK(world >= 1 && world <= CX_ARC_MAX_RANKS, CX_E_INVALID, "world must be in [1, 64]");
    CX_CHECK(q == 0 || (src && keys && send_keys && send_src && perm), CX_E_INVALID,
             "null buffer");
    CX_CHECK(cap >= 1 && (uint64_t)world * cap < (1ull << 32) && q < (1ull << 32), CX_E_INVALID,
             "cap must be >= 1 with world * cap < 2^32");
    CX_CHECK(ring->arc_world == world && ring->d_arc_bounds, CX_E_STATE,
             "arc not built for this world size (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    CX_CHECK(!send_hint || ring->d_ring_ext, CX_E_STATE, "arc not built (cx_arc_build)");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    uint32_t *dcur = ring->d_scratch + CX_ARC_MAX_RANKS, *dovf = ring->d_scratch + 2 * CX_ARC_MAX_RANKS;
    uint32_t hc[CX_ARC_MAX_RANKS + 1];
    for (int g = 0; g < world; ++g) hc[g] = (uint32_t)(g * cap);
    hc[world] = 0;
    CX_HIP(hipMemcpyAsync(dcur, hc, world * sizeof(uint32_t), hipMemcpyHostToDevice, s));
    CX_HIP(hipMemsetAsync(dovf, 0, sizeof(uint32_t), s));
    CX_HIP(cxk::arc_partition_regions(src, reinterpret_cast<const cell128 *>(keys), q,
                                      ring->d_arc_bounds, ring->arc_nb, world, (uint32_t)cap,
                                      dcur, dovf, reinterpret_cast<cell128 *>(send_keys),
                                      send_src, perm, send_hint, ring->d_ring_ext, ring->n,
                                      ring->pk_ib, s));
    uint32_t ovf = 0;
    CX_HIP(hipMemcpyAsync(hc, dcur, world * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    CX_HIP(hipMemcpyAsync(&ovf, dovf, sizeof(ovf), hipMemcpyDeviceToHost, s));
    CX_HIP(hipStreamSynchronize(s));
    for (int g = 0; g < world; ++g) counts[g] = hc[g] - (uint64_t)g * cap;
    CX_CHECK(!ovf, CX_E_STATE, "arc partition: a destination's lookups exceed its region (cap)");
    return CX_OK;
}

int cx_arc_partition_regions_async(const cx_ring *ring, int world, const uint32_t *src,
                                   const cx_u128 *keys, size_t q, uint64_t cap,
                                   cx_u128 *send_keys, uint32_t *send_src, uint64_t *send_hint,
                                   uint32_t *perm, int64_t *counts_dev) {
    CX_CHECK(ring && counts_dev, CX_E_INVALID, "null argument");
    CX_CHECK(world >= 1 && world <= CX_ARC_MAX_RANKS, CX_E_INVALID, "world must be in [1, 64]");
    CX_CHECK(q == 0 || (src && keys && send_keys && send_src && perm), CX_E_INVALID,
             "null buffer");
    CX_CHECK(cap >= 1 && (uint64_t)world * cap < (1ull << 32) && q < (1ull << 32), CX_E_INVALID,
             "cap must be >= 1 with world * cap < 2^32");
    CX_CHECK(ring->arc_world == world && ring->d_arc_bounds, CX_E_STATE,
             "arc not built for this world size (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    CX_CHECK(!send_hint || ring->d_ring_ext, CX_E_STATE, "arc not built (cx_arc_build)");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    uint32_t *dcur = ring->d_scratch + CX_ARC_MAX_RANKS, *dovf = ring->d_scratch + 2 * CX_ARC_MAX_RANKS;
    CX_HIP(cxk::arc_cursor_init(dcur, dovf, world, (uint32_t)cap, s));
    CX_HIP(cxk::arc_partition_regions(src, reinterpret_cast<const cell128 *>(keys), q,
                                      ring->d_arc_bounds, ring->arc_nb, world, (uint32_t)cap,
                                      dcur, dovf, reinterpret_cast<cell128 *>(send_keys),
                                      send_src, perm, send_hint, ring->d_ring_ext, ring->n,
                                      ring->pk_ib, s));
    CX_HIP(cxk::arc_counts_out(dcur, dovf, world, (uint32_t)cap, counts_dev, s));
    return CX_OK;
}

int cx_arc_count_async(const cx_ring *ring, int world, const cx_u128 *keys, size_t q,
                       int64_t *counts_dev, int me, uint32_t *own_idx, uint32_t *own_ws) {
    CX_CHECK(ring && counts_dev, CX_E_INVALID, "null argument");
    CX_CHECK(!own_idx || (own_ws && me >= 0 && me < world), CX_E_INVALID,
             "own_idx needs own_ws and 0 <= me < world");
    CX_CHECK(world >= 1 && world <= CX_ARC_MAX_RANKS, CX_E_INVALID, "world must be in [1, 64]");
    CX_CHECK(q == 0 || keys, CX_E_INVALID, "null buffer");
    CX_CHECK(q < (1ull << 32), CX_E_INVALID, "too many lookups for one rank");
    CX_CHECK(ring->arc_world == world && ring->d_arc_bounds, CX_E_STATE,
             "arc not built for this world size (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    int rc = use_device(ring);
    if (rc) return rc;
    CX_HIP(cxk::arc_count_keys(reinterpret_cast<const cell128 *>(keys), q, ring->d_arc_bounds,
                               ring->arc_nb, world, counts_dev, me, own_idx, own_ws,
                               ring->stream));
    return CX_OK;
}

int cx_arc_scatter_async(const cx_ring *ring, int world, const uint32_t *src,
                         const cx_u128 *keys, size_t q, const int64_t *counts_dev,
                         uint32_t *cursor_dev, cx_u128 *send_keys, uint32_t *send_src,
                         uint64_t *send_hint, uint32_t *perm, int skip_rank) {
    CX_CHECK(ring && counts_dev && cursor_dev, CX_E_INVALID, "null argument");
    CX_CHECK(skip_rank >= -1 && skip_rank < world, CX_E_INVALID, "skip_rank out of range");
    CX_CHECK(world >= 1 && world <= CX_ARC_MAX_RANKS, CX_E_INVALID, "world must be in [1, 64]");
    CX_CHECK(q == 0 || (src && keys && send_keys && send_src && perm), CX_E_INVALID,
             "null buffer");
    CX_CHECK(q < (1ull << 32), CX_E_INVALID, "too many lookups for one rank");
    CX_CHECK(ring->arc_world == world && ring->d_arc_bounds, CX_E_STATE,
             "arc not built for this world size (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    CX_CHECK(!send_hint || ring->d_ring_ext, CX_E_STATE, "arc not built (cx_arc_build)");
    int rc = use_device(ring);
    if (rc) return rc;
    CX_HIP(cxk::arc_scatter_exact(src, reinterpret_cast<const cell128 *>(keys), q,
                                  ring->d_arc_bounds, ring->arc_nb, world, counts_dev, cursor_dev,
                                  reinterpret_cast<cell128 *>(send_keys), send_src, perm,
                                  send_hint, ring->d_ring_ext, ring->n, ring->pk_ib, skip_rank,
                                  ring->stream));
    return CX_OK;
}

int cx_arc_route_local(const cx_ring *ring, const uint32_t *src, const cx_u128 *keys,
                       const uint32_t *idx, size_t q, uint32_t *owner, uint8_t *hops,
                       uint8_t *status) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(ring->arc_world > 0 && ring->d_arc_tree, CX_E_STATE, "arc not built (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    CX_CHECK(q == 0 || (src && keys && idx && owner && hops), CX_E_INVALID, "null buffer");
    CX_CHECK(q < (1ull << 32), CX_E_INVALID, "too many lookups for one rank");
    int rc = use_device(ring);
    if (rc) return rc;
    SearchView v = ring->sv();
    v.dir = ring->d_dir;
    CX_HIP(cxk::route_walk_arc_local(ring->d_ring_ext, ring->d_ring, ring->n, ring->d_arc_tree,
                                     ring->rt_l0, ring->pk_ib, v, ring->arc_Lh, ring->arc_plo,
                                     ring->arc_M, src, reinterpret_cast<const cell128 *>(keys),
                                     idx, q, owner, hops, status, ring->stream));
    return CX_OK;
}

int cx_arc_route_hinted(const cx_ring *ring, const uint32_t *src, const cx_u128 *keys,
                        const uint64_t *hint, size_t q, uint64_t *res) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(ring->arc_world > 0 && ring->d_arc_tree, CX_E_STATE, "arc not built (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    CX_CHECK(q == 0 || (src && keys && res && hint), CX_E_INVALID, "null buffer");
    int rc = use_device(ring);
    if (rc) return rc;
    SearchView v = ring->sv();
    v.dir = ring->d_dir;
    CX_HIP(cxk::route_walk_arc(ring->d_ring_ext, ring->d_ring, ring->n, ring->d_arc_tree,
                               ring->rt_l0, ring->pk_ib, v, ring->arc_Lh, ring->arc_plo,
                               ring->arc_M, src, reinterpret_cast<const cell128 *>(keys), q, hint,
                               res, ring->stream));
    return CX_OK;
}

int cx_arc_route(const cx_ring *ring, const uint32_t *src, const cx_u128 *keys, size_t q,
                 uint64_t *res) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(ring->arc_world > 0 && ring->d_arc_tree, CX_E_STATE, "arc not built (cx_arc_build)");
    CX_CHECK(!ring->edited(), CX_E_STATE, "state uploaded after cx_arc_build: use cx_route");
    CX_CHECK(q == 0 || (src && keys && res), CX_E_INVALID, "null buffer");
    int rc = use_device(ring);
    if (rc) return rc;
    SearchView v = ring->sv();
    v.dir = ring->d_dir;  // exact below-table fingers by directory search
    CX_HIP(cxk::route_walk_arc(ring->d_ring_ext, ring->d_ring, ring->n, ring->d_arc_tree,
                               ring->rt_l0, ring->pk_ib, v, ring->arc_Lh, ring->arc_plo,
                               ring->arc_M, src, reinterpret_cast<const cell128 *>(keys), q,
                               nullptr, res, ring->stream));
    return CX_OK;
}

int cx_arc_deliver(const cx_ring *ring, const uint64_t *res, const uint32_t *perm, size_t q,
                   uint32_t *owner, uint8_t *hops, uint8_t *status) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(q == 0 || (res && owner && hops), CX_E_INVALID, "null buffer");
    int rc = use_device(ring);
    if (rc) return rc;
    CX_HIP(cxk::arc_deliver(res, perm, q, owner, hops, status, ring->stream));
    return CX_OK;
}

// ---- internal (not part of chordx.h): allocation-path counters since the
// process started (bench.py reports their change per membership epoch):
// out[8] = {fresh hipMalloc bytes, fresh allocations, bytes reused from the
// pool, pooled allocations, pool blocks trimmed, bytes trimmed, allocations
// retried after a trim, allocations that failed}.
int cxi_pool_stats(uint64_t *out) {
    CX_CHECK(out != nullptr, CX_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(g_pool_mu);
    const uint64_t v[8] = {g_stats.fresh_bytes, g_stats.fresh_allocs, g_stats.reused_bytes,
                           g_stats.reused_allocs, g_stats.trims, g_stats.trimmed_bytes,
                           g_stats.retries, g_stats.failures};
    for (int k = 0; k < 8; ++k) out[k] = v[k];
    return CX_OK;
}

// ---- internal: fault injection for tests (bit 0: the route-table build's
// finger-plane allocation fails; bit 1: the default route-table build defers
// the rows past 48 distinct roots per block to overflow launches).
int cxi_set_fault(int mask) {
    g_fault.store(mask);
    cxk::cz2_set_cap(mask & 2 ? 48u : 256u);
    return CX_OK;
}

// ---- internal (not part of chordx.h): error reporting for cx_wire.cpp
int cxi_set_error(int code, const char *msg) { return fail(code, msg ? msg : ""); }

// ---- internal (not part of chordx.h): route-walk switch for parity tests and
// benches.  0 = finger + ring gathers per hop (no table), 4 = lookahead-tree
// table (the automatic choice above 2^24 peers), 5 = pattern-keyed window table
// (k_walk), -1 = automatic (5 up to 2^24 peers, else 4).
int cxi_set_route_variant(cx_ring *ring, int variant) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(variant == -1 || variant == 0 || variant == 4 || variant == 5, CX_E_INVALID,
             "variant must be -1 (auto), 0, 4 or 5");
    ring->route_variant = variant;
    return CX_OK;
}

// Route-table depth A/B: the table covers levels [128 - R, 128) (0 = the
// default).  Only before the ring's first finger build (the table sizes follow R).
int cxi_set_route_depth(cx_ring *ring, int R) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    // the pattern-keyed build needs its lowest plane level (128 - R - 5) >= 64
    CX_CHECK(R == 0 || (R >= 16 && R <= 59), CX_E_INVALID, "R must be 0 or in [16, 59]");
    CX_CHECK(!ring->d_cz && !ring->d_tree && !ring->d_arc_tree,
             CX_E_STATE, "route depth is fixed once a route table exists");
    ring->depth_override = R;
    return CX_OK;
}

// Route variant in effect, variant-5 nodes its format could not represent, and
// the bytes of the route table the variant reads (0 if not built).
int cxi_route_info(const cx_ring *ring, int *variant, uint64_t *cz_escapes,
                   uint64_t *table_bytes) {
    CX_CHECK(ring && variant && cz_escapes && table_bytes, CX_E_INVALID, "null argument");
    const int v = ring->literal() ? -1 : ring->variant();
    const size_t ent = ring->n * (size_t)ring->rt_R;
    *variant = v;
    *cz_escapes = ring->cz_escapes;
    *table_bytes = v == 5 && ring->cz_valid     ? ent * 128
                   : v == 4 && ring->tree_valid ? ent * 64
                                                : 0;
    return CX_OK;
}

// Gather counters of the default route kernel (bench.py's byte model):
// enable = 1 zeroes them and makes later cx_route calls run the counting
// instantiation of the walk; enable = 0 switches back and copies the totals to
// out[4] = {64-B table gathers, exact 16-B ring gathers, exact hops (F + ring
// gather each), lookups}.
int cxi_route_counters(cx_ring *ring, int enable, uint64_t *out) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    int rc = use_device(ring);
    if (rc) return rc;
    hipStream_t s = ring->stream;
    if (!ring->d_stats) CX_HIP(dev_malloc(&ring->d_stats, 4 * sizeof(unsigned long long)));
    if (enable) {
        CX_HIP(hipMemsetAsync(ring->d_stats, 0, 4 * sizeof(unsigned long long), s));
        ring->counting = true;
        return CX_OK;
    }
    ring->counting = false;
    CX_CHECK(out != nullptr, CX_E_INVALID, "null out");
    unsigned long long h[4];
    CX_HIP(hipMemcpyAsync(h, ring->d_stats, sizeof(h), hipMemcpyDeviceToHost, s));
    CX_HIP(hipStreamSynchronize(s));
    for (int k = 0; k < 4; ++k) out[k] = h[k];
    return CX_OK;
}

// Request-rate ceiling measured on this ring's own route table (the
// pattern-keyed window table, else the finger table): dependent random 64-B
// gathers by quads of lanes, entries/s.  Read only.
int cxi_gather_probe(const cx_ring *ring, int lanes, int hops, double *rate) {
    CX_CHECK(ring && rate, CX_E_INVALID, "null argument");
    int rc = use_device(ring);
    if (rc) return rc;
    const void *t = nullptr;
    size_t bytes = 0;
    if (ring->cz_valid) {
        t = ring->d_cz;
        bytes = ring->n * (size_t)ring->rt_R * 128;
    } else if (ring->d_fingers) {
        t = ring->d_fingers;
        bytes = ring->n * (size_t)CX_FINGERS * sizeof(uint32_t);
    }
    CX_CHECK(t != nullptr, CX_E_STATE, "no route table built");
    CX_HIP(cxk::gather_probe(t, bytes, lanes, hops, rate, ring->stream));
    return CX_OK;
}

// The same probe over the first span_bytes of the route table (footprint A/B:
// the request ceiling of a smaller table, measured on real table memory).
int cxi_gather_probe_span(const cx_ring *ring, int lanes, int hops, uint64_t span_bytes,
                          double *rate) {
    CX_CHECK(ring && rate, CX_E_INVALID, "null argument");
    CX_CHECK(ring->cz_valid, CX_E_STATE, "no pattern-keyed table built");
    int rc = use_device(ring);
    if (rc) return rc;
    size_t bytes = ring->n * (size_t)ring->rt_R * 128;
    if (span_bytes && span_bytes < bytes) bytes = span_bytes & ~(uint64_t)63;
    CX_CHECK(bytes >= 64 * 1024, CX_E_INVALID, "span too small");
    CX_HIP(cxk::gather_probe(ring->d_cz, bytes, lanes, hops, rate, ring->stream));
    return CX_OK;
}

// Ring-sort timing (A/B, bench setup_s.ring_sort_roofline): the (ID, index)
// sort of cx_ring_create over n device IDs, on a private stream with HIP
// events around the sort alone.  variant 0 = radix_sort (MSD buckets, the
// default), 1 = the 16-pass LSD sort.  *ms = the sort's time; *sorted = 1 if
// the output is ascending by (key, tag) (checked on the device afterwards:
// the MSD path's (key, tag) order).
int cxi_sort_time(const cx_u128 *ids, size_t n, int device, int variant, double *ms, int *sorted) {
    CX_CHECK(ids && ms && sorted && n >= 1 && n < ((size_t)1 << 31), CX_E_INVALID, "bad argument");
    CX_CHECK(variant == 0 || variant == 1, CX_E_INVALID, "variant must be 0 or 1");
    CX_HIP(hipSetDevice(device));
    hipStream_t s = nullptr;
    CX_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = [&]() -> int {
        DBuf k0, k1, t0, t1, ws, flag;
        CX_HIP(k0.alloc_pooled(n * sizeof(cell128), s));
        CX_HIP(k1.alloc_pooled(n * sizeof(cell128), s));
        CX_HIP(t0.alloc_pooled(n * sizeof(uint32_t), s));
        CX_HIP(t1.alloc_pooled(n * sizeof(uint32_t), s));
        CX_HIP(ws.alloc_pooled(cxk::sort_workspace_words(n) * sizeof(uint32_t), s));
        CX_HIP(flag.alloc(sizeof(uint32_t)));
        CX_HIP(hipMemcpyAsync(k0.p, ids, n * sizeof(cell128), hipMemcpyDeviceToDevice, s));
        CX_HIP(cxk::iota(t0.as<uint32_t>(), n, 0, s));
        CX_HIP(hipEventCreate(&e0));
        CX_HIP(hipEventCreate(&e1));
        CX_HIP(hipEventRecord(e0, s));
        if (variant == 0)
            CX_HIP(cxk::radix_sort(k0.as<cell128>(), t0.as<uint32_t>(), k1.as<cell128>(),
                                   t1.as<uint32_t>(), n, ws.as<uint32_t>(), s));
        else
            CX_HIP(cxk::radix_sort_lsd(k0.as<cell128>(), t0.as<uint32_t>(), k1.as<cell128>(),
                                       t1.as<uint32_t>(), n, ws.as<uint32_t>(), s));
        CX_HIP(hipEventRecord(e1, s));
        CX_HIP(cxk::check_sorted(k0.as<cell128>(), t0.as<uint32_t>(), n, flag.as<uint32_t>(), s));
        uint32_t bad = 1;
        CX_HIP(hipMemcpyAsync(&bad, flag.p, sizeof(bad), hipMemcpyDeviceToHost, s));
        CX_HIP(hipStreamSynchronize(s));
        float t = 0.f;
        CX_HIP(hipEventElapsedTime(&t, e0, e1));
        *ms = t;
        *sorted = bad == 0;
        return CX_OK;
    }();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    return rc;
}

// Hash of the route table the ring built (the pattern-keyed window table, or
// the arc planes when arc mode is on): A/B identity of two builds.
int cxi_route_table_hash(const cx_ring *ring, int arc, uint64_t *out) {
    CX_CHECK(ring && out, CX_E_INVALID, "null argument");
    int rc = use_device(ring);
    if (rc) return rc;
    const void *t = nullptr;
    size_t bytes = 0;
    if (arc) {
        CX_CHECK(ring->arc_world > 0, CX_E_STATE, "arc mode is off");
        t = ring->d_arc_tree;
        bytes = ((size_t)((int)CX_FINGERS - ring->arc_Lh) * 2 * ring->n +
                 (size_t)(ring->arc_Lh - ring->rt_l0) * 2 * ring->arc_M) * 64;
    } else {
        CX_CHECK(ring->cz_valid, CX_E_STATE, "no pattern-keyed table built");
        t = ring->d_cz;
        bytes = ring->n * (size_t)ring->rt_R * 128;
    }
    hipStream_t s = ring->stream;
    DBuf acc;
    CX_HIP(acc.alloc(sizeof(unsigned long long)));
    CX_HIP(cxk::table_hash(t, bytes, acc.as<unsigned long long>(), s));
    unsigned long long h = 0;
    CX_HIP(hipMemcpyAsync(&h, acc.p, sizeof(h), hipMemcpyDeviceToHost, s));
    CX_HIP(hipStreamSynchronize(s));
    *out = h;
    return CX_OK;
}

// Route-table build input (parity tests of the build's fallbacks): 0 = level +
// two-hop planes, root-centric windows in blocks sized by distinct roots
// (k_cz_build_roots2, default), 1 = row-major finger table (the fallback
// without HBM for the planes), 2 = level planes only, 3 = level + two-hop
// planes, one lane per entry (k_cz_build; also the build of rings with a gap
// too wide for the 32-bit ID slices).  All give the same table.  Takes effect
// at the next finger build.
int cxi_set_table_build(cx_ring *ring, int variant) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(variant >= 0 && variant <= 3, CX_E_INVALID, "variant must be 0 .. 3");
    ring->table_build = variant;
    return CX_OK;
}

// f2 finger repair (A/B): 1 = a churned ring's finger planes are remapped from
// its parent's, 0 = searched from scratch by the streaming build (default:
// faster).  Inherited by churned rings; a ring keeps its planes for its
// children only while it is on.  Takes effect at the next finger build.
int cxi_set_fingers_repair(cx_ring *ring, int on) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    ring->fingers_repair = on ? 1 : 0;
    return CX_OK;
}

// Last finger build: *repaired = 1 when its planes were remapped from the
// parent ring, *searched = fingers that needed an exact search in that repair.
int cxi_fingers_repair_info(const cx_ring *ring, int *repaired, uint64_t *searched) {
    CX_CHECK(ring && repaired && searched, CX_E_INVALID, "null argument");
    *repaired = ring->planes_repaired;
    *searched = ring->repair_searched;
    return CX_OK;
}

// Releases every pooled table (all devices).
int cx_pool_trim(void) {
    {
        std::lock_guard<std::mutex> g(g_pool_mu);
        pool_trim_locked(-1);
    }
    stage_trim();  // the idle staging blocks of host-memory calls too
    return CX_OK;
}
int cxi_pool_trim(void) { return cx_pool_trim(); }

int cx_pool_info(uint64_t *blocks, uint64_t *bytes) {
    CX_CHECK(blocks && bytes, CX_E_INVALID, "null argument");
    std::lock_guard<std::mutex> g(g_pool_mu);
    *blocks = g_pool.size();
    *bytes = g_pool_bytes;
    return CX_OK;
}

// 0 = full re-sort of survivors + joins, 1 = merge of the sorted joins (default).
int cxi_set_churn_variant(cx_ring *ring, int variant) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(variant == 0 || variant == 1, CX_E_INVALID, "variant must be 0 or 1");
    ring->churn_variant = variant;
    return CX_OK;
}

// 0 = Eytzinger search with LDS-staged top levels, 1 = bucket directory (default;
// large batches on rings that fit LDS: the LDS slice table), 2 = wave-cooperative
// 16-ary tree, 3 = wave-cooperative Eytzinger (16 lanes a query, four levels per
// ballot), 4 = LDS slice table whenever the ring fits, 5 = directory only, for
// cx_successor / cx_predecessor (variants 2 to 5: the other searches keep the
// directory).
int cxi_set_search_variant(cx_ring *ring, int variant) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(variant >= 0 && variant <= 5, CX_E_INVALID, "variant must be 0 to 5");
    if (variant == 0 || variant == 3) {
        int rc = use_device(ring);
        if (rc) return rc;
        if ((rc = ensure_eyt(ring, ring->stream))) return rc;
    }
    ring->search_variant = variant;
    return CX_OK;
}

// Misplaced scan after cx_churn: 0 = two directory searches + the old_to_new
// window per key, 1 = churn directory (default; one 32-B gather per key,
// built on first use from the rings and cx_churn's mapping).  Set on the NEW
// ring (rings from cx_churn inherit the parent's setting).
int cxi_set_misplaced_variant(cx_ring *ring, int variant) {
    CX_CHECK(ring != nullptr, CX_E_INVALID, "null ring");
    CX_CHECK(variant == 0 || variant == 1, CX_E_INVALID, "variant must be 0 or 1");
    ring->misplaced_variant = variant;
    return CX_OK;
}

}  // extern "C"
