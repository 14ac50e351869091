// runtime.hpp -- internal to libkraken_hip: device contexts, the stream-ordered
// scratch cache, the CRC work builder and the SHA job runner shared by the C ABI
// (runtime.cpp) and the submission engine (engine.cpp).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/kraken_hip_internal.h"
#include "crc_math.hpp"
#include "kernels.hpp"
#include "knobs.hpp"

namespace krk {

// ------------------------------------------------------------------ errors
extern thread_local std::string t_err;
extern thread_local int t_dev;

void set_error(int code, const char* fmt, ...);

#define KRK_HIP(expr)                                                                 \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess) {                                                       \
            set_error(KRK_EHIP, "%s: %s", #expr, hipGetErrorString(e_));              \
            return KRK_EHIP;                                                          \
        }                                                                             \
    } while (0)

#define KRK_CHECK(cond, code, ...)        \
    do {                                  \
        if (!(cond)) {                    \
            set_error(code, __VA_ARGS__); \
            return code;                  \
        }                                 \
    } while (0)

// ------------------------------------------------------------------ timing
enum Kern { K_CRC, K_SHA, K_HRW, K_FILTER, K_GATHER, K_SYNTH, K_HOSTG, K_N };
inline const char* kKernNames[K_N] = {"crc32_pieces", "sha256_multi", "hrw_order",   "ring_filter",
                                      "hrw_gather",   "synth_fill",   "host_gather"};
inline std::atomic<bool> g_timing{false};
struct Pending {
    hipEvent_t a, b;
    int k, dev, plan;
    uint64_t units;
};
struct TimelineRec {
    int k, dev, plan;
    uint64_t units;
    double t0, t1;  // ms after the device's first timed launch since the last reset
};
constexpr size_t kTimelineCap = 1u << 20;
constexpr int kMaxDevs = 64;
inline std::mutex g_tmu;
inline std::vector<Pending> g_pending;
inline std::vector<TimelineRec> g_timeline;
inline hipEvent_t g_origin[kMaxDevs];  // per device: the first timed launch's start event
inline double g_ms[K_N];
inline uint64_t g_cnt[K_N];

template <class F>
inline hipError_t timed(int k, hipStream_t s, F&& f) {
    if (!g_timing.load(std::memory_order_relaxed)) return f();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    t_launch_plan = 0;
    t_launch_units = 0;
    hipError_t e = f();
    hipEventRecord(b, s);
    std::lock_guard<std::mutex> g(g_tmu);
    g_pending.push_back({a, b, k, t_dev, t_launch_plan, t_launch_units});
    return e;
}

inline void drain_timing() {
    std::lock_guard<std::mutex> g(g_tmu);
    int cur = 0;
    hipGetDevice(&cur);
    for (auto& p : g_pending) {
        hipSetDevice(p.dev);
        hipEventSynchronize(p.b);
        float ms = 0;
        bool keep_a = false;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            g_ms[p.k] += ms;
            g_cnt[p.k] += 1;
            if (p.dev >= 0 && p.dev < kMaxDevs) {
                if (!g_origin[p.dev]) {
                    g_origin[p.dev] = p.a;
                    keep_a = true;
                }
                float t0 = 0, t1 = 0;
                if (g_timeline.size() < kTimelineCap &&
                    hipEventElapsedTime(&t0, g_origin[p.dev], p.a) == hipSuccess &&
                    hipEventElapsedTime(&t1, g_origin[p.dev], p.b) == hipSuccess)
                    g_timeline.push_back({p.k, p.dev, p.plan, p.units, (double)t0, (double)t1});
            }
        }
        if (!keep_a) hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    g_pending.clear();
    hipSetDevice(cur);
}

// ------------------------------------------------------------------ NUMA
// NUMA node of device `id` (its PCI function's sysfs entry); -1 if unknown.
inline int device_numa_node(int id) {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, id) != hipSuccess) return -1;
    for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
    std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return -1;
    int node = -1;
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
    return node;
}

// The CPUs of NUMA node `node` this process may run on (empty if none / unknown).
inline cpu_set_t numa_node_cpus(int node) {
    cpu_set_t s, allowed;
    CPU_ZERO(&s);
    if (node < 0 || sched_getaffinity(0, sizeof allowed, &allowed) != 0) return s;
    std::string path = "/sys/devices/system/node/node" + std::to_string(node) + "/cpulist";
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return s;
    char buf[4096] = {0};
    if (!fgets(buf, sizeof buf, f)) buf[0] = 0;
    fclose(f);
    for (char* p = strtok(buf, ",\n"); p; p = strtok(nullptr, ",\n")) {
        int a = 0, b = 0;
        const int k = sscanf(p, "%d-%d", &a, &b);
        if (k < 1) continue;
        if (k == 1) b = a;
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &allowed)) CPU_SET(c, &s);
    }
    return s;
}

// f() on the calling thread bound to the CPUs of NUMA node `node` (memory it allocates or
// first touches comes from that node under the default local policy), then the thread's
// affinity restored.  node < 0, or no allowed CPU there: f() as is.
template <class F>
inline void on_numa_node(int node, F&& f) {
    cpu_set_t want = numa_node_cpus(node), old;
    if (node < 0 || CPU_COUNT(&want) == 0 || pthread_getaffinity_np(pthread_self(), sizeof old, &old) != 0 ||
        pthread_setaffinity_np(pthread_self(), sizeof want, &want) != 0) {
        f();
        return;
    }
    f();
    pthread_setaffinity_np(pthread_self(), sizeof old, &old);
}

// ------------------------------------------------------------------ device
struct PinnedSlot {
    void* p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    hipStream_t s_last = nullptr;  // the stream the last copy (and ev) went on
    bool busy = false;
};
// upload()'s pinned slots, one ring per stream (at most kMaxUploadRings; more streams
// share rings).  A slot's bytes are rewritten only after hipEventSynchronize on its last
// copy, and a ring waits only for its own stream's copies, so a stream held behind a long
// kernel (a C3 window's pack copy waits for the window before it, ~0.6 s) never holds
// another stream's uploads -- the shared pool before it either waited under the device
// lock or skipped busy slots (hipEventQuery) and grew without bound.
constexpr int kRingSlots = 8;
constexpr size_t kMaxUploadRings = 32;
struct UploadRing {
    std::mutex mu;
    PinnedSlot slot[kRingSlots];
    unsigned next = 0;
};

// Stream-ordered device scratch.  Blocks are power-of-two sized and stay with the
// device context; a released block carries an event recorded on the releasing
// stream and its next user's stream waits on that event, so reuse is ordered on
// the device with no host stall and no allocator work per call.  A block is taken
// from another stream only once its event has completed: waiting on a block still
// held behind another stream's long kernel would serialize independent streams (the
// CRC launch of krk_metainfo_digest_dev queued behind the whole SHA-256 kernel when
// both took blocks of one size), so a fresh block is allocated instead.
struct DevCache {
    struct Blk {
        void* p = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
        hipStream_t s = nullptr;  // the stream that released it
        bool pending = false;
    };
    std::mutex mu;
    std::unordered_map<void*, Blk> live;
    std::unordered_multimap<size_t, Blk> idle;

    hipError_t alloc(void** out, size_t n, hipStream_t s) {
        size_t cap = 256;
        while (cap < n) cap <<= 1;
        Blk b;
        {
            std::lock_guard<std::mutex> g(mu);
            auto r = idle.equal_range(cap);
            auto pick = idle.end();
            for (auto it = r.first; it != r.second; ++it) {
                const Blk& c = it->second;
                if (!c.pending || c.s == s) {  // free, or ordered by this stream already
                    pick = it;
                    break;
                }
                if (pick == idle.end() && hipEventQuery(c.ev) == hipSuccess) pick = it;
            }
            if (pick != idle.end()) {
                b = pick->second;
                idle.erase(pick);
            }
        }
        hipError_t e = hipSuccess;
        if (b.p) {
            if (b.pending) e = hipStreamWaitEvent(s, b.ev, 0);  // free when s released it
        } else {
            e = hipMalloc(&b.p, cap);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&b.ev, hipEventDisableTiming);
            b.cap = cap;
        }
        if (e != hipSuccess) return e;
        std::lock_guard<std::mutex> g(mu);
        live[b.p] = b;
        *out = b.p;
        return hipSuccess;
    }
    void release(void* p, hipStream_t s) {
        if (!p) return;
        std::lock_guard<std::mutex> g(mu);
        auto it = live.find(p);
        if (it == live.end()) return;
        Blk b = it->second;
        live.erase(it);
        b.s = s;
        b.pending = hipEventRecord(b.ev, s) == hipSuccess;
        if (!b.pending) hipStreamSynchronize(s);
        idle.emplace(b.cap, b);
    }
};

struct Pipeline;
struct Engine;
struct OffloadPool;

struct OwnerTables;  // runtime.cpp
struct Device {
    // Submission engine (engine.cpp): the batching queues of the streaming
    // Digester / piece-stream / crc32.Update calls, created on first use.
    Engine* engine = nullptr;
    std::mutex engine_mu;
    DevCache cache;
    // Staging windows of the host paths, kept across calls (pinning 2 x 256 MiB
    // costs ~0.2 s, a third of a 16 GB end-to-end batch).  Leaked at exit like the
    // other device resources: freeing pinned memory during static destruction can
    // race the HIP runtime's own teardown.
    Pipeline* staging = nullptr;
    std::mutex staging_mu;
    // Host threads + pinned double buffers of the SHA-256 host offload (offload.cpp).
    OffloadPool* offload = nullptr;
    std::mutex offload_mu;
    // The 65,536 ShardID keys (2 bytes each) of the Locations shard table, uploaded
    // once: constant input of every krk_ring_locations_dev call.
    uint8_t* shard_kb = nullptr;
    uint64_t* shard_koff = nullptr;
    uint8_t* shard_bad = nullptr;
    std::once_flag shard_once;
    int shard_rc = 0;
    // ring.Locations owner tables by membership (runtime.cpp OwnerTables): the reference's
    // Ring rebuilds its hrw only on Refresh (lib/hashring/ring.go:141-165).
    OwnerTables* owners = nullptr;
    std::mutex owners_mu;
    int id = 0;
    int cus = 0;
    hipStream_t s_main = nullptr, s_a = nullptr, s_b = nullptr;
    uint32_t* d_tabs = nullptr;
    int crc_variant = 0;
    std::mutex mu;  // the ring table and the retired list
    std::unordered_map<hipStream_t, UploadRing*> ring_of;
    std::vector<std::unique_ptr<UploadRing>> rings;
    std::vector<void*> retired_pinned;  // grown-out upload buffers (freed at krk_shutdown)
};

template <class T>
inline hipError_t scratch_alloc(Device* D, T** p, size_t n, hipStream_t s) {
    void* v = nullptr;
    hipError_t e = D->cache.alloc(&v, n, s);
    *p = static_cast<T*>(v);
    return e;
}
inline void scratch_free(Device* D, void* p, hipStream_t s) { D->cache.release(p, s); }

inline std::mutex g_dmu;
inline std::vector<std::unique_ptr<Device>> g_devs;
inline X8Pow g_x8;
inline std::once_flag g_x8_once;

inline const X8Pow& x8() {
    std::call_once(g_x8_once, [] { g_x8 = make_x8pow(); });
    return g_x8;
}

inline int init_device(Device& D, int id) {
    D.id = id;
    KRK_HIP(hipSetDevice(id));
    hipDeviceProp_t prop;
    KRK_HIP(hipGetDeviceProperties(&prop, id));
    KRK_CHECK(strncmp(prop.gcnArchName, "gfx950", 6) == 0, KRK_ENODEV,
              "device %d is %s, this build targets gfx950 (MI355X)", id, prop.gcnArchName);
    D.cus = prop.multiProcessorCount;
    KRK_HIP(hipStreamCreateWithFlags(&D.s_main, hipStreamNonBlocking));
    KRK_HIP(hipStreamCreateWithFlags(&D.s_a, hipStreamNonBlocking));
    KRK_HIP(hipStreamCreateWithFlags(&D.s_b, hipStreamNonBlocking));
    std::vector<uint32_t> tabs(kTabWords);
    make_slice_tables(tabs.data() + kTabT);
    const X8Pow& xp = x8();
    make_shift_tables(tabs.data() + kTabG, x8n(kGap, xp.v));
    for (int l = 0; l < 64; ++l) tabs[kTabLaneMul + l] = x8n(uint64_t(63 - l) * kSeg, xp.v);
    for (int k = 0; k < 64; ++k) tabs[kTabX8Pow + k] = xp.v[k];
    make_shift_tables(tabs.data() + kTabGC, x8n(kGapC, xp.v));
    for (int k = 0; k < 4; ++k)
        for (int l = 0; l < 64; ++l)
            tabs[kTabLaneMulC + k * 64 + l] = x8n(uint64_t(kGapC) - 1024 * k - 16 * l, xp.v);
    KRK_HIP(hipMalloc(&D.d_tabs, kTabWords * 4));
    KRK_HIP(hipMemcpy(D.d_tabs, tabs.data(), kTabWords * 4, hipMemcpyHostToDevice));
    // Launch variant, read once per device context (crc32_pieces.hip: 16 = byte-addressable
    // tables with the work queue, the default; 7 = the same with a static item stride; 8,
    // 14, 15, 17 = measured alternatives; the rest only in the KRK_DIAG build).
    const char* v = KRK_AB_ENV("KRK_CRC_VARIANT");
    const int want = v ? atoi(v) : 16;
    D.crc_variant = crc_variant_valid(want) ? want : 16;
    return KRK_OK;
}

// The context of device `id` (created on first use); also makes it the calling
// thread's current HIP device.
inline Device* device_id(int id, int* rc) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_error(KRK_ENODEV, "no HIP device visible");
        *rc = KRK_ENODEV;
        return nullptr;
    }
    if (id < 0 || id >= n) {
        set_error(KRK_ENODEV, "device %d out of range (%d visible)", id, n);
        *rc = KRK_ENODEV;
        return nullptr;
    }
    std::lock_guard<std::mutex> g(g_dmu);
    if ((int)g_devs.size() < n) g_devs.resize(n);
    if (!g_devs[id]) {
        auto D = std::make_unique<Device>();
        int r = init_device(*D, id);
        if (r != KRK_OK) {
            *rc = r;
            return nullptr;
        }
        g_devs[id] = std::move(D);
    }
    if (hipSetDevice(id) != hipSuccess) {
        set_error(KRK_EHIP, "hipSetDevice(%d) failed", id);
        *rc = KRK_EHIP;
        return nullptr;
    }
    *rc = KRK_OK;
    return g_devs[id].get();
}

// The calling thread's device (krk_set_device).
inline Device* device(int* rc) { return device_id(t_dev, rc); }

#define KRK_DEVICE(D)         \
    int rc_ = KRK_OK;         \
    Device* D = device(&rc_); \
    if (!D) return rc_;

inline hipStream_t pick(Device* D, void* s) { return s ? static_cast<hipStream_t>(s) : D->s_main; }

// Stage `n` host bytes through a pinned slot into a fresh stream-ordered device
// scratch block (released with scratch_free by the caller).
inline int upload(Device* D, const void* src, size_t n, void** d_out, hipStream_t s) {
    *d_out = nullptr;
    if (!n) return KRK_OK;
    KRK_HIP(scratch_alloc(D, d_out, n, s));
    UploadRing* R = nullptr;
    {
        std::lock_guard<std::mutex> g(D->mu);
        auto it = D->ring_of.find(s);
        if (it != D->ring_of.end()) {
            R = it->second;
        } else {
            if (D->rings.size() < kMaxUploadRings) D->rings.push_back(std::make_unique<UploadRing>());
            R = D->rings[D->ring_of.size() % D->rings.size()].get();  // beyond the cap: shared
            D->ring_of.emplace(s, R);
        }
    }
    std::lock_guard<std::mutex> g(R->mu);
    // The ring's next slot, once its last copy has run (this stream's upload kRingSlots
    // calls ago, queued before everything this call is about to queue).
    PinnedSlot& P = R->slot[R->next++ % kRingSlots];
    if (P.busy) {
        KRK_HIP(hipEventSynchronize(P.ev));
        P.busy = false;
    }
    if (!P.ev) KRK_HIP(hipEventCreateWithFlags(&P.ev, hipEventDisableTiming));
    if (P.cap < n) {
        // hipHostFree waits for the whole device (a kernel of another stream included), so
        // a grown slot's old buffer is kept until krk_shutdown: freeing it here held the C3
        // windows' CRC launch back until the window's SHA-256 kernel had ended.
        if (P.p) {
            std::lock_guard<std::mutex> gd(D->mu);
            D->retired_pinned.push_back(P.p);
        }
        P.p = nullptr;  // a failed grow leaves an empty slot, not a dangling one
        P.cap = 0;
        size_t cap = 1 << 16;
        while (cap < n) cap <<= 1;
        KRK_HIP(hipHostMalloc(&P.p, cap, hipHostMallocDefault));
        P.cap = cap;
    }
    memcpy(P.p, src, n);
    KRK_HIP(hipMemcpyAsync(*d_out, P.p, n, hipMemcpyHostToDevice, s));
    KRK_HIP(hipEventRecord(P.ev, s));
    P.s_last = s;
    P.busy = true;
    return KRK_OK;
}

// Before a stream the library has used is destroyed (krk_stream_destroy): its work is
// waited for, and every library event last recorded on it -- upload slots, idle scratch
// blocks -- is replaced by a fresh one.  HIP keeps a reference to the stream in an event
// it recorded; a later hipEventSynchronize / hipStreamWaitEvent on such an event after the
// stream was destroyed failed with "operation not permitted when stream is capturing"
// (the GPU suite once the C3 windows' and the concurrency test's streams came and went).
inline void forget_stream(Device* D, hipStream_t s) {
    if (!s) return;
    hipStreamSynchronize(s);
    std::vector<UploadRing*> rings;
    {
        std::lock_guard<std::mutex> g(D->mu);
        D->ring_of.erase(s);
        for (auto& R : D->rings) rings.push_back(R.get());
    }
    for (UploadRing* R : rings) {
        std::lock_guard<std::mutex> g(R->mu);
        for (PinnedSlot& P : R->slot)
            if (P.s_last == s) {
                if (P.ev) hipEventDestroy(P.ev);
                P.ev = nullptr;  // re-created at the slot's next use
                P.s_last = nullptr;
                P.busy = false;
            }
    }
    std::lock_guard<std::mutex> g(D->cache.mu);
    for (auto& kv : D->cache.idle) {
        DevCache::Blk& b = kv.second;
        if (b.s != s) continue;
        hipEvent_t fresh = nullptr;
        if (hipEventCreateWithFlags(&fresh, hipEventDisableTiming) == hipSuccess) {
            hipEventDestroy(b.ev);
            b.ev = fresh;
        }
        b.pending = false;  // its stream's work is done
        b.s = nullptr;
    }
}

// ------------------------------------------------------------------ CRC items
// The work of one CRC launch: runs of whole pieces (expanded into items on the
// device) plus explicit items for partial pieces and seeded CRCs.
struct CrcBatch {
    std::vector<CrcRun> runs;
    std::vector<CrcItem> items;
    std::vector<uint32_t> consts;
    std::unordered_map<uint64_t, uint32_t> pat;  // piece length -> consts index of its pattern
    uint64_t run_items = 0;
    bool empty() const { return runs.empty() && items.empty(); }
};

// Items for bytes [a, b) of one blob (length L, pieces of P bytes), where blob byte
// `a` lives at device address `base`.  `seed` is the register the IEEE CRC starts
// from (~crc of crc32.Update; ~0 for PieceHash()).
struct ItemBuilder {
    std::unordered_map<uint64_t, uint32_t> cache;

    uint32_t X(uint64_t n) {
        if (n == 0) return kOne;
        auto it = cache.find(n);
        if (it != cache.end()) return it->second;
        const uint32_t v = x8n(n, x8().v);
        cache.emplace(n, v);
        return v;
    }

    void piece(std::vector<CrcItem>& out, uint64_t ptr_of_ps, uint64_t ps, uint64_t pe, uint64_t s,
               uint64_t e, uint32_t out_idx, uint32_t seed) {
        // Items start at multiples of kItemBytes from the piece start (or at s).
        for (uint64_t q = s; q < e;) {
            const uint64_t next = std::min(e, ps + ((q - ps) / kItemBytes + 1) * kItemBytes);
            CrcItem it{};
            it.ptr = ptr_of_ps + (q - ps);
            it.len = (uint32_t)(next - q);
            it.out = out_idx;
            it.mul = X(pe - next);
            it.xr = (q == ps) ? (gf2_mulmod(seed, X(pe - ps)) ^ 0xFFFFFFFFu) : 0u;
            out.push_back(it);
            q = next;
        }
    }

    // consts index of the whole-piece pattern for piece length P (item muls, then xr).
    uint32_t pattern(CrcBatch& B, uint64_t P) {
        auto it = B.pat.find(P);
        if (it != B.pat.end()) return it->second;
        const uint32_t at = (uint32_t)B.consts.size();
        for (uint64_t q = 0; q < P; q += kItemBytes) B.consts.push_back(X(P - std::min(q + kItemBytes, P)));
        B.consts.push_back(gf2_mulmod(0xFFFFFFFFu, X(P)) ^ 0xFFFFFFFFu);
        B.pat.emplace(P, at);
        return at;
    }

    // Whole pieces [f0, f1) of a blob whose piece f0 starts at device address ptr.
    void run(CrcBatch& B, uint64_t ptr, uint64_t f0, uint64_t f1, uint64_t P, uint64_t sums_off) {
        const uint64_t ipp = (P + kItemBytes - 1) / kItemBytes;
        const uint32_t cpat = pattern(B, P);
        for (uint64_t f = f0; f < f1;) {  // a run's item count stays below 2^31
            const uint64_t n = std::min<uint64_t>(f1 - f, std::max<uint64_t>(1, (1ull << 31) / ipp));
            CrcRun r{};
            r.ptr = ptr + (f - f0) * P;
            r.plen = P;
            r.n_pieces = (uint32_t)n;
            r.out = (uint32_t)(sums_off + f);
            r.item_base = (uint32_t)B.run_items;
            r.ipp = (uint32_t)ipp;
            r.cpat = cpat;
            B.runs.push_back(r);
            B.run_items += n * ipp;
            f += n;
        }
    }

    void add(CrcBatch& B, uint64_t base, uint64_t a, uint64_t b, uint64_t L, uint64_t P, uint64_t sums_off,
             uint32_t seed = 0xFFFFFFFFu) {
        if (a >= b) return;
        const uint64_t pa = a / P, pb = (b - 1) / P;  // pieces touched, inclusive
        // Whole pieces [f0, f1): inside [a, b), full length, unseeded -> one run.
        uint64_t f0 = (a + P - 1) / P, f1 = std::min(b, L) / P;
        if (seed != 0xFFFFFFFFu || f1 <= f0) f0 = f1 = pb + 1;
        for (uint64_t pi = pa; pi <= pb; ++pi) {
            if (pi == f0) {
                run(B, base + f0 * P - a, f0, f1, P, sums_off);
                pi = f1 - 1;
                continue;
            }
            const uint64_t ps = pi * P, pe = std::min(ps + P, L);
            const uint64_t s = std::max(a, ps), e = std::min(b, pe);
            const uint64_t ptr_ps = base + ps - a;  // may point before base; only offsets >= s used
            piece(B.items, ptr_ps, ps, pe, s, e, (uint32_t)(sums_off + pi), seed);
        }
    }
};

inline int validate_blobs(const krk_blob* blobs, uint64_t n) {
    KRK_CHECK(n == 0 || blobs, KRK_EINVAL, "blobs is NULL");
    for (uint64_t i = 0; i < n; ++i) {
        KRK_CHECK(blobs[i].piece_length > 0, KRK_EINVAL, "piece length must be positive");
        KRK_CHECK(blobs[i].length == 0 || blobs[i].data, KRK_EINVAL, "blob %llu: data is NULL",
                  (unsigned long long)i);
        const uint64_t np = krk_num_pieces(blobs[i].length, blobs[i].piece_length);
        KRK_CHECK(blobs[i].sums_offset + np <= 0xFFFFFFFFull, KRK_EINVAL,
                  "sums index exceeds 2^32 in one call");
    }
    return KRK_OK;
}

// Zero the sums span [lo, hi) that the blobs cover.
inline void sums_span(const krk_blob* blobs, uint64_t n, uint64_t* lo, uint64_t* hi) {
    *lo = UINT64_MAX;
    *hi = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t np = krk_num_pieces(blobs[i].length, blobs[i].piece_length);
        if (!np) continue;
        *lo = std::min(*lo, blobs[i].sums_offset);
        *hi = std::max(*hi, blobs[i].sums_offset + np);
    }
    if (*lo > *hi) *lo = *hi = 0;
}

inline int run_items(Device* D, const CrcBatch& B, uint32_t* sums_dev, hipStream_t s) {
    if (B.empty()) return KRK_OK;
    KRK_CHECK(B.run_items + B.items.size() < (1ull << 32), KRK_EINVAL, "more than 2^32 CRC work items in one call");
    // One upload: [runs][items][consts], each part 16-byte aligned.
    const size_t nr = B.runs.size() * sizeof(CrcRun), ni = B.items.size() * sizeof(CrcItem);
    const size_t nc = B.consts.size() * 4;
    std::vector<uint8_t> pack(nr + ni + nc);
    if (nr) memcpy(pack.data(), B.runs.data(), nr);
    if (ni) memcpy(pack.data() + nr, B.items.data(), ni);
    if (nc) memcpy(pack.data() + nr + ni, B.consts.data(), nc);
    void* d_pack = nullptr;
    int r = upload(D, pack.data(), pack.size(), &d_pack, s);
    if (r) return r;
    const uint8_t* dp = static_cast<const uint8_t*>(d_pack);
    CrcWork w{};
    w.runs = reinterpret_cast<const CrcRun*>(dp);
    w.items = reinterpret_cast<const CrcItem*>(dp + nr);
    w.consts = reinterpret_cast<const uint32_t*>(dp + nr + ni);
    w.n_runs = (uint32_t)B.runs.size();
    w.run_items = (uint32_t)B.run_items;
    w.n_items = (uint32_t)B.items.size();
    uint32_t* d_next = nullptr;  // the work-queue head, zeroed in stream order
    if (scratch_alloc(D, &d_next, 4, s) != hipSuccess || hipMemsetAsync(d_next, 0, 4, s) != hipSuccess) {
        scratch_free(D, d_pack, s);
        set_error(KRK_EHIP, "crc32_pieces: work-queue head");
        return KRK_EHIP;
    }
    w.next = d_next;
    CrcLaunchCfg cfg{D->cus, D->crc_variant};
    hipError_t e = timed(K_CRC, s, [&] { return launch_crc_items(w, D->d_tabs, sums_dev, cfg, s); });
    scratch_free(D, d_next, s);
    scratch_free(D, d_pack, s);
    KRK_CHECK(e == hipSuccess, KRK_EHIP, "crc32_pieces launch: %s", launch_error_text(e));
    return KRK_OK;
}

inline int piece_sums_dev(Device* D, const krk_blob* blobs, uint64_t n, uint32_t* sums_dev, hipStream_t s) {
    int r = validate_blobs(blobs, n);
    if (r) return r;
    uint64_t lo, hi;
    sums_span(blobs, n, &lo, &hi);
    if (hi == lo) return KRK_OK;
    KRK_CHECK(sums_dev, KRK_EINVAL, "sums_dev is NULL");
    KRK_HIP(hipMemsetAsync(sums_dev + lo, 0, (hi - lo) * 4, s));
    ItemBuilder B;
    CrcBatch items;
    for (uint64_t i = 0; i < n; ++i)
        B.add(items, reinterpret_cast<uint64_t>(blobs[i].data), 0, blobs[i].length, blobs[i].length,
              (uint64_t)blobs[i].piece_length, blobs[i].sums_offset);
    return run_items(D, items, sums_dev, s);
}

// ------------------------------------------------------------------ SHA jobs
inline const uint32_t kIV[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

inline int run_jobs(Device* D, std::vector<ShaJob>& jobs, uint8_t* digests_dev, uint32_t* state_dev,
                    hipStream_t s) {
    if (jobs.empty()) return KRK_OK;
    // Longest streams first: lanes of one wave then carry similar lengths.
    std::stable_sort(jobs.begin(), jobs.end(), [](const ShaJob& a, const ShaJob& b) { return a.len > b.len; });
    void* d_jobs = nullptr;
    int r = upload(D, jobs.data(), jobs.size() * sizeof(ShaJob), &d_jobs, s);
    if (r) return r;
    hipError_t e = timed(K_SHA, s, [&] {
        return launch_sha256(static_cast<const ShaJob*>(d_jobs), (uint32_t)jobs.size(), digests_dev,
                             state_dev, s);
    });
    scratch_free(D, d_jobs, s);
    KRK_CHECK(e == hipSuccess, KRK_EHIP, "sha256_multi launch: %s", launch_error_text(e));
    return KRK_OK;
}

// ------------------------------------------------------------------ host gather
// Spans of page-locked host bytes (src: the device-visible address of a hipHostMalloc'd or
// registered mapping, any alignment) into device memory (dst: 16-B aligned, room for n
// rounded up to 16): ONE gather launch (gather.hip) on s, the bytes read over PCIe by the
// kernel -- no host thread copies them and no DMA descriptor is built per span.
struct GatherSpan {
    uint8_t* dst;
    const uint8_t* src;
    uint64_t n;
};
inline int run_gather(Device* D, const std::vector<GatherSpan>& spans, hipStream_t s) {
    std::vector<GatherTile> tiles;
    for (const GatherSpan& g : spans)
        for (uint64_t o = 0; o < g.n; o += kGatherTile)
            tiles.push_back({reinterpret_cast<uint64_t>(g.src + o), reinterpret_cast<uint64_t>(g.dst + o),
                             std::min<uint64_t>(kGatherTile, g.n - o), 0});
    if (tiles.empty()) return KRK_OK;
    KRK_CHECK(tiles.size() < (1ull << 32), KRK_EINVAL, "more than 2^32 gather tiles in one call");
    void* d_tiles = nullptr;
    int r = upload(D, tiles.data(), tiles.size() * sizeof(GatherTile), &d_tiles, s);
    if (r) return r;
    hipError_t e = timed(K_HOSTG, s, [&] {
        return launch_gather(static_cast<const GatherTile*>(d_tiles), (uint32_t)tiles.size(), D->cus, s);
    });
    scratch_free(D, d_tiles, s);
    KRK_CHECK(e == hipSuccess, KRK_EHIP, "host_gather launch: %s", launch_error_text(e));
    return KRK_OK;
}

inline ShaJob full_job(const void* p, uint64_t len, uint32_t out) {
    ShaJob j{};
    j.ptr = reinterpret_cast<uint64_t>(p);
    j.len = len;
    j.prefix = 0;
    j.out = out;
    j.flags = kShaFinal;
    memcpy(j.h, kIV, sizeof kIV);
    return j;
}



// SHA-256 host offload (offload.cpp): the longest blobs of a batch hashed on host threads
// while the GPU hashes the rest (krk_set_sha_host_offload).  Where the batch lives
// decides what the host saves:
//  * kOffDevice: blobs in HBM; the host reads its blobs out over D2H, the GPU still
//    computes every piece CRC (krk_sha256_dev, krk_metainfo_digest_dev);
//  * kOffHostSha: blobs in host memory, digests only; the host's blobs are hashed in place
//    and never uploaded (krk_sha256_host);
//  * kOffHostWhole: blobs in host memory, digests and piece sums; the host's blobs are
//    hashed AND piece-summed in place and never uploaded (krk_metainfo_digest_host) --
//    the batch's bytes over the host link shrink by theirs.
//  * kOffHostFiles: cache files (krk_metainfo_digest_files): a host blob is read once and
//    hashed and piece-summed chunk by chunk on one host thread.
enum OffMode { kOffDevice = 0, kOffHostSha = 1, kOffHostWhole = 2, kOffHostFiles = 3 };
// Host threads the offload of a `mode` batch may use (krk_set_sha_host_offload; 0 = off).
int offload_threads(int mode = kOffDevice);
bool offload_auto();  // the offload's threads are KRK_OFFLOAD_AUTO (not set by the caller)
// What the planners know about this box (offload.cpp): per-stream SHA-256 rate of each
// AUTO tier at full residency (eight / two / one lane(s)), pinned D2H / H2D, one host
// thread's SHA-256 and CRC-32; measured on the device at first use.
struct Rates {
    double stream[3];
    double d2h, h2d, host_sha, host_crc, host_copy;
    int cus;
    int source;  // KRK_RATES_*
};
Rates planner_rates(Device* D);  // D == nullptr: the override or the nominal rates
int calibrate_device(Device* D);  // (re)measure D's rates now (krk_init, krk_planner_calibrate)
// Host CPUs this process may use (offload.cpp): KRK_HOST_CPUS, else the node's CPUs
// (affinity capped by the cgroup quota) / LOCAL_WORLD_SIZE under a launcher, else the
// node's capped by OMP_NUM_THREADS.
int host_cpu_budget();
// Host threads a call on this thread may use (0: host_cpu_budget()): a *_multi worker runs
// with its share of the budget, so N devices' workers do not start N x 16 copy threads.
inline thread_local int t_host_share = 0;
inline int host_threads_for_call() { return t_host_share > 0 ? t_host_share : host_cpu_budget(); }
uint32_t host_crc32_update(uint32_t crc, const uint8_t* p, size_t n);  // host_meta.cpp
// One host thread's rates, bytes/s, each measured once per process on 16 MiB (offload.cpp;
// no device needed): SHA-256 (x86 SHA extensions), CRC-32 (PCLMUL folding), memcpy.
double host_sha_rate();
double host_crc_rate();
double host_copy_rate();

// The process's host worker pool (host_pool.cpp, host_cpu_budget() - 1 threads).  A batch
// of n items runs on up to `helpers` pool threads idle at construction and on the thread
// that calls join() (which returns once all n are done; the destructor joins).  Items are
// claimed one at a time, so a busy pool delays nobody.
struct HostJob;
class HostBatch {
  public:
    HostBatch(size_t n, int helpers, std::function<void(size_t)> f);
    ~HostBatch() { join(); }
    void join();

  private:
    std::shared_ptr<HostJob> j_;
};
int host_pool_idle();  // pool threads idle right now (not yet promised to a batch)
// Held while a thread runs host hash work: at most host_cpu_budget() such threads at once
// (host_pool.cpp); re-entrant on one thread.  Pool items take one themselves.
struct HostCpuToken {
    HostCpuToken();
    ~HostCpuToken();
    HostCpuToken(const HostCpuToken&) = delete;
    HostCpuToken& operator=(const HostCpuToken&) = delete;
};
void host_parallel_for(size_t n, int helpers, std::function<void(size_t)> f);
// crc(A||B) from crc(A), crc(B), |B| (crc32.Update values).
uint32_t crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
// crc32.Update(crc, p[0, n)) with idle pool threads taking spans of a large buffer.
uint32_t host_crc32_update_par(uint32_t crc, const uint8_t* p, size_t n);
// The placement (KRK_PLACE_HOST / KRK_PLACE_GPU) of a CRC-only call asked for `placement`
// (engine.cpp): AUTO follows krk_set_crc_placement, then the measured host-vs-link
// crossover; -1 with *rc set when GPU is forced and no device is usable.
int resolve_crc_placement(int placement, int* rc);
double host_link(const Rates& R);
// GPU-placed digesters' modelled aggregate for m live streams, and the AUTO Digester
// crossover: the fewest live digesters whose GPU aggregate beats `threads` host SHA-NI
// threads (INT64_MAX: never) -- offload.cpp.
double engine_gpu_bps(uint64_t m, const Rates& R);
int64_t digester_crossover(const Rates& R, int threads);
std::vector<uint32_t> offload_plan(const uint64_t* lens, uint64_t n, int threads, const Rates& R, double* gpu_s,
                                   double* host_s, int mode = kOffDevice);
// Tail handoff of device-resident chains (offload.cpp): chain idx[k] runs its first start[k]
// bytes on the GPU (0: none) and the rest on a host thread from the GPU's midstate; listed in
// the order of start (the host threads' queue).  end_s = the planned batch end, gpu_s = the
// GPU alone; empty when host takeovers would not end the batch sooner.
struct TailPlan {
    std::vector<uint32_t> idx;
    std::vector<uint64_t> start;
    double gpu_s = 0, end_s = 0;
};
TailPlan tail_plan(const uint64_t* lens, uint64_t n, int threads, const Rates& R);
// Where the host threads' chains start (offload_hash): chain j from byte start[j], from the
// GPU's midstate at note + 8 * slot[j] once the GPU has written it there (all eight words
// off kTailSentinel, or gpu_done complete), from the IV when start[j] == 0.
constexpr uint32_t kTailSentinel = 0xFFFFFFFFu;
struct TailSrc {
    const volatile uint32_t* note;
    const uint32_t* slot;
    const uint64_t* start;
    hipEvent_t gpu_done;
};
void offload_teardown(Device& D);  // krk_shutdown: the offload threads' streams and pinned buffers
void offload_hash_host(const std::vector<const uint8_t*>& ptrs, const std::vector<uint64_t>& lens, int threads,
                       uint8_t* out);
// kOffHostWhole: blob j's digest to out + 32 j and its piece sums (piece length plen[j])
// to sums[j][0 .. ceil(len / plen)), on up to `threads` threads; the SHA-256 pass and the
// CRC pass of a blob are separate tasks, longest first.
void offload_whole_host(const std::vector<const uint8_t*>& ptrs, const std::vector<uint64_t>& lens,
                        const std::vector<uint64_t>& plen, const std::vector<uint32_t*>& sums, int threads,
                        uint8_t* out);
int offload_whole_files(const std::vector<const char*>& paths, const std::vector<uint64_t>& lens,
                        const std::vector<uint64_t>& plen, const std::vector<uint32_t*>& sums, int threads,
                        uint8_t* out);
int offload_hash(Device* D, const std::vector<const uint8_t*>& ptrs, const std::vector<uint64_t>& lens, int threads,
                 hipEvent_t ready, uint8_t* out, const TailSrc* tail = nullptr);
int offload_store(Device* D, const std::vector<uint32_t>& idx, const uint8_t* dig, uint8_t* digests_dev,
                  hipStream_t s);

}  // namespace krk
