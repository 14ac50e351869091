// offload.cpp -- host offload of the longest SHA-256 chains of a batch
// (krk_set_sha_host_offload; used by krk_sha256_dev / krk_metainfo_digest_dev on blobs in
// HBM and by krk_sha256_host / krk_metainfo_digest_host on blobs in host memory).
//
// SHA-256 is one sequential chain per blob (core/digester.go:28-72).  A GPU stream runs
// at ~59 MB/s (eight lanes), one x86 core with the SHA extensions at
// ~2 GB/s.  A batch whose longest blobs dominate (C1: one 1 GiB blob; the log-uniform
// regen batches of C5) therefore finishes sooner when host threads take the longest
// chains -- reading them out of HBM through pinned double buffers -- while the GPU
// hashes the rest and the piece CRCs of every blob.  The planner picks how many of the
// longest blobs go to the host by minimising max(GPU time, host time); a batch of equal
// blobs (C2) gains nothing (the GPU's chain is the same blob length) and stays on the GPU.
// Blobs in host memory are worked on in place, never uploaded; krk_metainfo_digest_host's
// host blobs get their piece sums on the host too, which takes their bytes off the host
// link -- C2 end-to-end, link-bound, then hands the host the blobs the link would carry
// past the GPU's own chain time.
#include <fcntl.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <queue>
#include <thread>

#include "runtime.hpp"

namespace krk {

void host_sha256_blocks(uint32_t h[8], const uint8_t* p, size_t nblocks);
void host_sha256_final(const uint32_t h[8], uint64_t absorbed, const uint8_t* tail, size_t n, uint8_t out[32]);
uint32_t host_crc32_update(uint32_t crc, const uint8_t* p, size_t n);

// One host thread, bytes/s: measured once (16 MiB) and derated for the clock a fully
// loaded socket holds.  SHA-256 (x86 SHA extensions) and the piece CRC (PCLMUL folding).
constexpr double kHostDerate = 0.85;
static double time_rate(const std::function<void(const uint8_t*, size_t)>& f) {
    std::vector<uint8_t> buf(16u << 20, 0x5a);
    f(buf.data(), 64 << 10);  // warm
    const auto t0 = std::chrono::steady_clock::now();
    f(buf.data(), buf.size());
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return kHostDerate * buf.size() / std::max(s, 1e-6);
}
double host_sha_rate() {
    static const double r = time_rate([](const uint8_t* p, size_t n) {
        uint32_t h[8];
        memcpy(h, kIV, sizeof h);
        host_sha256_blocks(h, p, n / 64);
    });
    return r;
}
double host_copy_rate() {
    static const double r = [] {
        std::vector<uint8_t> dst(16u << 20, 0);  // touched: page faults are not the copy's cost
        return time_rate([&](const uint8_t* p, size_t n) { memcpy(dst.data(), p, n); });
    }();
    return r;
}
double host_crc_rate() {
    static const double r = time_rate([](const uint8_t* p, size_t n) {
        volatile uint32_t c = host_crc32_update(0, p, n);
        (void)c;
    });
    return r;
}

namespace {

// Host threads of the offload: KRK_OFFLOAD_AUTO (the default) = the CPUs this call may use
// for blobs read out of HBM (their D2H copies need no host CPU), a quarter of them for
// host-resident batches, whose windows need the rest as copy threads (C2 end-to-end: 4 of
// 16 threads 55.5 GB/s, 8 54.4-55.2, 16 49.9).  0 = off, n = n threads.
std::atomic<int> g_off_threads{KRK_OFFLOAD_AUTO};

constexpr uint64_t kOffChunk = 8ull << 20;  // D2H chunk (multiple of 64)

// ------------------------------------------------------------------ planner rates
// Kernel geometry (a property of the code, not of the box): the AUTO launch plan's three
// tiers -- eight lanes a stream up to 16 x CUs streams, two lanes up to 64 x CUs, one
// lane beyond -- and the streams each tier keeps resident per CU (one pair a workgroup
// at eight lanes, two pairs of 32 / 64 streams at two / one lane(s)).
constexpr uint64_t kTierMaxPerCu[2] = {16, 64};
constexpr uint64_t kResidentPerCu[3] = {16, 64, 128};
constexpr int kTierPlan[3] = {KRK_SHA_PLAN_8LANE, KRK_SHA_PLAN_2LANE_2PAIR, KRK_SHA_PLAN_1LANE_2PAIR};

int tier_of(uint64_t m, int cus) {
    return m <= kTierMaxPerCu[0] * (uint64_t)cus ? 0 : m <= kTierMaxPerCu[1] * (uint64_t)cus ? 1 : 2;
}

// Without a device and without krk_planner_rates_set (planning on a host that has no
// GPU, e.g. the CPU tests): one MI355X as measured in rounds 1-2 -- per-stream rates at
// full residency of 52.6 / 51.6 / 35.7 MB/s (profiles/r02/sha8_probe_c2shape.jsonl,
// sha2_read_groups.jsonl), PCIe Gen5 x16 pinned copies of 54 GB/s.
Rates nominal_rates(int cus) {
    Rates R{};
    R.stream[0] = 52.6e6;
    R.stream[1] = 51.6e6;
    R.stream[2] = 35.7e6;
    R.d2h = R.h2d = 54e9;
    R.host_sha = host_sha_rate();
    R.host_crc = host_crc_rate();
    R.host_copy = host_copy_rate();
    R.cus = cus > 0 ? cus : 256;
    R.source = KRK_RATES_NOMINAL;
    return R;
}

}  // namespace

// The calibration's device and pinned buffers, stream and events, kept until krk_shutdown:
// hipFree / hipHostFree wait for the whole device, i.e. for whatever other work is running
// on it when a later call re-measures.
struct CalBufs {
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    uint8_t *d_in = nullptr, *d_dig = nullptr, *d_copy = nullptr, *h_copy = nullptr;
    uint32_t* d_state = nullptr;
    ShaJob* d_jobs = nullptr;
    uint32_t mmax = 0;
};

// Per device: host threads + pinned double buffers of the offload phases, and the planner
// calibration (measured once per device and process, or again on krk_planner_calibrate).
struct Worker;
// A resumer (krk_sha256_resume_dev_on_host): one copy stream, kResumeBufs pinned buffers and
// their events -- copies run up to kResumeBufs - 1 pieces ahead of the hash, so a copy held
// back a few ms behind another stream's packet in a shared hardware queue does not stall it.
constexpr int kResumeBufs = 4;
constexpr uint64_t kResumeChunk = 8ull << 20;  // a copy (16 MiB measured slower beside the C3 windows)
struct Resumer {
    hipStream_t s = nullptr;
    uint8_t* buf[kResumeBufs] = {};
    hipEvent_t ev[kResumeBufs] = {};
};

struct OffloadPool {
    std::mutex mu;
    std::vector<std::vector<Worker>> free_sets;
    std::vector<Resumer> free_resumers;
    std::mutex cal_mu;  // one calibration of this device at a time
    CalBufs cal;
    bool measured = false;
    Rates rates{};
};

namespace {

OffloadPool* pool_of(Device* D) {
    std::lock_guard<std::mutex> g(D->offload_mu);
    if (!D->offload) D->offload = new OffloadPool();
    return D->offload;
}

// The device's own rates (~50 ms): each SHA-256 tier's plan timed on 16 / 64 / 128 x CUs
// streams of 256 KiB (every stream reads the same bytes: the kernel is issue-bound, not
// HBM-bound), pinned 64 MiB copies each way, on a stream of the calibration's own.
int calibrate(Device* D, CalBufs& cb, Rates& R) {
    R = Rates{};
    R.cus = D->cus;
    KRK_HIP(hipSetDevice(D->id));
    const uint64_t L = 256u << 10, C = 64u << 20;
    const uint32_t mmax = (uint32_t)(kResidentPerCu[2] * (uint64_t)D->cus);
    hipStream_t& s = cb.s;
    hipEvent_t &e0 = cb.e0, &e1 = cb.e1;
    uint8_t *&d_in = cb.d_in, *&d_dig = cb.d_dig, *&d_copy = cb.d_copy, *&h_copy = cb.h_copy;
    uint32_t*& d_state = cb.d_state;
    ShaJob*& d_jobs = cb.d_jobs;
    int rc = KRK_OK;
    auto ok = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && !rc) {
            set_error(KRK_EHIP, "planner calibration: %s: %s", what, hipGetErrorString(e));
            rc = KRK_EHIP;
        }
        return !rc;
    };
    auto timed_ms = [&](const std::function<hipError_t()>& f) {
        float ms = 0;
        for (int rep = 0; rep < 2 && !rc; ++rep) {  // the first run loads code and warms up
            ok(hipEventRecord(e0, s), "event");
            ok(f(), "launch");
            ok(hipEventRecord(e1, s), "event");
            ok(hipEventSynchronize(e1), "sync");
            ok(hipEventElapsedTime(&ms, e0, e1), "elapsed");
        }
        return (double)std::max(ms, 1e-3f);
    };
    auto have = [&](bool present, const std::function<hipError_t()>& make, const char* what) {
        return present || ok(make(), what);
    };
    if (cb.mmax < mmax) {  // a device with more CUs than the buffers were made for: start over
        for (void* p : {(void*)d_state, (void*)d_dig, (void*)d_jobs})
            if (p) hipFree(p);
        d_state = nullptr;
        d_dig = nullptr;
        d_jobs = nullptr;
        cb.mmax = mmax;
    }
    if (have(s, [&] { return hipStreamCreateWithFlags(&s, hipStreamNonBlocking); }, "stream") &&
        have(e0, [&] { return hipEventCreate(&e0); }, "event") && have(e1, [&] { return hipEventCreate(&e1); }, "event") &&
        have(d_in, [&] { return hipMalloc(&d_in, L); }, "alloc") &&
        have(d_state, [&] { return hipMalloc(&d_state, 32ull * mmax); }, "alloc") &&
        have(d_dig, [&] { return hipMalloc(&d_dig, 32ull * mmax); }, "alloc") &&
        have(d_jobs, [&] { return hipMalloc(&d_jobs, sizeof(ShaJob) * mmax); }, "alloc") &&
        ok(hipMemsetAsync(d_in, 0x5a, L, s), "memset")) {
        std::vector<ShaJob> jobs(mmax);
        for (uint32_t i = 0; i < mmax; ++i) {
            jobs[i] = ShaJob{};
            jobs[i].ptr = reinterpret_cast<uint64_t>(d_in);
            jobs[i].len = L;
            jobs[i].out = i;
            memcpy(jobs[i].h, kIV, 32);
        }
        if (ok(hipMemcpyAsync(d_jobs, jobs.data(), sizeof(ShaJob) * mmax, hipMemcpyHostToDevice, s), "upload"))
            for (int t = 0; t < 3 && !rc; ++t) {
                const uint32_t m = (uint32_t)(kResidentPerCu[t] * (uint64_t)D->cus);
                const double ms = timed_ms([&] { return launch_sha256_plan(kTierPlan[t], d_jobs, m, d_dig, d_state, s); });
                R.stream[t] = (double)L / (ms * 1e-3);
            }
    }
    if (!rc && have(d_copy, [&] { return hipMalloc(&d_copy, C); }, "alloc") &&
        have(h_copy, [&] { return hipHostMalloc(reinterpret_cast<void**>(&h_copy), C, 0); }, "pin")) {
        // the fastest of three timed copies each way: one copy alone read 45.7 against ~56.5
        // GB/s on one box (bench.py host_link_peak), and the planners price the link with it
        auto best_ms = [&](const std::function<hipError_t()>& f) {
            double ms = timed_ms(f);
            for (int k = 0; k < 2 && !rc; ++k) ms = std::min(ms, timed_ms(f));
            return ms;
        };
        R.h2d = (double)C / (best_ms([&] { return hipMemcpyAsync(d_copy, h_copy, C, hipMemcpyHostToDevice, s); }) * 1e-3);
        R.d2h = (double)C / (best_ms([&] { return hipMemcpyAsync(h_copy, d_copy, C, hipMemcpyDeviceToHost, s); }) * 1e-3);
    }
    if (s) {
        // The buffers stay (freeing waits for the device); the stream does not: a stream
        // kept alive takes a turn in the round-robin of normal-priority streams over the
        // hardware queues, and moved the C3 host lane's D2H copies onto a queue behind the
        // windows' kernels (rank 0's shard of 8 GPUs: lane 16.5 -> 18-20 s).
        hipStreamSynchronize(s);
        hipStreamDestroy(s);
        s = nullptr;
    }
    R.host_sha = host_sha_rate();
    R.host_crc = host_crc_rate();
    R.host_copy = host_copy_rate();
    R.source = KRK_RATES_MEASURED;
    return rc;
}

std::mutex g_rates_mu;  // the override only: a calibration never runs under it
bool g_rates_set = false;
Rates g_rates_override{};

// GPU time of m streams (longest `longest` bytes, `bytes` in all) under the AUTO launch
// plan: the longest chain at the tier's per-stream rate, or the streams' bytes at the
// tier's aggregate (per-stream rate x streams resident on the chip) when they outnumber
// what runs at once.
double gpu_seconds(uint64_t longest, double bytes, uint64_t m, const Rates& R) {
    if (!m) return 0;
    const int t = tier_of(m, R.cus);
    const double r = R.stream[t];
    const double cap = (double)kResidentPerCu[t] * R.cus * r;
    return std::max(longest / r, bytes / std::min(m * r, cap));
}

// One host thread's copy resources: buffer b is filled on stream s[b].  Completion is
// awaited with hipStreamSynchronize, not an event: an event record is a packet on the
// stream's hardware queue, and with more streams than hardware queues (4) it can sit
// behind the batch's own long SHA-256 kernel (tools/micro/d2h_probe.hip: copy kernels
// on 4 of 16 streams waited 1 s for a 1 s kernel on a fifth), while the DMA copies
// themselves do not wait for it.
}  // namespace

// Each offload phase takes a set of worker resources of its own (two streams + two pinned
// buffers a thread), so concurrent callers on one device (several krk_sha256_dev callers,
// *_multi workers sharing a GPU) hash at the same time.
struct Worker {
    hipStream_t s[2] = {nullptr, nullptr};
    uint8_t* buf[2] = {nullptr, nullptr};
};

// (Re)measure device D's rates now; a failed calibration plans with the nominal rates.
int calibrate_device(Device* D) {
    OffloadPool* P = pool_of(D);
    std::lock_guard<std::mutex> g(P->cal_mu);
    Rates R{};
    const int rc = calibrate(D, P->cal, R);
    if (rc != KRK_OK) R = nominal_rates(D->cus);
    std::lock_guard<std::mutex> gp(P->mu);
    P->rates = R;
    P->measured = true;
    return rc;
}

// The rates the planners use on device D: the override, else D's measured rates (the first
// caller on a device measures them; krk_init measures them eagerly, before the device
// carries any work of the library's), else -- no device -- the nominal ones.  Only the
// device being measured waits for its calibration: no process-wide lock is held across it.
Rates planner_rates(Device* D) {
    {
        std::lock_guard<std::mutex> g(g_rates_mu);
        if (g_rates_set) return g_rates_override;
    }
    if (!D) return nominal_rates(0);
    OffloadPool* P = pool_of(D);
    {
        std::lock_guard<std::mutex> g(P->mu);
        if (P->measured) return P->rates;
    }
    {
        std::lock_guard<std::mutex> g(P->cal_mu);  // a concurrent first caller waits for the one measuring
        bool done;
        {
            std::lock_guard<std::mutex> gp(P->mu);
            done = P->measured;
        }
        if (!done) {
            Rates R{};
            if (calibrate(D, P->cal, R) != KRK_OK) R = nominal_rates(D->cus);
            std::lock_guard<std::mutex> gp(P->mu);
            P->rates = R;
            P->measured = true;
        }
    }
    std::lock_guard<std::mutex> g(P->mu);
    return P->rates;
}

// Host-resident batches: the caller's pageable bytes are copied into pinned windows on
// host threads while the previous window uploads; measured end to end at ~0.85 of the
// pinned H2D rate (C2 end-to-end 45.7-54.4 GB/s against 54 GB/s pinned).
double host_link(const Rates& R) { return 0.85 * R.h2d; }

// The AUTO Digester crossover (engine.cpp host_stream_limit): m live digesters on the
// host run SHA-NI on their writers' threads, min(m, threads) x one thread's rate; on the
// GPU their pending slots are coalesced into multi-stream launches that read the pinned
// slots in place, m x the tier's per-stream rate (x kEngineEff: the engine's launches
// start and end with the writers, measured 0.93 of the batch kernel's rate at 256
// digesters, profiles/r04/bench_engine.json) up to the tier's residency, capped by what the
// engine's zero-copy slot reads carry over the link (kEngineLinkFrac of the pinned H2D
// rate: at most 32.7 GB/s of 56.3 measured, at 2,048 digesters, profiles/r05/
// bench_engine_inflight_cap.json).  The crossover is the smallest m whose GPU aggregate beats the host's;
// none (the host out-hashes the engine) is INT64_MAX: every AUTO digester stays on the host.
constexpr double kEngineEff = 0.93;
constexpr double kEngineLinkFrac = 0.58;
double engine_gpu_bps(uint64_t m, const Rates& R) {
    if (!m) return 0;
    const int t = tier_of(m, R.cus);
    const double r = R.stream[t] * kEngineEff;
    return std::min({(double)m * r, (double)kResidentPerCu[t] * R.cus * r, kEngineLinkFrac * R.h2d});
}
int64_t digester_crossover(const Rates& R, int threads) {
    const double host = std::max(1, threads) * R.host_sha;
    for (int t = 0; t < 3; ++t) {  // the first m (tier by tier) with m x r > host
        const uint64_t lo = t == 0 ? 1 : kTierMaxPerCu[t - 1] * (uint64_t)R.cus + 1;
        const uint64_t hi = t < 2 ? kTierMaxPerCu[t] * (uint64_t)R.cus : UINT64_MAX / 2;
        const double r = R.stream[t] * kEngineEff;
        const uint64_t m = std::max<uint64_t>(lo, (uint64_t)(host / r) + 1);
        if (m <= hi && engine_gpu_bps(m, R) > host) return (int64_t)m;
    }
    return INT64_MAX;
}

std::vector<uint32_t> offload_plan(const uint64_t* lens, uint64_t n, int threads, const Rates& R, double* gpu_s,
                                   double* host_s, int mode) {
    std::vector<uint32_t> order(n);
    for (uint64_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return lens[a] > lens[b]; });
    std::vector<double> suffix(n + 1, 0.0);
    for (uint64_t k = n; k-- > 0;) suffix[k] = suffix[k + 1] + (double)lens[order[k]];
    // GPU side with blobs k.. on the GPU: their longest chain / the chip's SHA rate, and for
    // host-resident batches their bytes over the host link (the host's blobs never cross).
    auto gpu_side = [&](uint64_t k) {
        double g = k < n ? gpu_seconds(lens[order[k]], suffix[k], n - k, R) : 0.0;
        if (mode != kOffDevice) g = std::max(g, suffix[k] / host_link(R));
        return g;
    };
    const double f0 = n ? gpu_side(0) : 0.0;
    double best = f0, best_g = f0, best_h = 0;
    uint64_t best_k = 0;
    if (threads > 0 && n) {
        const double rs = R.host_sha, rc = mode == kOffHostWhole ? R.host_crc : 0.0;
        // LPT over host threads of the tasks, in seconds: a SHA-256 pass per blob, and in
        // kOffHostWhole a piece-CRC pass per blob as its own task.
        std::priority_queue<double, std::vector<double>, std::greater<double>> load;
        for (int t = 0; t < threads; ++t) load.push(0.0);
        double maxload = 0, hbytes = 0;
        auto put = [&](double sec) {
            const double l = load.top() + sec;
            load.pop();
            load.push(l);
            maxload = std::max(maxload, l);
        };
        for (uint64_t k = 1; k <= n; ++k) {
            const double L = (double)lens[order[k - 1]];
            if (L == 0) break;  // empty blobs are not worth a thread
            if (mode == kOffHostFiles) {
                put(L / rs + L / R.host_crc + L / R.host_copy);  // one read, SHA-256 and CRC per chunk
            } else {
                put(L / rs);
                if (mode == kOffHostWhole) put(L / rc);
            }
            hbytes += L;
            const double h = mode == kOffDevice ? std::max(maxload, hbytes / R.d2h) : maxload;
            const double g = gpu_side(k);
            if (std::max(g, h) < best) {
                best = std::max(g, h);
                best_k = k;
                best_g = g;
                best_h = h;
            }
            if (h > f0) break;  // the host alone is already slower than no offload
        }
        if (best > (mode == kOffDevice ? 0.9 : 0.97) * f0) {
            best_k = 0;
            best_g = f0;
            best_h = 0;
        }
    }
    if (gpu_s) *gpu_s = best_g;
    if (host_s) *host_s = best_h;
    order.resize(best_k);
    return order;
}

// Tail handoff of device-resident chains (kOffDevice): every chain starts on the GPU and
// host threads take over the tails of the longest ones.  A SHA-256 chain is one sequential
// Merkle-Damgard stream, so a batch of equally long chains (C2: 1,000 x 100 MiB) ends when
// one chain ends at the GPU's ~59 MB/s a stream, however many are moved whole to the host --
// but a host thread (SHA-NI, ~2 GB/s) that takes chain i over at time t finishes it in
// (L_i - r t) / h, and the GPU has done r t of it meanwhile.  Host threads working through
// takeovers one after another shrink the batch's end E: for C2 on 16 threads the model gives
// ~1.48 s against 1.78 s on the GPU alone.
// Plan for a target E: chains the GPU ends by E (L_i <= r E) stay; every other chain must be
// taken over by its deadline (E - L_i / h) / (1 - r / h); earliest deadline first over the
// threads (each free at the end of its previous tail), the GPU's prefix Y_i = r t_i rounded
// down to a 64-byte block.  E is the smallest feasible target (bisection).  r = the per-
// stream rate of the batch's plan tier, h = one thread's SHA-NI rate, capped by its share of
// the device-to-host copy rate.
TailPlan tail_plan(const uint64_t* lens, uint64_t n, int threads, const Rates& R) {
    TailPlan best;
    if (!n || threads <= 0) return best;
    const double r = R.stream[tier_of(n, R.cus)];
    // a tail thread runs SHA-NI alone over its two pinned buffers: 16 of them hashed 2.42
    // GB/s each against 2.47 for one C1 thread (profiles/r05/c2_tail_handoff_trace.txt), so
    // the rate is derated 2 %, not the 15 % that holds for the host-whole and file modes
    // (SHA + CRC + copies: the warm files leg lost 58.9 -> 55.0 GB/s when those were priced
    // at 5 %)
    const double h = std::min(R.host_sha * (0.98 / kHostDerate), R.d2h / threads);
    if (!(r > 0) || !(h > r)) return best;
    uint64_t longest = 0;
    double total = 0;
    for (uint64_t i = 0; i < n; ++i) {
        longest = std::max(longest, lens[i]);
        total += (double)lens[i];
    }
    best.gpu_s = gpu_seconds(longest, total, n, R);
    // only chain-bound batches gain (the GPU's time is its longest chain, not its aggregate
    // rate), and the plan stays cheap: at most 65,536 chains
    if (n > (1u << 16) || longest / r < 0.9 * best.gpu_s) return best;
    std::vector<uint32_t> order(n);
    for (uint64_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return lens[a] > lens[b]; });
    auto plan = [&](double E, TailPlan* out) {
        std::priority_queue<double, std::vector<double>, std::greater<double>> free_at;
        for (int t = 0; t < threads; ++t) free_at.push(0.0);
        for (uint32_t i : order) {  // longest first = earliest deadline first
            const double L = (double)lens[i];
            if (L <= r * E) break;
            const double deadline = (E - L / h) / (1.0 - r / h);
            const double t = free_at.top();
            if (deadline < 0 || t > deadline) return false;
            free_at.pop();
            const uint64_t y = std::min<uint64_t>((uint64_t)(r * t) / 64 * 64, lens[i] / 64 * 64);
            free_at.push(t + (L - (double)y) / h);
            if (out) {
                out->idx.push_back(i);
                out->start.push_back(y);
            }
        }
        return true;
    };
    double lo = 0, hi = best.gpu_s;
    if (plan(0.0, nullptr) || !plan(hi, nullptr)) return best;  // nothing to gain
    for (int it = 0; it < 40; ++it) {
        const double mid = 0.5 * (lo + hi);
        (plan(mid, nullptr) ? hi : lo) = mid;
    }
    plan(hi, &best);
    best.end_s = hi;
    // takeovers in the order their prefixes end on the GPU (the host threads' queue)
    std::vector<size_t> o(best.idx.size());
    for (size_t k = 0; k < o.size(); ++k) o[k] = k;
    std::stable_sort(o.begin(), o.end(), [&](size_t a, size_t b) { return best.start[a] < best.start[b]; });
    TailPlan sorted;
    sorted.gpu_s = best.gpu_s;
    sorted.end_s = best.end_s;
    for (size_t k : o) {
        sorted.idx.push_back(best.idx[k]);
        sorted.start.push_back(best.start[k]);
    }
    return sorted;
}

bool offload_auto() { return g_off_threads.load(std::memory_order_relaxed) == KRK_OFFLOAD_AUTO; }

int offload_threads(int mode) {
    const int t = g_off_threads.load(std::memory_order_relaxed);
    if (t != KRK_OFFLOAD_AUTO) return t;
    const int budget = host_threads_for_call();
    return mode == kOffDevice ? budget : std::max(1, budget / 4);
}

// The node's CPUs as this process sees them: its affinity mask capped by the cgroup v2 CPU
// quota (the GPU boxes expose the whole machine in the mask but grant a share of it).
static int node_cpu_count() {
    cpu_set_t set;
    int c = sched_getaffinity(0, sizeof set, &set) == 0 ? std::max(1, CPU_COUNT(&set))
                                                        : (int)std::max(1u, std::thread::hardware_concurrency());
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {  // "<quota> <period>" or "max <period>"
        char q[32] = {0};
        long long per = 0;
        if (fscanf(f, "%31s %lld", q, &per) == 2 && strcmp(q, "max") != 0 && per > 0)
            c = std::min<int>(c, std::max<long long>(1, atoll(q) / per));
        fclose(f);
    }
    return c;
}

static int env_pos(const char* e) {
    return e && atoi(e) > 0 ? atoi(e) : 0;
}

struct CpuBudget {
    int cpus, node;
    const char* source;
};

// One process per GPU (origin/cmd/cmd.go:164 runs one origin a host; bench.py and
// torch.distributed.run start one rank a GPU): the ranks of a node share its CPUs.
//   KRK_HOST_CPUS            an operator's explicit per-process budget;
//   LOCAL_WORLD_SIZE > 1     the node's CPUs / the ranks on it -- a launcher's
//                            OMP_NUM_THREADS (torch.distributed.run sets 1 a rank) is
//                            about OpenMP pools, not this library's hash threads;
//   otherwise                the node's CPUs, capped by OMP_NUM_THREADS when set.
static const CpuBudget& cpu_budget() {
    static const CpuBudget b = [] {
        const int node = node_cpu_count();
        if (int x = env_pos(KRK_OP_ENV("KRK_HOST_CPUS"))) return CpuBudget{x, node, "KRK_HOST_CPUS"};
        if (int w = env_pos(getenv("LOCAL_WORLD_SIZE")); w > 1)
            return CpuBudget{std::max(1, node / w), node, "node/LOCAL_WORLD_SIZE"};
        if (int o = env_pos(getenv("OMP_NUM_THREADS")); o > 0 && o < node)
            return CpuBudget{o, node, "OMP_NUM_THREADS"};
        return CpuBudget{node, node, "node"};
    }();
    return b;
}

int host_cpu_budget() { return cpu_budget().cpus; }

// Hash blobs (device pointers, lengths) on up to `threads` host threads; digest j to
// out + 32 j.  The D2H copies start once `ready` (recorded on the caller's stream: the
// bytes may still be being written there) has completed.  Blocks until all are hashed.
int offload_hash(Device* D, const std::vector<const uint8_t*>& ptrs, const std::vector<uint64_t>& lens, int threads,
                 hipEvent_t ready, uint8_t* out, const TailSrc* tail) {
    if (ptrs.empty()) return KRK_OK;
    OffloadPool& P = *pool_of(D);
    // at least one thread: the knob may have been lowered since the plan was made
    const int T = (int)std::min<size_t>((size_t)std::max(threads, 1), ptrs.size());
    std::vector<Worker> set;
    {
        std::lock_guard<std::mutex> g(P.mu);
        if (!P.free_sets.empty()) {
            set = std::move(P.free_sets.back());
            P.free_sets.pop_back();
        }
    }
    struct Return {  // the set goes back to the pool whatever happens below
        OffloadPool& P;
        std::vector<Worker>& set;
        ~Return() {
            std::lock_guard<std::mutex> g(P.mu);
            P.free_sets.push_back(std::move(set));
        }
    } give_back{P, set};
    while ((int)set.size() < T) {
        Worker w;
        for (int b = 0; b < 2; ++b) {
            const hipError_t es = hipStreamCreateWithFlags(&w.s[b], hipStreamNonBlocking);
            const hipError_t eb = es == hipSuccess
                                      ? hipHostMalloc(reinterpret_cast<void**>(&w.buf[b]), kOffChunk, hipHostMallocDefault)
                                      : es;
            if (eb != hipSuccess) {  // undo what this worker made so far
                for (int c = 0; c <= b; ++c) {
                    if (w.s[c]) hipStreamDestroy(w.s[c]);
                    if (w.buf[c]) hipHostFree(w.buf[c]);
                }
                if (es != hipSuccess) set_error(KRK_EHIP, "sha256 host offload: stream: %s", hipGetErrorString(es));
                else set_error(KRK_ENOMEM, "sha256 host offload: pinned buffers");
                return es != hipSuccess ? KRK_EHIP : KRK_ENOMEM;
            }
        }
        set.push_back(w);
    }
    std::atomic<size_t> next{0};
    std::atomic<int> err{0};
    static const bool trace = KRK_OP_ENV("KRK_TRACE") && atoi(KRK_OP_ENV("KRK_TRACE")) > 0;
    std::vector<double> t_wait(T, 0.0), t_hash(T, 0.0);
    const auto t_start = std::chrono::steady_clock::now();
    auto secs = [](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t)
        pool.emplace_back([&, t] {
            Worker& W = set[t];
            // The host waits for `ready` (the caller's stream up to the call; the batch's own
            // kernels come after it): a stream wait packet could queue behind those kernels.
            if (hipSetDevice(D->id) != hipSuccess || hipEventSynchronize(ready) != hipSuccess) {
                err.store(1);
                return;
            }
            for (size_t j; !err.load() && (j = next.fetch_add(1)) < ptrs.size();) {
                const uint64_t st = tail ? tail->start[j] : 0;  // the GPU's prefix of the chain
                const uint8_t* src = ptrs[j] + st;
                const uint64_t L = lens[j] - st;
                const uint64_t nch = std::max<uint64_t>(1, (L + kOffChunk - 1) / kOffChunk);
                auto issue = [&](uint64_t c) {
                    const uint64_t o = c * kOffChunk, m = std::min(kOffChunk, L - o);
                    return m == 0 ||
                           hipMemcpyAsync(W.buf[c & 1], src + o, m, hipMemcpyDeviceToHost, W.s[c & 1]) == hipSuccess;
                };
                uint32_t h[8];
                memcpy(h, kIV, sizeof h);
                uint64_t absorbed = st;
                bool ok = issue(0);  // the first chunk comes down while the midstate is awaited
                if (ok && st) {
                    const volatile uint32_t* w = tail->note + 8 * (uint64_t)tail->slot[j];
                    const auto tw = std::chrono::steady_clock::now();
                    for (;;) {
                        bool all = true;
                        for (int k = 0; k < 8 && all; ++k) all = w[k] != kTailSentinel;
                        if (all) break;
                        const hipError_t q = hipEventQuery(tail->gpu_done);
                        if (q == hipSuccess) break;  // the kernel has ended: the words are final
                        if (q != hipErrorNotReady) {
                            ok = false;
                            break;
                        }
                        std::this_thread::sleep_for(std::chrono::microseconds(20));
                    }
                    for (int k = 0; k < 8; ++k) h[k] = w[k];
                    t_wait[t] += secs(tw);
                }
                for (uint64_t c = 0; ok && c < nch; ++c) {
                    if (c + 1 < nch) ok = issue(c + 1);  // into the other buffer, hashed at c - 1
                    const auto tw = std::chrono::steady_clock::now();
                    if (!ok || hipStreamSynchronize(W.s[c & 1]) != hipSuccess) {
                        ok = false;
                        break;
                    }
                    const auto th = std::chrono::steady_clock::now();
                    t_wait[t] += std::chrono::duration<double>(th - tw).count();
                    const uint64_t m = std::min(kOffChunk, L - c * kOffChunk);
                    if (c + 1 < nch) {
                        host_sha256_blocks(h, W.buf[c & 1], m / 64);
                        absorbed += m;
                    } else {
                        host_sha256_final(h, absorbed, W.buf[c & 1], m, out + 32 * j);
                    }
                    t_hash[t] += secs(th);
                }
                if (!ok) {
                    hipStreamSynchronize(W.s[0]);  // leave no copy in flight into the buffers
                    hipStreamSynchronize(W.s[1]);
                    err.store(1);
                }
            }
        });
    for (auto& th : pool) th.join();
    if (trace) {
        uint64_t bytes = 0;
        for (uint64_t L : lens) bytes += L;
        double w = 0, h = 0;
        for (int t = 0; t < T; ++t) {
            w += t_wait[t];
            h += t_hash[t];
        }
        fprintf(stderr, "krk_trace sha_offload: threads=%d blobs=%zu bytes=%llu wall=%.3fs wait=%.3fs hash=%.3fs (thread sums)\n",
                T, ptrs.size(), (unsigned long long)bytes, secs(t_start), w, h);
    }
    KRK_CHECK(!err.load(), KRK_EHIP, "sha256 host offload: device-to-host copy failed");
    return KRK_OK;
}

// The calling thread's seconds in krk_sha256_resume_dev_on_host waiting for device-to-host
// copies and hashing (krk_sha256_resume_stats).
static thread_local double t_resume_wait = 0, t_resume_hash = 0, t_resume_issue = 0, t_resume_ready = 0;

// One chain continued on the calling thread from device bytes (krk_sha256_resume_dev_on_host):
// a resumer of the device's pool, the D2H copies kResumeBufs - 1 kOffChunk pieces ahead of
// SHA-NI over each.
static int resume_on_host(Device* D, uint32_t h[8], uint64_t absorbed, const uint8_t* src, uint64_t L, bool final,
                          uint8_t* digest, hipEvent_t ready) {
    OffloadPool& P = *pool_of(D);
    Resumer R;
    {
        std::lock_guard<std::mutex> g(P.mu);
        if (!P.free_resumers.empty()) {
            R = P.free_resumers.back();
            P.free_resumers.pop_back();
        }
    }
    if (!R.s) {
        bool ok = hipStreamCreateWithFlags(&R.s, hipStreamNonBlocking) == hipSuccess;
        for (int b = 0; ok && b < kResumeBufs; ++b)
            ok = hipHostMalloc(reinterpret_cast<void**>(&R.buf[b]), kResumeChunk, hipHostMallocDefault) == hipSuccess &&
                 hipEventCreateWithFlags(&R.ev[b], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            if (R.s) hipStreamDestroy(R.s);
            for (int b = 0; b < kResumeBufs; ++b) {
                if (R.buf[b]) hipHostFree(R.buf[b]);
                if (R.ev[b]) hipEventDestroy(R.ev[b]);
            }
            KRK_CHECK(false, KRK_ENOMEM, "sha256 resume: pinned buffers / stream");
        }
    }
    struct Return {
        OffloadPool& P;
        Resumer& R;
        ~Return() {
            std::lock_guard<std::mutex> g(P.mu);
            P.free_resumers.push_back(R);
        }
    } give_back{P, R};
    if (ready) {
        const auto tr = std::chrono::steady_clock::now();
        KRK_HIP(hipEventSynchronize(ready));
        t_resume_ready += std::chrono::duration<double>(std::chrono::steady_clock::now() - tr).count();
    }
    const uint64_t nch = std::max<uint64_t>(1, (L + kResumeChunk - 1) / kResumeChunk);
    auto issue = [&](uint64_t c) {
        const auto ti = std::chrono::steady_clock::now();
        const uint64_t o = c * kResumeChunk, m = std::min(kResumeChunk, L - o);
        const int b = (int)(c % kResumeBufs);
        const bool ok = (m == 0 || hipMemcpyAsync(R.buf[b], src + o, m, hipMemcpyDeviceToHost, R.s) == hipSuccess) &&
                        hipEventRecord(R.ev[b], R.s) == hipSuccess;
        t_resume_issue += std::chrono::duration<double>(std::chrono::steady_clock::now() - ti).count();
        return ok;
    };
    bool ok = true;
    uint64_t issued = 0;
    for (; ok && issued < std::min<uint64_t>(nch, kResumeBufs - 1); ++issued) ok = issue(issued);
    for (uint64_t c = 0; ok && c < nch; ++c) {
        if (issued < nch) ok = issue(issued++);  // into the buffer hashed at c - 1
        const auto tw = std::chrono::steady_clock::now();
        if (!ok || hipEventSynchronize(R.ev[c % kResumeBufs]) != hipSuccess) {
            ok = false;
            break;
        }
        const auto th = std::chrono::steady_clock::now();
        const uint64_t m = std::min(kResumeChunk, L - c * kResumeChunk);
        const uint8_t* p = R.buf[c % kResumeBufs];
        if (c + 1 < nch || !final) {
            host_sha256_blocks(h, p, m / 64);
            absorbed += m;
        } else {
            host_sha256_final(h, absorbed, p, m, digest);
        }
        t_resume_wait += std::chrono::duration<double>(th - tw).count();
        t_resume_hash += std::chrono::duration<double>(std::chrono::steady_clock::now() - th).count();
    }
    if (!ok) hipStreamSynchronize(R.s);  // leave no copy in flight into the buffers
    KRK_CHECK(ok, KRK_EHIP, "sha256 resume: device-to-host copy failed");
    return KRK_OK;
}

void offload_teardown(Device& D) {  // krk_shutdown: no offload phase is running (contract)
    OffloadPool* P = D.offload;
    if (!P) return;
    for (auto& set : P->free_sets)
        for (Worker& w : set)
            for (int b = 0; b < 2; ++b) {
                if (w.s[b]) hipStreamSynchronize(w.s[b]), hipStreamDestroy(w.s[b]);
                if (w.buf[b]) hipHostFree(w.buf[b]);
            }
    for (Resumer& r : P->free_resumers) {
        if (r.s) hipStreamSynchronize(r.s), hipStreamDestroy(r.s);
        for (int b = 0; b < kResumeBufs; ++b) {
            if (r.buf[b]) hipHostFree(r.buf[b]);
            if (r.ev[b]) hipEventDestroy(r.ev[b]);
        }
    }
    CalBufs& c = P->cal;
    if (c.s) hipStreamSynchronize(c.s), hipStreamDestroy(c.s);
    for (void* p : {(void*)c.d_in, (void*)c.d_state, (void*)c.d_dig, (void*)c.d_jobs, (void*)c.d_copy})
        if (p) hipFree(p);
    if (c.h_copy) hipHostFree(c.h_copy);
    if (c.e0) hipEventDestroy(c.e0);
    if (c.e1) hipEventDestroy(c.e1);
    delete P;
    D.offload = nullptr;
}

// Hash host-resident blobs on up to `threads` threads (next-longest first); digest j to
// out + 32 j.
void offload_hash_host(const std::vector<const uint8_t*>& ptrs, const std::vector<uint64_t>& lens, int threads,
                       uint8_t* out) {
    std::atomic<size_t> next{0};
    auto work = [&] {
        for (size_t j; (j = next.fetch_add(1)) < ptrs.size();) {
            HostCpuToken tok;  // a blob at a time under the process's CPU tokens
            uint32_t h[8];
            memcpy(h, kIV, sizeof h);
            host_sha256_final(h, 0, ptrs[j], lens[j], out + 32 * j);
        }
    };
    const int T = (int)std::min<size_t>((size_t)std::max(threads, 1), ptrs.size());
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
}

void offload_whole_host(const std::vector<const uint8_t*>& ptrs, const std::vector<uint64_t>& lens,
                        const std::vector<uint64_t>& plen, const std::vector<uint32_t*>& sums, int threads,
                        uint8_t* out) {
    // Task t: blob t / 2, its SHA-256 pass (even t) or its piece-CRC pass (odd t), in
    // order of cost (the CRC pass runs ~6x the SHA-256 rate on one core).
    const double rs = host_sha_rate(), rc = host_crc_rate();
    std::vector<std::pair<double, size_t>> tasks;
    tasks.reserve(2 * ptrs.size());
    for (size_t j = 0; j < ptrs.size(); ++j) {
        tasks.push_back({lens[j] / rs, 2 * j});
        if (lens[j]) tasks.push_back({lens[j] / rc, 2 * j + 1});  // an empty blob has no pieces
    }
    std::stable_sort(tasks.begin(), tasks.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
    std::atomic<size_t> next{0};
    auto work = [&] {
        for (size_t q; (q = next.fetch_add(1)) < tasks.size();) {
            HostCpuToken tok;  // a task at a time under the process's CPU tokens
            const size_t j = tasks[q].second / 2;
            const uint8_t* p = ptrs[j];
            const uint64_t L = lens[j];
            if (tasks[q].second % 2 == 0) {
                uint32_t h[8];
                memcpy(h, kIV, sizeof h);
                host_sha256_final(h, 0, p, L, out + 32 * j);
            } else {
                // core/metainfo.go:157-179: piece i = bytes [iP, min((i+1)P, L)), crc32 each
                const uint64_t P = plen[j];
                for (uint64_t o = 0, i = 0; o < L; o += P, ++i) sums[j][i] = host_crc32_update(0, p + o, std::min(P, L - o));
            }
        }
    };
    const int T = (int)std::min<size_t>((size_t)std::max(threads, 1), tasks.size());
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
}

// kOffHostFiles: file j read once in 1 MiB chunks, each chunk hashed (SHA-256) and its
// piece portions CRC'd while it is in the cache; digest to out + 32 j, sums to sums[j].
// Errors keep the reference's texts ("open <path>: ...", "read blob: <path>: ...").
int offload_whole_files(const std::vector<const char*>& paths, const std::vector<uint64_t>& lens,
                        const std::vector<uint64_t>& plen, const std::vector<uint32_t*>& sums, int threads,
                        uint8_t* out) {
    constexpr size_t kChunk = size_t(1) << 20;  // a multiple of 64: only the last chunk is partial
    std::atomic<size_t> next{0};
    std::atomic<bool> failed{false};
    std::mutex emu;
    int rc = KRK_OK;
    std::string msg;
    auto fail = [&](int code, const std::string& m) {
        std::lock_guard<std::mutex> g(emu);
        if (!rc) {
            rc = code;
            msg = m;
        }
        failed = true;
    };
    auto work = [&] {
        std::vector<uint8_t> buf(kChunk);
        for (size_t j; !failed && (j = next.fetch_add(1)) < paths.size();) {
            HostCpuToken tok;  // a file at a time under the process's CPU tokens
            const int fd = open(paths[j], O_RDONLY | O_CLOEXEC);
            if (fd < 0) {
                fail(KRK_EIO, std::string("open ") + paths[j] + ": " + strerror(errno));
                return;
            }
            const uint64_t L = lens[j], P = plen[j];
            uint32_t h[8];
            memcpy(h, kIV, sizeof h);
            uint32_t crc = 0;
            uint64_t pos = 0, in_piece = 0, piece = 0;
            bool ok = true;
            do {
                const size_t m = (size_t)std::min<uint64_t>(kChunk, L - pos);
                for (size_t got = 0; got < m;) {
                    const ssize_t g = pread(fd, buf.data() + got, m - got, (off_t)(pos + got));
                    if (g < 0 && errno == EINTR) continue;
                    if (g <= 0) {
                        fail(KRK_EIO, std::string("read blob: ") + paths[j] + ": " +
                                          (g < 0 ? strerror(errno) : "unexpected EOF"));
                        ok = false;
                        break;
                    }
                    got += (size_t)g;
                }
                if (!ok) break;
                for (size_t q = 0; q < m;) {  // core/metainfo.go:157-179 over this chunk
                    const size_t take = (size_t)std::min<uint64_t>(m - q, P - in_piece);
                    crc = host_crc32_update(crc, buf.data() + q, take);
                    q += take;
                    in_piece += take;
                    if (in_piece == P) {
                        sums[j][piece++] = crc;
                        crc = 0;
                        in_piece = 0;
                    }
                }
                if (pos + m < L) host_sha256_blocks(h, buf.data(), m / 64);
                else host_sha256_final(h, pos, buf.data(), m, out + 32 * j);
                pos += m;
            } while (pos < L);
            if (ok && in_piece) sums[j][piece] = crc;
            close(fd);
            if (!ok) return;
        }
    };
    const int T = (int)std::min<size_t>((size_t)std::max(threads, 1), paths.size());
    std::vector<std::thread> pool;
    for (int t = 1; t < T; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
    if (rc) set_error(rc, "%s", msg.c_str());
    return rc;
}

// Write host-computed digests into digests_dev (record j: 4-byte blob index, 32-byte
// digest) on stream s: one upload + one scatter launch.
int offload_store(Device* D, const std::vector<uint32_t>& idx, const uint8_t* dig, uint8_t* digests_dev,
                  hipStream_t s) {
    if (idx.empty()) return KRK_OK;
    std::vector<uint8_t> rec(idx.size() * 36);
    for (size_t j = 0; j < idx.size(); ++j) {
        memcpy(&rec[36 * j], &idx[j], 4);
        memcpy(&rec[36 * j + 4], dig + 32 * j, 32);
    }
    void* d = nullptr;
    int r = upload(D, rec.data(), rec.size(), &d, s);
    if (r) return r;
    hipError_t e = launch_digest_scatter(static_cast<const uint8_t*>(d), (uint32_t)idx.size(), digests_dev, s);
    scratch_free(D, d, s);
    KRK_CHECK(e == hipSuccess, KRK_EHIP, "digest scatter launch: %s", launch_error_text(e));
    return KRK_OK;
}

}  // namespace krk

using namespace krk;

extern "C" {

int krk_set_sha_host_offload(int threads) {
    KRK_CHECK(threads == KRK_OFFLOAD_AUTO || (threads >= 0 && threads <= 1024), KRK_EINVAL,
              "host offload threads %d outside -1 (auto), 0..1024", threads);
    g_off_threads.store(threads);
    return KRK_OK;
}

int krk_sha_host_offload(int* threads) {
    KRK_CHECK(threads, KRK_EINVAL, "threads is NULL");
    *threads = g_off_threads.load();
    return KRK_OK;
}

int krk_planner_calibrate(void) {
    KRK_DEVICE(D);
    return calibrate_device(D);
}

int krk_host_offload_plan(const uint64_t* lengths, uint64_t n, int threads, int cus, int mode, uint32_t* host_idx,
                          uint64_t* n_host, double* gpu_seconds_out, double* host_seconds_out) {
    KRK_CHECK(n == 0 || lengths, KRK_EINVAL, "lengths is NULL");
    KRK_CHECK(n_host, KRK_EINVAL, "n_host is NULL");
    KRK_CHECK(threads >= 0 && cus >= 0, KRK_EINVAL, "threads and cus must be >= 0");
    static_assert(KRK_OFFLOAD_DEVICE == kOffDevice && KRK_OFFLOAD_HOST_SHA == kOffHostSha &&
                      KRK_OFFLOAD_HOST_WHOLE == kOffHostWhole && KRK_OFFLOAD_HOST_FILES == kOffHostFiles,
                  "offload modes");
    KRK_CHECK(mode >= KRK_OFFLOAD_DEVICE && mode <= KRK_OFFLOAD_HOST_FILES, KRK_EINVAL, "offload mode %d", mode);
    int drc = KRK_OK;
    Device* D = device(&drc);  // none: the override or the nominal rates
    Rates R = planner_rates(D);
    if (cus > 0) R.cus = cus;
    std::vector<uint32_t> idx = offload_plan(lengths, n, threads, R, gpu_seconds_out, host_seconds_out, mode);
    *n_host = idx.size();
    if (host_idx && !idx.empty()) memcpy(host_idx, idx.data(), idx.size() * 4);
    return KRK_OK;
}

int krk_planner_rates_get(krk_planner_rates* out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    int drc = KRK_OK;
    const Rates R = planner_rates(device(&drc));
    for (int t = 0; t < 3; ++t) out->sha_stream_bps[t] = R.stream[t];
    out->d2h_bps = R.d2h;
    out->h2d_bps = R.h2d;
    out->host_sha_bps = R.host_sha;
    out->host_crc_bps = R.host_crc;
    out->host_copy_bps = R.host_copy;
    out->cus = R.cus;
    out->source = R.source;
    return KRK_OK;
}

int krk_planner_rates_set(const krk_planner_rates* in) {
    std::lock_guard<std::mutex> g(g_rates_mu);
    if (!in) {
        g_rates_set = false;
        return KRK_OK;
    }
    KRK_CHECK(in->sha_stream_bps[0] > 0 && in->sha_stream_bps[1] > 0 && in->sha_stream_bps[2] > 0 &&
                  in->d2h_bps > 0 && in->h2d_bps > 0 && in->host_sha_bps > 0 && in->host_crc_bps > 0 && in->host_copy_bps > 0 && in->cus > 0,
              KRK_EINVAL, "planner rates must be positive");
    Rates R{};
    for (int t = 0; t < 3; ++t) R.stream[t] = in->sha_stream_bps[t];
    R.d2h = in->d2h_bps;
    R.h2d = in->h2d_bps;
    R.host_sha = in->host_sha_bps;
    R.host_crc = in->host_crc_bps;
    R.host_copy = in->host_copy_bps;
    R.cus = in->cus;
    R.source = KRK_RATES_SET;
    g_rates_override = R;
    g_rates_set = true;
    return KRK_OK;
}

int krk_sha256_resume_dev_on_host(uint32_t* state8, uint64_t absorbed, const uint8_t* data_dev, uint64_t n,
                                  int final, uint8_t* digest32, void* stream) {
    KRK_CHECK(state8, KRK_EINVAL, "sha256_resume: state is NULL");
    KRK_CHECK(n == 0 || data_dev, KRK_EINVAL, "sha256_resume: data is NULL");
    KRK_CHECK(absorbed % 64 == 0, KRK_EINVAL, "sha256_resume: absorbed bytes not a multiple of 64");
    KRK_CHECK(final || n % 64 == 0, KRK_EINVAL, "sha256_resume: a non-final run must be whole 64-byte blocks");
    KRK_CHECK(!final || digest32, KRK_EINVAL, "sha256_resume: digest is NULL");
    KRK_DEVICE(D);
    if (!stream)  // the caller has waited for the bytes: an event on an idle stream would still
                  // queue behind other streams' packets in its shared hardware queue (ms each)
        return resume_on_host(D, state8, absorbed, data_dev, n, final != 0, digest32, nullptr);
    hipEvent_t ready;
    KRK_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    int r = KRK_OK;
    if (hipEventRecord(ready, static_cast<hipStream_t>(stream)) != hipSuccess) {
        set_error(KRK_EHIP, "sha256_resume: event record failed");
        r = KRK_EHIP;
    }
    if (!r) r = resume_on_host(D, state8, absorbed, data_dev, n, final != 0, digest32, ready);
    hipEventDestroy(ready);
    return r;
}

int krk_sha256_resume_host(uint32_t* state8, uint64_t absorbed, const uint8_t* data_host, uint64_t n, int final,
                           uint8_t* digest32) {
    KRK_CHECK(state8, KRK_EINVAL, "sha256_resume: state is NULL");
    KRK_CHECK(n == 0 || data_host, KRK_EINVAL, "sha256_resume: data is NULL");
    KRK_CHECK(absorbed % 64 == 0, KRK_EINVAL, "sha256_resume: absorbed bytes not a multiple of 64");
    KRK_CHECK(final || n % 64 == 0, KRK_EINVAL, "sha256_resume: a non-final run must be whole 64-byte blocks");
    KRK_CHECK(!final || digest32, KRK_EINVAL, "sha256_resume: digest is NULL");
    const auto t = std::chrono::steady_clock::now();
    if (!final)
        host_sha256_blocks(state8, data_host, n / 64);
    else
        host_sha256_final(state8, absorbed, data_host, n, digest32);
    t_resume_hash += std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count();
    return KRK_OK;
}

int krk_sha256_resume_stats(double* copy_wait_s, double* hash_s) {
    if (copy_wait_s) *copy_wait_s = t_resume_wait;
    if (hash_s) *hash_s = t_resume_hash;
    return KRK_OK;
}
int krk_sha256_resume_stats2(double* issue_s, double* ready_s) {
    if (issue_s) *issue_s = t_resume_issue;
    if (ready_s) *ready_s = t_resume_ready;
    return KRK_OK;
}

int krk_sha_tail_plan(const uint64_t* lengths, uint64_t n, int threads, uint32_t* host_idx, uint64_t* start,
                      uint64_t* n_out, double* end_s, double* gpu_s) {
    KRK_CHECK(lengths && host_idx && start && n_out, KRK_EINVAL, "sha_tail_plan: null argument");
    KRK_CHECK(threads >= 0, KRK_EINVAL, "sha_tail_plan: threads < 0");
    int drc = KRK_OK;
    Device* D = device(&drc);  // none: the override or the nominal rates
    const TailPlan tp = tail_plan(lengths, n, threads, planner_rates(D));
    *n_out = tp.idx.size();
    for (size_t k = 0; k < tp.idx.size(); ++k) {
        host_idx[k] = tp.idx[k];
        start[k] = tp.start[k];
    }
    if (end_s) *end_s = tp.end_s;
    if (gpu_s) *gpu_s = tp.gpu_s;
    return KRK_OK;
}

int krk_sha_offload_plan(const uint64_t* lengths, uint64_t n, int threads, int cus, uint32_t* host_idx,
                         uint64_t* n_host, double* gpu_seconds_out, double* host_seconds_out) {
    return krk_host_offload_plan(lengths, n, threads, cus, KRK_OFFLOAD_DEVICE, host_idx, n_host, gpu_seconds_out,
                                 host_seconds_out);
}

int krk_host_cpu_budget(int* cpus, int* node_cpus, char* source, uint32_t cap) {
    const CpuBudget& b = cpu_budget();
    if (cpus) *cpus = b.cpus;
    if (node_cpus) *node_cpus = b.node;
    if (source && cap) snprintf(source, cap, "%s", b.source);
    return KRK_OK;
}

}  // extern "C"
