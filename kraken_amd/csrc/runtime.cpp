// runtime.cpp -- the C ABI (include/kraken_hip.h): device contexts, work
// descriptor builders, pinned staging pipelines and kernel launches.
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <optional>
#include <unistd.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "runtime.hpp"
#include "staging.hpp"

namespace krk {

thread_local std::string t_err;
thread_local int t_dev = 0;

void set_error(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    // A HIP failure the library reports is consumed here: left pending on the thread, the
    // next launch would report it again as an unchecked earlier error (launch_precheck).
    if (code == KRK_EHIP || code == KRK_ENOMEM) (void)hipGetLastError();
}

void engine_teardown(Device& D);                 // engine.cpp
void owner_tables_teardown(Device& D);           // below
void set_device_set_from_mask(uint64_t mask);    // multidev.cpp

// Everything a device context holds: streams, tables, scratch cache, pinned
// upload slots, staging windows, the shard-key table.  Only for krk_shutdown.
static void teardown_device(Device& D) {
    hipSetDevice(D.id);
    for (hipStream_t s : {D.s_main, D.s_a, D.s_b})
        if (s) hipStreamSynchronize(s);
    delete D.staging;  // drains its windows' events
    D.staging = nullptr;
    offload_teardown(D);
    owner_tables_teardown(D);  // before the scratch cache: the tables' blocks go back to it
    {
        std::lock_guard<std::mutex> g(D.cache.mu);
        for (auto& kv : D.cache.idle) {
            hipFree(kv.second.p);
            if (kv.second.ev) hipEventDestroy(kv.second.ev);
        }
        D.cache.idle.clear();
        for (auto& kv : D.cache.live) {  // none unless a call is in flight (contract)
            hipFree(kv.second.p);
            if (kv.second.ev) hipEventDestroy(kv.second.ev);
        }
        D.cache.live.clear();
    }
    for (auto& R : D.rings)
        for (PinnedSlot& P : R->slot) {
            if (P.ev) hipEventSynchronize(P.ev), hipEventDestroy(P.ev);
            if (P.p) hipHostFree(P.p);
        }
    D.rings.clear();
    D.ring_of.clear();
    for (void* p : D.retired_pinned) hipHostFree(p);
    D.retired_pinned.clear();
    for (void* p : {(void*)D.shard_kb, (void*)D.shard_koff, (void*)D.shard_bad, (void*)D.d_tabs})
        if (p) hipFree(p);
    for (hipStream_t s : {D.s_main, D.s_a, D.s_b})
        if (s) hipStreamDestroy(s);
}

}  // namespace krk

using namespace krk;

// ======================================================================= C ABI
extern "C" {

const char* krk_version(void) { return "kraken_amd 0.1 (gfx950)"; }
const char* krk_last_error(void) { return t_err.c_str(); }

int krk_device_count(int* n) {
    KRK_CHECK(n, KRK_EINVAL, "n is NULL");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    int good = 0;
    for (int i = 0; i < c; ++i) {
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, i) == hipSuccess && strncmp(p.gcnArchName, "gfx950", 6) == 0) ++good;
    }
    *n = good;
    return KRK_OK;
}

int krk_init(uint64_t dev_mask) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_error(KRK_ENODEV, "no HIP device visible");
        return KRK_ENODEV;
    }
    const int saved = t_dev;
    int r = KRK_OK;
    for (int i = 0; i < n && i < 64 && !r; ++i) {
        if (dev_mask ? !((dev_mask >> i) & 1) : i != saved) continue;
        t_dev = i;
        int rc = KRK_OK;
        Device* D = device(&rc);
        if (!D) r = rc;
        // the planners' rates, measured now while the library has no work on the device
        // (a first use under load would fix a contended split for the process)
        else if (!KRK_OP_ENV("KRK_NO_CALIBRATE")) r = calibrate_device(D);
    }
    for (int i = n; i < 64 && !r; ++i)
        if ((dev_mask >> i) & 1) {
            set_error(KRK_ENODEV, "device %d out of range (%d visible)", i, n);
            r = KRK_ENODEV;
        }
    t_dev = saved;
    if (!r) {
        int rc = KRK_OK;
        device(&rc);  // restore the calling thread's current device
        if (dev_mask) set_device_set_from_mask(dev_mask);  // the multi-device entry points' devices
    }
    return r;
}

int krk_shutdown(void) {
    std::lock_guard<std::mutex> g(g_dmu);
    for (auto& D : g_devs)
        if (D) {
            engine_teardown(*D);  // dispatcher threads first: they launch on this context
            teardown_device(*D);
            D.reset();
        }
    return KRK_OK;
}

int krk_set_device(int dev) {
    t_dev = dev;
    KRK_DEVICE(D);
    (void)D;
    return KRK_OK;
}

int krk_synchronize(void) {
    KRK_DEVICE(D);
    KRK_HIP(hipStreamSynchronize(D->s_main));
    KRK_HIP(hipStreamSynchronize(D->s_a));
    KRK_HIP(hipStreamSynchronize(D->s_b));
    return KRK_OK;
}

uint64_t krk_num_pieces(uint64_t length, int64_t piece_length) {
    if (piece_length <= 0) return 0;
    return (length + (uint64_t)piece_length - 1) / (uint64_t)piece_length;
}

int krk_piece_sums_dev(const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_dev, void* stream) {
    KRK_DEVICE(D);
    return piece_sums_dev(D, blobs, n_blobs, sums_dev, pick(D, stream));
}

// The chains of a device-resident batch host threads finish (krk_set_sha_host_offload; empty
// when it is off or would not shorten the batch), and a per-blob mark: whole blobs
// (`start` empty: offload_plan), or the tails of chains the GPU starts (tail_plan) when those
// end the batch sooner -- the model's ends compared, KRK_SHA_TAIL=0 keeps whole blobs only.
struct HostShare {
    std::vector<uint32_t> idx;
    std::vector<uint64_t> start;  // tail handoff: the GPU's prefix of chain idx[k]
};
struct TailStats {
    uint64_t chains = 0, gpu_prefix_bytes = 0;
};
static thread_local TailStats t_last_tail;  // krk_sha_last_tail
static HostShare offload_split(Device* D, const uint64_t* lens, uint64_t n, std::vector<char>& on_host) {
    on_host.assign(n, 0);
    HostShare hs;
    const int T = offload_threads();
    if (T <= 0 || n == 0) return hs;
    const Rates R = planner_rates(D);
    double g = 0, h = 0;
    hs.idx = offload_plan(lens, n, T, R, &g, &h);
    static const bool tails = !KRK_AB_ENV("KRK_SHA_TAIL") || atoi(KRK_AB_ENV("KRK_SHA_TAIL")) != 0;
    if (tails) {
        const double whole = std::max(g, h);
        TailPlan tp = tail_plan(lens, n, T, R);
        if (!tp.idx.empty() && tp.end_s < 0.95 * whole) {
            hs.idx = std::move(tp.idx);
            hs.start = std::move(tp.start);
        }
    }
    for (uint32_t i : hs.idx) on_host[i] = 1;
    t_last_tail = {hs.start.empty() ? 0 : hs.idx.size(), 0};
    for (uint64_t y : hs.start) t_last_tail.gpu_prefix_bytes += y;
    return hs;
}

// The GPU's side of a batch: whole chains, and the prefixes of the chains whose tails host
// threads finish -- those write their midstates to `note` (page-locked, coherent host memory
// the kernel stores to over PCIe) instead of a digest.
static void host_share_jobs(const HostShare& hs, const uint8_t* const* ptrs, std::vector<ShaJob>& jobs) {
    for (size_t k = 0; k < hs.start.size(); ++k)
        if (hs.start[k]) {
            ShaJob j = full_job(ptrs[hs.idx[k]], hs.start[k], hs.idx[k]);
            j.flags = 0;  // a midstate, not a digest
            jobs.push_back(j);
        }
}

// Page-locked note for the midstates of n chains, every word kTailSentinel; its device
// address in *dev.
static int tail_note(uint64_t n, uint32_t** host, uint32_t** dev) {
    *host = *dev = nullptr;
    KRK_HIP(hipHostMalloc(reinterpret_cast<void**>(host), std::max<uint64_t>(n, 1) * 32,
                          hipHostMallocMapped | hipHostMallocCoherent));
    memset(*host, 0xFF, std::max<uint64_t>(n, 1) * 32);
    static_assert(kTailSentinel == 0xFFFFFFFFu, "the note's fill");
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, *host, 0) != hipSuccess) {
        hipHostFree(*host);
        *host = nullptr;
        KRK_CHECK(false, KRK_EHIP, "sha256 tail handoff: no device address for the midstate note");
    }
    *dev = static_cast<uint32_t*>(d);
    return KRK_OK;
}

// Hash the host threads' chains (their D2H waits for `ready`; tails wait for their midstates
// in `note`, written by the launch `gpu_done` follows) and store the digests into digests_dev
// on stream s.
static int offload_run(Device* D, const HostShare& hs, const uint8_t* const* ptrs, const uint64_t* lens,
                       hipEvent_t ready, uint8_t* digests_dev, hipStream_t s, const uint32_t* note = nullptr,
                       hipEvent_t gpu_done = nullptr) {
    const std::vector<uint32_t>& host = hs.idx;
    std::vector<const uint8_t*> p(host.size());
    std::vector<uint64_t> l(host.size());
    for (size_t j = 0; j < host.size(); ++j) {
        p[j] = ptrs[host[j]];
        l[j] = lens[host[j]];
    }
    std::vector<uint8_t> dig(32 * host.size());
    TailSrc tail{note, host.data(), hs.start.data(), gpu_done};
    int r = offload_hash(D, p, l, offload_threads(), ready, dig.data(), hs.start.empty() ? nullptr : &tail);
    return r ? r : offload_store(D, host, dig.data(), digests_dev, s);
}

// A batch's SHA-256 launch plus its host share, in two steps so that other launches (the
// CRC) can be queued between them: launch() queues the GPU part on `s` (whole chains, and
// the prefixes of the tails with their midstate note); finish() runs the host threads'
// chains beside it and returns once their digests are queued into digests_dev on `s_out`
// (with tails: once the launch has ended too, so the note can go).
struct ShaHostShare {
    const HostShare& hs;
    uint32_t *note = nullptr, *note_dev = nullptr;
    hipEvent_t done = nullptr;
    int r = KRK_OK;
    explicit ShaHostShare(const HostShare& h) : hs(h) {}
    ShaHostShare(const ShaHostShare&) = delete;
    ShaHostShare& operator=(const ShaHostShare&) = delete;
    ~ShaHostShare() { release(nullptr); }
    void release(hipStream_t s) {
        if (note) {  // the launch wrote the note: it goes only once the launch has ended
            if (done) hipEventSynchronize(done);
            else if (s) hipStreamSynchronize(s);
            hipHostFree(note);
            note = nullptr;
        }
        if (done) hipEventDestroy(done);
        done = nullptr;
    }
    int launch(Device* D, const std::vector<char>& on_host, const uint8_t* const* ptrs, const uint64_t* lens,
               uint64_t n, uint8_t* digests_dev, hipStream_t s) {
        std::vector<ShaJob> jobs;
        jobs.reserve(n);
        for (uint64_t i = 0; i < n; ++i)
            if (!on_host[i]) jobs.push_back(full_job(ptrs[i], lens[i], (uint32_t)i));
        const bool tails = !hs.start.empty();
        if (tails) {
            host_share_jobs(hs, ptrs, jobs);
            if ((r = tail_note(n, &note, &note_dev))) return r;
            if (hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) {
                done = nullptr;
                set_error(KRK_EHIP, "sha256 tail handoff: event");
                return r = KRK_EHIP;
            }
        }
        if ((r = run_jobs(D, jobs, digests_dev, note_dev, s))) return r;
        if (tails && hipEventRecord(done, s) != hipSuccess) {
            set_error(KRK_EHIP, "sha256 tail handoff: event record");
            return r = KRK_EHIP;
        }
        return r;
    }
    int finish(Device* D, const uint8_t* const* ptrs, const uint64_t* lens, hipEvent_t ready, uint8_t* digests_dev,
               hipStream_t s, hipStream_t s_out) {
        if (!r && !hs.idx.empty()) r = offload_run(D, hs, ptrs, lens, ready, digests_dev, s_out, note, done);
        release(s);
        return r;
    }
};

int krk_sha_last_tail(uint64_t* chains, uint64_t* gpu_prefix_bytes) {
    if (chains) *chains = t_last_tail.chains;
    if (gpu_prefix_bytes) *gpu_prefix_bytes = t_last_tail.gpu_prefix_bytes;
    return KRK_OK;
}

int krk_sha256_dev(const uint8_t* const* data_dev, const uint64_t* lengths, uint64_t n, uint8_t* digests_dev,
                   void* stream) {
    KRK_DEVICE(D);
    if (!n) return KRK_OK;
    KRK_CHECK(data_dev && lengths && digests_dev, KRK_EINVAL, "sha256_dev: null argument");
    hipStream_t s = pick(D, stream);
    std::vector<char> on_host;
    const HostShare hs = offload_split(D, lengths, n, on_host);
    if (hs.idx.empty()) {
        std::vector<ShaJob> jobs;
        jobs.reserve(n);
        for (uint64_t i = 0; i < n; ++i) jobs.push_back(full_job(data_dev[i], lengths[i], (uint32_t)i));
        return run_jobs(D, jobs, digests_dev, nullptr, s);
    }
    hipEvent_t ready;
    KRK_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    int r = KRK_OK;
    if (hipEventRecord(ready, s) != hipSuccess) {
        set_error(KRK_EHIP, "sha256_dev: event record failed");
        r = KRK_EHIP;
    }
    if (!r) {
        ShaHostShare sh(hs);
        sh.launch(D, on_host, data_dev, lengths, n, digests_dev, s);  // the GPU part runs while the host hashes
        r = sh.finish(D, data_dev, lengths, ready, digests_dev, s, s);
    }
    hipEventDestroy(ready);
    return r;
}

int krk_sha256_dev_on_host(const uint8_t* const* data_dev, const uint64_t* lengths, uint64_t n, int threads,
                           void* stream, uint8_t* digests_host) {
    KRK_DEVICE(D);
    if (!n) return KRK_OK;
    KRK_CHECK(data_dev && lengths && digests_host, KRK_EINVAL, "sha256_dev_on_host: null argument");
    hipStream_t s = pick(D, stream);
    hipEvent_t ready;
    KRK_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
    int r = KRK_OK;
    if (hipEventRecord(ready, s) != hipSuccess) {
        set_error(KRK_EHIP, "sha256_dev_on_host: event record failed");
        r = KRK_EHIP;
    }
    if (!r) {
        const std::vector<const uint8_t*> p(data_dev, data_dev + n);
        const std::vector<uint64_t> l(lengths, lengths + n);
        r = offload_hash(D, p, l, threads > 0 ? threads : host_threads_for_call(), ready, digests_host);
    }
    hipEventDestroy(ready);
    return r;
}

int krk_metainfo_batch_dev(const krk_blob* blobs, uint64_t n_blobs, const char* names, const uint64_t* name_off,
                           uint32_t* sums_dev, uint32_t* sums_host, uint8_t* info_hash20, void* stream) {
    KRK_DEVICE(D);
    int r = validate_blobs(blobs, n_blobs);
    if (r) return r;
    if (!n_blobs) return KRK_OK;
    KRK_CHECK(sums_dev && sums_host && info_hash20 && name_off, KRK_EINVAL, "metainfo_batch_dev: null argument");
    hipStream_t s = pick(D, stream);
    // Groups of about equal bytes, run back to back on `s`; the host hashes group g
    // while the device runs groups g+1.. (one event per group).
    std::vector<int64_t> pl(n_blobs), ln(n_blobs);
    std::vector<uint64_t> so(n_blobs), ns(n_blobs);
    uint64_t total = 0;
    for (uint64_t i = 0; i < n_blobs; ++i) {
        pl[i] = blobs[i].piece_length;
        ln[i] = (int64_t)blobs[i].length;
        so[i] = blobs[i].sums_offset;
        ns[i] = krk_num_pieces(blobs[i].length, blobs[i].piece_length);
        total += blobs[i].length;
    }
    // Four groups (KRK_REGEN_GROUPS): C5 regen 9.84-9.90 ms a step against 10.14-10.16
    // with eight (each launch's ramp and tail cost more than the InfoHash overlap buys) and
    // 9.70-10.07 with one (profiles/r03/regen_groups_ab.txt).
    static const uint64_t kGroups = [] {
        const char* g = KRK_AB_ENV("KRK_REGEN_GROUPS");
        return (uint64_t)std::max(1, g ? atoi(g) : 4);
    }();
    const uint64_t G = std::min<uint64_t>(n_blobs, kGroups);
    // The host's InfoHash of the last group is the only host work not hidden behind a later
    // group's kernel, so that group is small: 4 % of the bytes (KRK_REGEN_TAIL; <= 0 or >= 1:
    // equal groups), the others sharing the rest equally.  C5 regen 5.10-5.24 TB/s with equal
    // groups, 5.44-5.58 with a 4 % tail, 5.35-5.41 with 2 % (profiles/r03/regen_tail_ab.txt).
    static const double kTail = [] {
        const char* t = KRK_AB_ENV("KRK_REGEN_TAIL");
        return t ? atof(t) : 0.04;
    }();
    const double tail = (kTail > 0 && kTail < 1 && G > 1) ? kTail : 1.0 / (double)G;
    std::vector<uint64_t> cut{0};
    for (uint64_t i = 0, acc = 0; i < n_blobs && cut.size() < G; ++i) {
        acc += blobs[i].length;
        const double want = G > 1 ? (1.0 - tail) * (double)cut.size() / (double)(G - 1) : 1.0;
        if ((double)acc >= (double)total * want && i + 1 < n_blobs) cut.push_back(i + 1);
    }
    cut.push_back(n_blobs);
    const size_t ng = cut.size() - 1;
    std::vector<hipEvent_t> ev(ng, nullptr);
    // sums copies on one of the context's other non-blocking streams (creating a stream
    // per call costs milliseconds on ROCm)
    hipStream_t cs = s == D->s_b ? D->s_a : D->s_b;
    size_t launched = 0;
    for (size_t g = 0; g < ng && !r; ++g) {
        if (hipEventCreateWithFlags(&ev[g], hipEventDisableTiming) != hipSuccess) {
            set_error(KRK_EHIP, "metainfo_batch_dev: event create");
            r = KRK_EHIP;
            break;
        }
        r = piece_sums_dev(D, blobs + cut[g], cut[g + 1] - cut[g], sums_dev, s);
        if (!r && hipEventRecord(ev[g], s) != hipSuccess) {
            set_error(KRK_EHIP, "metainfo_batch_dev: event record");
            r = KRK_EHIP;
        }
        if (!r) ++launched;
    }
    for (size_t g = 0; g < launched; ++g) {
        if (hipEventSynchronize(ev[g]) != hipSuccess) {
            if (!r) { set_error(KRK_EHIP, "metainfo_batch_dev: kernel failed"); r = KRK_EHIP; }
            continue;
        }
        if (r) continue;  // keep draining the launched groups before returning
        uint64_t lo = UINT64_MAX, hi = 0;
        for (uint64_t i = cut[g]; i < cut[g + 1]; ++i)
            if (ns[i]) { lo = std::min(lo, so[i]); hi = std::max(hi, so[i] + ns[i]); }
        if (hi > lo) {
            if (hipMemcpyAsync(sums_host + lo, sums_dev + lo, (hi - lo) * 4, hipMemcpyDeviceToHost, cs) != hipSuccess ||
                hipStreamSynchronize(cs) != hipSuccess) {
                set_error(KRK_EHIP, "metainfo_batch_dev: sums copy");
                r = KRK_EHIP;
                continue;
            }
        }
        const uint64_t a = cut[g], m = cut[g + 1] - cut[g];
        r = krk_info_hash_batch(pl.data() + a, sums_host, so.data() + a, ns.data() + a, names, name_off + a,
                                ln.data() + a, m, info_hash20 + 20 * a);
    }
    if (hipStreamSynchronize(s) != hipSuccess && !r) { set_error(KRK_EHIP, "metainfo_batch_dev: sync"); r = KRK_EHIP; }
    for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
    return r;
}

int krk_metainfo_digest_dev(const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_dev, uint8_t* digests_dev,
                            void* stream) {
    KRK_DEVICE(D);
    int r = validate_blobs(blobs, n_blobs);
    if (r) return r;
    if (!n_blobs) return KRK_OK;
    KRK_CHECK(digests_dev, KRK_EINVAL, "digests_dev is NULL");
    hipStream_t s = pick(D, stream);
    hipEvent_t fork, j1, j2;
    KRK_HIP(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    KRK_HIP(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
    KRK_HIP(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
    KRK_HIP(hipEventRecord(fork, s));
    KRK_HIP(hipStreamWaitEvent(D->s_a, fork, 0));
    KRK_HIP(hipStreamWaitEvent(D->s_b, fork, 0));
    // The longest chains may go to host threads (krk_set_sha_host_offload), off by default.
    std::vector<uint64_t> lens(n_blobs);
    std::vector<const uint8_t*> ptrs(n_blobs);
    for (uint64_t i = 0; i < n_blobs; ++i) {
        lens[i] = blobs[i].length;
        ptrs[i] = blobs[i].data;
    }
    std::vector<char> on_host;
    const HostShare hs = offload_split(D, lens.data(), n_blobs, on_host);
    if (hs.idx.empty()) {
        // SHA first: it is the long pole; the CRC kernel fills the rest of the chip.
        std::vector<ShaJob> jobs;
        jobs.reserve(n_blobs);
        for (uint64_t i = 0; i < n_blobs; ++i) jobs.push_back(full_job(blobs[i].data, blobs[i].length, (uint32_t)i));
        r = run_jobs(D, jobs, digests_dev, nullptr, D->s_a);
        if (!r) r = piece_sums_dev(D, blobs, n_blobs, sums_dev, D->s_b);
        hipEventRecord(j1, D->s_a);
        hipEventRecord(j2, D->s_b);
        hipStreamWaitEvent(s, j1, 0);
        hipStreamWaitEvent(s, j2, 0);
    } else {
        // SHA first here too (the long pole), then the CRC, then the host share, which
        // returns once the host is done
        ShaHostShare sh(hs);
        r = sh.launch(D, on_host, ptrs.data(), lens.data(), n_blobs, digests_dev, D->s_a);
        if (!r) r = piece_sums_dev(D, blobs, n_blobs, sums_dev, D->s_b);
        hipEventRecord(j2, D->s_b);
        hipStreamWaitEvent(s, j2, 0);
        const int rf = sh.finish(D, ptrs.data(), lens.data(), fork, digests_dev, D->s_a, s);
        if (!r) r = rf;
        hipEventRecord(j1, D->s_a);
        hipStreamWaitEvent(s, j1, 0);
    }
    hipEventDestroy(fork);
    hipEventDestroy(j1);
    hipEventDestroy(j2);
    return r;
}

// The GPU pass of krk_piece_sums_host over host blobs: windows of their bytes go up
// (pageable bytes through the pinned staging windows; `direct`: the caller's bytes are
// pinned and DMA'd straight into the device window) and the CRC kernel runs on each.
static int piece_sums_host_gpu(Device* D, const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_host,
                               bool direct) {
    int r = KRK_OK;
    uint64_t lo, hi;
    sums_span(blobs, n_blobs, &lo, &hi);
    if (hi == lo) return KRK_OK;
    KRK_CHECK(sums_host, KRK_EINVAL, "sums_host is NULL");
    uint32_t* d_sums = nullptr;
    DevMem mem;
    KRK_HIP(mem.alloc(&d_sums, hi * 4));
    KRK_HIP(hipMemset(d_sums, 0, hi * 4));
    const size_t W = window_bytes();
    StagingLease lease;
    r = lease_staging(D, W, lease);
    if (r) return r;
    Pipeline& pl = *lease.p;
    hipStream_t cp = D->s_a, ks = D->s_b;
    ItemBuilder B;
    int k = 0;
    uint64_t bi = 0, boff = 0;
    bool gather_ok = direct;  // every blob read at its host address
    MappedAtHost mapped;
    for (uint64_t i = 0; gather_ok && i < n_blobs; ++i) gather_ok = mapped(blobs[i].data, blobs[i].length);
    while (!r && bi < n_blobs) {
        r = pl.acquire(k);
        if (r) break;
        Window& w = pl.w[k];
        size_t fill = 0;
        CrcBatch items;
        std::vector<CopyTask> copies;
        while (bi < n_blobs && fill < W) {
            const krk_blob& b = blobs[bi];
            const uint64_t take = std::min<uint64_t>(b.length - boff, W - fill);
            if (take) {
                copies.push_back({w.host + fill, b.data + boff, take});
                B.add(items, reinterpret_cast<uint64_t>(w.dev + fill), boff, boff + take, b.length,
                      (uint64_t)b.piece_length, b.sums_offset);
            }
            fill += take;
            boff += take;
            // keep 16-byte alignment of every run inside the window
            fill = (fill + 15) & ~size_t(15);
            if (boff >= b.length) { ++bi; boff = 0; }
        }
        // pinned bytes go up straight from the caller's pages: a DMA a copy in windows of few
        // copies (many small DMAs cost more than the staging copy, staging.hpp
        // kDirectMaxCalls), else one gather launch that reads them over PCIe (gather.hip)
        const bool dw = direct && copies.size() <= kDirectMaxCalls;
        const bool gw = direct && !dw && gather_ok;
        hipError_t up = hipSuccess;
        if (dw || gw)
            for (CopyTask& c : copies) c.dst = w.dev + (c.dst - w.host);
        if (gw) {
            std::vector<GatherSpan> spans;
            spans.reserve(copies.size());
            for (const CopyTask& c : copies) spans.push_back({c.dst, c.src, c.n});
            r = pl.h2d_gather(D, k, spans, cp);
            if (r) break;
        } else {
            up = dw ? pl.h2d_direct(k, copies, cp) : (par_copy(copies), pl.h2d(k, std::min(fill, W), cp));
        }
        if (up != hipSuccess || hipStreamWaitEvent(ks, w.copied, 0) != hipSuccess) {
            set_error(KRK_EHIP, "piece_sums_host: staging copy failed");
            r = KRK_EHIP;
            break;
        }
        r = run_items(D, items, d_sums, ks);
        if (r) break;
        pl.release(k, 0, ks);
        k = pl.next(k);
    }
    if (!r && hipStreamSynchronize(ks) != hipSuccess) { set_error(KRK_EHIP, "sync failed"); r = KRK_EHIP; }
    if (!r && hipMemcpy(sums_host + lo, d_sums + lo, (hi - lo) * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        set_error(KRK_EHIP, "sums copy-out failed");
        r = KRK_EHIP;
    }
    return r;
}

// krk_piece_sums_host / krk_verify_pieces_host: the reference hashes each received
// piece on the host (lib/torrent/storage/agentstorage/torrent.go:182-193), and one host
// core's PCLMUL CRC (~12 GB/s) is within a few x of what the host link carries to the
// GPU, so the batch is split by bytes, whole pieces at a time, between host threads and
// the GPU pass in proportion to the measured rates (planner_rates):
//  * pinned caller bytes: the GPU side costs no host CPU (DMA straight into the device
//    window), so the GPU takes h2d / (h2d + threads x crc) of the bytes;
//  * pageable bytes: the GPU side needs a host memcpy into pinned staging, so it helps
//    only if a core copies faster than it CRCs; otherwise everything stays on the host.
// Host threads = the CPUs this process may use (affinity and cgroup quota).
struct PieceTask {
    const uint8_t* p;
    uint64_t n;
    uint64_t out;
};

// NUMA-aware hand-out of host CRC tasks (runs of ~8 MiB), opt-in: the node of each task's
// first, middle and last page (move_pages, one call for all of them) and, per claim, the
// node of the CPU the claiming thread runs on; a thread takes the next task of its own node
// and steals from the others once its node has none (KRK_CRC_NUMA=1), and with
// KRK_CRC_NUMA=2, for a batch spread over both sockets' memory, a thread that takes another
// node's task runs it on that node's CPUs (NodeVisit).  Off by default (0 = one plain
// cursor): on the GPU boxes' two-socket hosts, five interleaved A/B runs of the three modes
// (profiles/r05/host_mem_probe_numa.jsonl) moved the spread-buffer case by +33, +8, +14,
// -14, +31 % with visits and left every one-node buffer equal or a few % lower -- inside the
// host's minute-to-minute swing, not a win to ship.
class NodeTasks {
  public:
    // sysfs's CPU lists per node, parsed once: node of each CPU and the CPUs of each node
    struct Topology {
        std::vector<int> node_of_cpu = std::vector<int>(CPU_SETSIZE, 0);
        std::vector<cpu_set_t> cpus;
        Topology() {
            for (int nd = 0; nd < 64; ++nd) {
                FILE* f = fopen(("/sys/devices/system/node/node" + std::to_string(nd) + "/cpulist").c_str(), "r");
                if (!f) break;
                char buf[4096] = {0};
                const size_t got = fread(buf, 1, sizeof buf - 1, f);
                fclose(f);
                buf[got] = 0;
                cpu_set_t set;
                CPU_ZERO(&set);
                for (char* q = buf; *q && *q != '\n';) {  // "0-63,128-191"
                    char* e = nullptr;
                    const long lo = strtol(q, &e, 10);
                    if (e == q) break;
                    long hi = lo;
                    if (*e == '-') hi = strtol(e + 1, &e, 10);
                    for (long c = lo; c <= hi && c < CPU_SETSIZE; ++c) {
                        node_of_cpu[(size_t)c] = nd;
                        CPU_SET((int)c, &set);
                    }
                    q = (*e == ',') ? e + 1 : e;
                }
                cpus.push_back(set);
            }
        }
    };
    static const Topology& topo() {
        static const Topology t;
        return t;
    }
    static int cpu_node(int cpu) { return cpu >= 0 && cpu < CPU_SETSIZE ? topo().node_of_cpu[(size_t)cpu] : 0; }
    // the CPUs of node nd (nullptr when sysfs did not list it)
    static const cpu_set_t* node_cpus(int nd) {
        return nd >= 0 && (size_t)nd < topo().cpus.size() ? &topo().cpus[(size_t)nd] : nullptr;
    }
    // node visits (mode 2) only for a batch spread over nodes: two or more nodes holding at least
    // an eighth of the tasks each.  A batch on one node keeps its threads spread over both
    // sockets (moving all of them to the memory's socket measured 10 % slower).
    bool visits() const {
        if (mode_ < 2) return false;
        std::vector<size_t> on(list_.size(), 0);
        for (int nd : node_)
            if (nd >= 0) ++on[(size_t)nd];
        size_t big = 0;
        for (size_t c : on) big += c * 8 >= node_.size();
        return big >= 2;
    }
    int node_of(size_t task) const { return task < node_.size() ? node_[task] : -1; }
    // tasks' first, middle and last pages -> per-node lists; a task whose three pages are
    // not on one node (interleaved memory) is nobody's: it goes on its first page's list and
    // is never visited.  False when there is one node or the query fails.
    bool build(const std::vector<const void*>& first, const std::vector<const void*>& mid,
               const std::vector<const void*>& last) {
        const char* v = KRK_AB_ENV("KRK_CRC_NUMA");
        mode_ = v ? atoi(v) : 0;
        const size_t n = first.size();
        if (mode_ <= 0 || n < 2) return false;
        std::vector<int> status(3 * n, -1);
        std::vector<void*> pages(3 * n);
        auto page = [](const void* q) { return reinterpret_cast<void*>(reinterpret_cast<uintptr_t>(q) & ~uintptr_t(4095)); };
        for (size_t i = 0; i < n; ++i) {
            pages[3 * i] = page(first[i]);
            pages[3 * i + 1] = page(mid[i]);
            pages[3 * i + 2] = page(last[i]);
        }
        if (syscall(SYS_move_pages, 0, (unsigned long)pages.size(), pages.data(), nullptr, status.data(), 0) != 0)
            return false;
        int nodes = 0;
        for (int st : status) nodes = std::max(nodes, st + 1);
        if (nodes < 2) return false;
        list_.assign((size_t)nodes, {});
        node_.assign(n, -1);
        for (size_t i = 0; i < n; ++i) {
            const int a = status[3 * i], b = status[3 * i + 1], c = status[3 * i + 2];
            if (a >= 0 && a == b && b == c) node_[i] = a;
            list_[(size_t)std::max(0, a)].push_back(i);
        }
        next_ = std::vector<std::atomic<size_t>>(list_.size());
        return true;
    }
    // the next task for a thread on the CPU it runs on now (SIZE_MAX: none left)
    size_t claim() {
        const int home = std::min<int>((int)list_.size() - 1, cpu_node(sched_getcpu()));
        for (size_t k = 0; k < list_.size(); ++k) {
            const size_t nd = ((size_t)home + k) % list_.size();
            if (next_[nd].load(std::memory_order_relaxed) >= list_[nd].size()) continue;
            const size_t i = next_[nd].fetch_add(1);
            if (i < list_[nd].size()) return list_[nd][i];
        }
        return SIZE_MAX;
    }

  private:
    int mode_ = 0;
    std::vector<int> node_;
    std::vector<std::vector<size_t>> list_;
    std::vector<std::atomic<size_t>> next_;
};

// Mode 2 of KRK_CRC_NUMA (the default): a thread that takes a task of another node moves to
// that node's CPUs for the task (within the CPUs it may use) and back afterwards.
struct NodeVisit {
    cpu_set_t old;
    bool moved = false;
    explicit NodeVisit(int nd) {
        if (sched_getaffinity(0, sizeof old, &old) != 0) return;
        const cpu_set_t* on = NodeTasks::node_cpus(nd);
        if (!on) return;
        cpu_set_t to;
        CPU_AND(&to, &old, on);
        if (CPU_COUNT(&to) == 0) return;
        moved = sched_setaffinity(0, sizeof to, &to) == 0;
    }
    ~NodeVisit() {
        if (moved) sched_setaffinity(0, sizeof old, &old);
    }
};

// The pinned-batch split of each device, learned from earlier calls (per device).
//  * frac: the balanced GPU share -- where both sides would have ended together at the
//    rates the last split call measured (-1: none yet; first call: the rates' model, <= 10 %);
//  * r_split / r_host: whole-call throughput (bytes / wall time) of calls at that split and
//    of host-only calls.  The DMA reads share host memory with the CRC threads, so a balanced
//    split can still lose to the host alone (C4's 20 GiB pinned blob on one box: 131 GB/s at
//    the balanced 27 % against 260 host-only; f1verify on another: 282 at 10 % against 228).
//    So the first split call sets up the windows (not a sample), the second measures the
//    split, the next runs host-only, later calls take whichever measured faster, and every
//    16th call re-measures the other one.
struct CrcSplit {
    std::mutex mu;
    double frac = -1, r_split = 0, r_host = 0;
    uint64_t calls = 0;
    bool warm = false;  // a split call has run: the staging windows exist (the first pays their set-up)
    bool use_split() const { return r_host <= 0 || r_split >= r_host; }
};
static CrcSplit g_crc_split[kMaxDevs];
static CrcSplit& crc_split_of(int dev) { return g_crc_split[(dev >= 0 && dev < kMaxDevs) ? dev : 0]; }
static thread_local uint64_t t_split_gpu = 0, t_split_host = 0;

int krk_piece_sums_host(const krk_blob* blobs, uint64_t n_blobs, uint32_t* sums_host) {
    int r = validate_blobs(blobs, n_blobs);
    if (r) return r;
    uint64_t lo, hi;
    sums_span(blobs, n_blobs, &lo, &hi);
    if (hi == lo) return KRK_OK;
    KRK_CHECK(sums_host, KRK_EINVAL, "sums_host is NULL");
    // Concurrent callers (the agent's dispatcher verifying from several goroutines) share the
    // CPU budget instead of each starting a full set of threads.
    static std::atomic<int> callers{0};
    struct Caller {
        Caller() { callers.fetch_add(1); }
        ~Caller() { callers.fetch_sub(1); }
    } caller;
    const int T = std::max(1, host_threads_for_call() / std::max(1, callers.load()));
    bool all_pinned = true;
    double bytes = 0;
    for (uint64_t i = 0; i < n_blobs; ++i) {
        bytes += (double)blobs[i].length;
        if (all_pinned && blobs[i].length && !host_pinned(blobs[i].data, blobs[i].length)) all_pinned = false;
    }
    const char* forced = KRK_OP_ENV("KRK_CRC_GPU_FRACTION");
    // Pageable batches stay on the host threads and need no device; pinned (or forced) ones
    // split by the device's rates.
    Device* D = nullptr;
    if (all_pinned || forced) {
        int drc = KRK_OK;
        D = device(&drc);
        if (!D) return drc;
    }
    const Rates R = D ? planner_rates(D) : Rates{};
    // Pinned bytes: the GPU's share starts from the rates' model, capped at 10 %, and is then
    // set from what the previous calls measured (each side's bytes over its own wall time
    // while both ran): the DMA reads share the host's memory with the CRC threads, so the
    // static model overestimates the GPU side (f1verify, same box: 10 % 282 GB/s, 20 % 182,
    // host only 228).  Pageable bytes stay on the host: a copy into pinned staging per byte
    // cost more than the GPU saved (host only 241 GB/s, the model's split 202).
    const double c = R.host_crc, H = T * c;
    double gpu_frac = 0.0;
    CrcSplit& cs = crc_split_of(D ? D->id : 0);
    if (all_pinned && !forced) {
        std::lock_guard<std::mutex> g(cs.mu);
        const uint64_t k = ++cs.calls;
        bool split = cs.r_split <= 0 || (cs.r_host > 0 && cs.use_split());
        if (cs.r_split > 0 && cs.r_host <= 0) split = false;  // the second call: host only
        else if (k % 16 == 0) split = !split;                    // re-measure the other side
        gpu_frac = split ? (cs.frac >= 0 ? cs.frac : std::min(0.10, R.h2d / (R.h2d + H))) : 0.0;
    }
    if (forced) gpu_frac = std::clamp(atof(forced), 0.0, 1.0);
    // Whole pieces to the GPU until its share of the bytes is reached, the rest to the host.
    const double quota = gpu_frac * bytes;
    double gbytes = 0;
    std::vector<krk_blob> gpu;
    std::vector<uint64_t> gpu_dst;  // sums_host index of each GPU blob's first sum
    std::vector<PieceTask> host;
    uint64_t g_sums = 0;
    for (uint64_t i = 0; i < n_blobs; ++i) {
        const krk_blob& b = blobs[i];
        const uint64_t P = (uint64_t)b.piece_length, np = krk_num_pieces(b.length, b.piece_length);
        uint64_t q = 0;  // pieces [0, q) of this blob go to the GPU
        while (q < np && gbytes < quota) {
            gbytes += (double)std::min(P, b.length - q * P);
            ++q;
        }
        if (q) {
            gpu.push_back(krk_blob{b.data, std::min(b.length, q * P), b.piece_length, g_sums});
            gpu_dst.push_back(b.sums_offset);
            g_sums += q;
        }
        for (uint64_t k = q; k < np; ++k) host.push_back({b.data + k * P, std::min(P, b.length - k * P), b.sums_offset + k});
    }
    // The host share on the host pool's idle threads (and this thread once the GPU pass is
    // queued): at most T threads, one per 8 MiB of host bytes (a small share stays on the
    // calling thread).
    const auto t0 = std::chrono::steady_clock::now();
    std::atomic<int64_t> host_end_ns{0};
    std::atomic<size_t> left{host.size()};
    double hbytes_all = 0;
    for (const PieceTask& h : host) hbytes_all += (double)h.n;
    const int TH = (int)std::min<size_t>({(size_t)T, host.size(), (size_t)(hbytes_all / (8 << 20)) + 1});
    // A task is a run of consecutive pieces (~8 MiB): one thread streams through adjacent
    // bytes, which the hardware prefetchers follow (256 KiB tasks handed out one at a time ran
    // C4's host side ~30 % below contiguous spans, profiles/r04/host_mem_probe_lib.jsonl).
    static const double task_bytes = [] {  // KRK_CRC_TASK_KB overrides the run length (A/B)
        const char* v = KRK_AB_ENV("KRK_CRC_TASK_KB");
        return v ? atof(v) * 1024.0 : double(8u << 20);
    }();
    const size_t G = host.empty() ? 1
                                  : std::max<size_t>(1, (size_t)(task_bytes / std::max(1.0, hbytes_all / host.size())));
    const size_t n_tasks = (host.size() + G - 1) / G;
    left.store(n_tasks);
    NodeTasks nt;
    bool numa = false;
    if (n_tasks >= 2) {
        std::vector<const void*> first(n_tasks), mid(n_tasks), last(n_tasks);
        for (size_t t = 0; t < n_tasks; ++t) {
            const size_t j0 = t * G, j1 = std::min(host.size(), (t + 1) * G) - 1;
            first[t] = host[j0].p;
            mid[t] = host[(j0 + j1) / 2].p + host[(j0 + j1) / 2].n / 2;
            last[t] = host[j1].p + (host[j1].n ? host[j1].n - 1 : 0);
        }
        numa = nt.build(first, mid, last);
    }
    const bool visits = numa && nt.visits();
    HostBatch hb(n_tasks, gpu.empty() ? TH - 1 : TH, [&](size_t t) {
        if (numa) {  // every call claims one task: n_tasks calls take them all
            const size_t k = nt.claim();
            if (k != SIZE_MAX) t = k;
        }
        std::optional<NodeVisit> visit;
        if (visits && nt.node_of(t) >= 0 && nt.node_of(t) != NodeTasks::cpu_node(sched_getcpu()))
            visit.emplace(nt.node_of(t));
        for (size_t j = t * G; j < std::min(host.size(), (t + 1) * G); ++j)
            sums_host[host[j].out] = host_crc32_update(0, host[j].p, host[j].n);
        if (left.fetch_sub(1) == 1)  // the last task: the host side's wall time
            host_end_ns.store(
                std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count());
    });
    double gpu_s = 0;
    if (!gpu.empty()) {
        std::vector<uint32_t> gs(g_sums);
        r = piece_sums_host_gpu(D, gpu.data(), gpu.size(), gs.data(), all_pinned);
        gpu_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (!r)
            for (size_t j = 0; j < gpu.size(); ++j) {
                const uint64_t cnt = krk_num_pieces(gpu[j].length, gpu[j].piece_length);
                memcpy(sums_host + gpu_dst[j], gs.data() + gpu[j].sums_offset, cnt * 4);
            }
    }
    hb.join();
    const double hbytes = bytes - gbytes, host_s = host_end_ns.load() * 1e-9;
    t_split_gpu = (uint64_t)gbytes;
    t_split_host = (uint64_t)hbytes;
    const double call_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!r && all_pinned && !forced && bytes >= (128u << 20) && call_s > 0) {
        std::lock_guard<std::mutex> g(cs.mu);
        auto ema = [](double& x, double v) { x = x > 0 ? 0.5 * x + 0.5 * v : v; };
        if (gbytes > 0 && !cs.warm) {
            cs.warm = true;  // not a sample: this call allocated and pinned the windows
        } else if (gbytes > 0) {
            ema(cs.r_split, bytes / call_s);
            if (gbytes >= (64u << 20) && hbytes >= (64u << 20) && gpu_s > 0 && host_s > 0) {
                // the split where both sides would have ended together at the rates just measured
                const double rg = gbytes / gpu_s, rh = hbytes / host_s, want = rg / (rg + rh);
                cs.frac = cs.frac >= 0 ? 0.5 * cs.frac + 0.5 * want : want;
            }
        } else {
            ema(cs.r_host, bytes / call_s);
        }
    }
    return r;
}

int krk_crc_host_split(uint64_t* gpu_bytes, uint64_t* host_bytes, double* gpu_fraction) {
    if (gpu_bytes) *gpu_bytes = t_split_gpu;
    if (host_bytes) *host_bytes = t_split_host;
    if (gpu_fraction) {
        CrcSplit& cs = crc_split_of(t_dev);
        std::lock_guard<std::mutex> g(cs.mu);
        *gpu_fraction = cs.r_host > 0 && !cs.use_split() ? 0.0 : cs.frac;
    }
    return KRK_OK;
}

// The host placement of krk_piece_sums_files: what the reference's Generate does with a
// cache file (lib/metainfogen/generator.go:41-58 -> core.NewMetaInfo over the file reader,
// core/metainfo.go:157-179), spread over the host pool.  Each file is cut into spans of
// whole pieces (~16 MiB); a span's thread preads it in 512 KiB chunks into a buffer of its
// own and folds each chunk into the piece's CRC while the chunk is in cache.  The same
// bytes through the GPU cost the same pread (into a pinned window) plus the host link, so
// where the host's CRC capacity exceeds the link this placement is faster.
static int piece_sums_files_host(const krk_file_blob* files, uint64_t n, uint32_t* sums_host) {
    struct Span {
        uint64_t file, first, pieces;
    };
    std::vector<Span> spans;
    constexpr uint64_t kSpan = 16ull << 20;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t P = (uint64_t)files[i].piece_length, np = krk_num_pieces(files[i].length, files[i].piece_length);
        const uint64_t per = std::max<uint64_t>(1, kSpan / P);
        for (uint64_t k = 0; k < np; k += per) spans.push_back({i, k, std::min(per, np - k)});
    }
    std::mutex emu;
    std::string emsg;
    std::atomic<bool> failed{false};
    auto fail = [&](const std::string& m) {
        std::lock_guard<std::mutex> g(emu);
        if (emsg.empty()) emsg = m;
        failed.store(true);
    };
    const int T = std::max(1, host_threads_for_call());
    // 512 KiB reads: 328 GB/s against 277 at the oracle's 32 KiB, alternated with the oracle
    // on one box (profiles/r06/c5regen_files_chunk_ab.jsonl)
    constexpr size_t kChunk = 512u << 10;
    host_parallel_for(spans.size(), T - 1, [&](size_t s) {
        if (failed.load(std::memory_order_relaxed)) return;
        thread_local std::vector<uint8_t> buf;
        if (buf.size() < kChunk) buf.resize(kChunk);
        const Span& sp = spans[s];
        const krk_file_blob& f = files[sp.file];
        const int fd = open(f.path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) {
            fail(std::string("open ") + f.path + ": " + strerror(errno));
            return;
        }
        const uint64_t P = (uint64_t)f.piece_length;
        for (uint64_t k = sp.first; k < sp.first + sp.pieces; ++k) {
            uint64_t a = k * P;
            const uint64_t e = std::min(f.length, a + P);
            uint32_t c = 0;
            while (a < e) {
                const ssize_t got = pread(fd, buf.data(), std::min<uint64_t>(kChunk, e - a), (off_t)a);
                if (got < 0 && errno == EINTR) continue;
                if (got <= 0) {
                    fail(std::string("read blob: ") + f.path + ": " + (got < 0 ? strerror(errno) : "unexpected EOF"));
                    close(fd);
                    return;
                }
                c = host_crc32_update(c, buf.data(), (size_t)got);
                a += (uint64_t)got;
            }
            sums_host[f.sums_offset + k] = c;
        }
        close(fd);
    });
    if (failed.load()) {
        set_error(KRK_EIO, "%s", emsg.c_str());
        return KRK_EIO;
    }
    return KRK_OK;
}

int krk_piece_sums_files(const krk_file_blob* files, uint64_t n, uint32_t* sums_host) {
    if (!n) return KRK_OK;
    KRK_CHECK(files, KRK_EINVAL, "files is NULL");
    uint64_t lo = ~0ull, hi = 0, bytes = 0;
    for (uint64_t i = 0; i < n; ++i) {
        KRK_CHECK(files[i].path, KRK_EINVAL, "file %llu: path is NULL", (unsigned long long)i);
        KRK_CHECK(files[i].piece_length > 0, KRK_EINVAL, "piece length must be positive");
        const uint64_t np = krk_num_pieces(files[i].length, files[i].piece_length);
        bytes += files[i].length;
        if (np) {
            lo = std::min(lo, files[i].sums_offset);
            hi = std::max(hi, files[i].sums_offset + np);
        }
    }
    // An empty file has no piece to read, but Generate opens it (GetCacheFileReader,
    // lib/metainfogen/generator.go:47-49): a missing or unreadable one fails.
    for (uint64_t i = 0; i < n; ++i)
        if (files[i].length == 0) {
            const int fd = open(files[i].path, O_RDONLY | O_CLOEXEC);
            KRK_CHECK(fd >= 0, KRK_EIO, "open %s: %s", files[i].path, strerror(errno));
            close(fd);
        }
    if (hi == 0) return KRK_OK;
    KRK_CHECK(sums_host, KRK_EINVAL, "sums_host is NULL");
    // CRC placement (krk_set_crc_placement, else the measured crossover; HOST without a device)
    int prc = KRK_OK;
    const int where = resolve_crc_placement(KRK_PLACE_AUTO, &prc);
    if (where < 0) return prc;
    t_split_gpu = where == KRK_PLACE_GPU ? bytes : 0;
    t_split_host = where == KRK_PLACE_GPU ? 0 : bytes;
    if (where != KRK_PLACE_GPU) return piece_sums_files_host(files, n, sums_host);
    KRK_DEVICE(D);
    const bool want_direct = KRK_OP_ENV("KRK_FILE_DIRECT") && atoi(KRK_OP_ENV("KRK_FILE_DIRECT")) > 0;
    uint32_t* d_sums = nullptr;
    DevMem mem;
    KRK_HIP(mem.alloc(&d_sums, hi * 4));
    KRK_HIP(hipMemset(d_sums, 0, hi * 4));
    const size_t W = window_bytes();  // a multiple of 1 MiB
    StagingLease lease;
    int r = lease_staging(D, W, lease);
    Pipeline* pl = lease.p;
    hipStream_t cp = D->s_a, ks = D->s_b;
    ItemBuilder B;
    std::vector<int> fds(n, -1);
    std::vector<char> direct(n, 0);
    auto open_file = [&](uint64_t i) -> int {
        if (fds[i] >= 0) return KRK_OK;
        int fd = -1;
        if (want_direct) {
            fd = open(files[i].path, O_RDONLY | O_DIRECT | O_CLOEXEC);
            direct[i] = fd >= 0;
        }
        if (fd < 0) fd = open(files[i].path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) {
            set_error(KRK_EIO, "open %s: %s", files[i].path, strerror(errno));
            return KRK_EIO;
        }
        fds[i] = fd;
        return KRK_OK;
    };
    int k = 0;
    uint64_t bi = 0, boff = 0;
    while (!r && bi < n) {
        r = pl->acquire(k);
        if (r) break;
        Window& w = pl->w[k];
        size_t fill = 0;
        CrcBatch items;
        std::vector<ReadTask> plain, odirect;
        std::vector<uint64_t> finished;
        while (bi < n && fill < W) {
            const krk_file_blob& f = files[bi];
            const uint64_t take = std::min<uint64_t>(f.length - boff, W - fill);
            if (take) {
                r = open_file(bi);
                if (r) break;
                (direct[bi] ? odirect : plain).push_back({fds[bi], boff, w.host + fill, (size_t)take, (size_t)bi});
                B.add(items, reinterpret_cast<uint64_t>(w.dev + fill), boff, boff + take, f.length,
                      (uint64_t)f.piece_length, f.sums_offset);
            }
            fill += take;
            boff += take;
            fill = (fill + 4095) & ~size_t(4095);  // every file starts page-aligned in the window
            if (boff >= f.length) {
                finished.push_back(bi);
                ++bi;
                boff = 0;
            }
        }
        if (r) break;
        for (int pass = 0; pass < 2 && !r; ++pass) {
            const auto& tasks = pass ? odirect : plain;
            if (tasks.empty()) continue;
            int e = 0;
            const long bad = par_read(tasks, pass == 1, &e);
            if (bad >= 0) {
                const char* path = files[tasks[bad].blob].path;
                if (e) set_error(KRK_EIO, "read blob: %s: %s", path, strerror(e));
                else set_error(KRK_EIO, "read blob: %s: unexpected EOF", path);
                r = KRK_EIO;
            }
        }
        for (uint64_t i : finished) {
            if (fds[i] >= 0) close(fds[i]);
            fds[i] = -1;
        }
        if (r) break;
        if (pl->h2d(k, std::min(fill, W), cp) != hipSuccess || hipStreamWaitEvent(ks, w.copied, 0) != hipSuccess) {
            set_error(KRK_EHIP, "piece_sums_files: staging copy failed");
            r = KRK_EHIP;
            break;
        }
        r = run_items(D, items, d_sums, ks);
        if (r) break;
        pl->release(k, 0, ks);
        k = pl->next(k);
    }
    for (int fd : fds)
        if (fd >= 0) close(fd);
    if (hipStreamSynchronize(ks) != hipSuccess && !r) { set_error(KRK_EHIP, "sync failed"); r = KRK_EHIP; }
    if (!r && hipMemcpy(sums_host + lo, d_sums + lo, (hi - lo) * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        set_error(KRK_EHIP, "sums copy-out failed");
        r = KRK_EHIP;
    }
    return r;
}

// crc_only: chunks of one blob may repeat (their CRCs XOR into the sums independently); a
// SHA-256 step takes at most one chunk a blob slot (one midstate each).
static int validate_chunks(const krk_chunk* c, uint64_t n, bool crc_only = false) {
    KRK_CHECK(n == 0 || c, KRK_EINVAL, "chunks is NULL");
    std::unordered_map<uint64_t, uint64_t> seen;
    seen.reserve(n);
    for (uint64_t i = 0; i < n; ++i) {
        KRK_CHECK(crc_only || seen.emplace(c[i].blob, i).second, KRK_EINVAL, "blob slot %llu appears twice in one call",
                  (unsigned long long)c[i].blob);
        KRK_CHECK(c[i].piece_length > 0, KRK_EINVAL, "piece length must be positive");
        KRK_CHECK(c[i].length == 0 || c[i].data, KRK_EINVAL, "chunk %llu: data is NULL", (unsigned long long)i);
        KRK_CHECK(c[i].offset + c[i].length <= c[i].blob_length, KRK_ERANGE, "chunk %llu runs past its blob",
                  (unsigned long long)i);
        KRK_CHECK(c[i].offset % 64 == 0, KRK_EINVAL, "chunk %llu: offset is not a multiple of 64",
                  (unsigned long long)i);
        KRK_CHECK(c[i].length % 64 == 0 || c[i].offset + c[i].length == c[i].blob_length, KRK_EINVAL,
                  "chunk %llu: only a blob's last chunk may be a partial block", (unsigned long long)i);
        KRK_CHECK(c[i].blob <= 0xFFFFFFFFull, KRK_EINVAL, "blob slot exceeds 2^32");
        KRK_CHECK(c[i].sums_offset + krk_num_pieces(c[i].blob_length, c[i].piece_length) <= 0xFFFFFFFFull,
                  KRK_EINVAL, "sums index exceeds 2^32 in one call");
    }
    return KRK_OK;
}

// One window step over device chunks: SHA jobs on D->s_a, CRC items on D->s_b, both
// forked from and joined back into s.  With the caller's SHA stream `ks`, the CRC items run
// on s itself: a caller that keeps its window streams at high priority (the C3 tail
// handoff, kraken_amd/windowed.py) then leaves no fork / join barrier of a window on the
// library's normal-priority streams, whose hardware queues its copy threads share -- a
// barrier waiting for a window's ~70 ms SHA launch blocks every packet behind it there.
//
// crc_after_sha (with ks): the CRC items are queued on s only once the SHA-256 launch has
// ended.  A launch on a high-priority queue whose workgroups wait for CUs (the CRC's 144 KiB
// of LDS, with a window's SHA workgroups holding every CU) keeps the dispatcher from the
// normal-priority queues meanwhile: device-to-host copies of other streams stall for the
// whole window (tools/tail_probe.py, profiles/r06/tail_probe.jsonl: 36 -> 0.18 GB/s).
static int chunks_step(Device* D, const krk_chunk* c, uint64_t n, uint32_t* state_dev, uint32_t* sums_dev,
                       uint8_t* digests_dev, hipStream_t s, ItemBuilder& B, hipStream_t ks = nullptr,
                       bool crc_after_sha = false) {
    const hipStream_t kc = ks ? s : D->s_b;
    if (!ks) ks = D->s_a;
    std::vector<ShaJob> jobs(n);
    CrcBatch items;
    for (uint64_t i = 0; i < n; ++i) {
        ShaJob& j = jobs[i];
        j = ShaJob{};
        j.ptr = reinterpret_cast<uint64_t>(c[i].data);
        j.len = c[i].length;
        j.prefix = c[i].offset;
        j.out = (uint32_t)c[i].blob;
        j.flags = (c[i].offset + c[i].length == c[i].blob_length ? kShaFinal : 0) | (c[i].offset ? kShaFromState : 0);
        memcpy(j.h, kIV, sizeof kIV);
        if (c[i].length)
            B.add(items, j.ptr, c[i].offset, c[i].offset + c[i].length, c[i].blob_length,
                  (uint64_t)c[i].piece_length, c[i].sums_offset);
    }
    hipEvent_t fork, j1, j2;
    KRK_HIP(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    KRK_HIP(hipEventCreateWithFlags(&j1, hipEventDisableTiming));
    KRK_HIP(hipEventCreateWithFlags(&j2, hipEventDisableTiming));
    KRK_HIP(hipEventRecord(fork, s));
    KRK_HIP(hipStreamWaitEvent(ks, fork, 0));
    if (kc != s) KRK_HIP(hipStreamWaitEvent(kc, fork, 0));
    int r = run_jobs(D, jobs, digests_dev, state_dev, ks);
    hipEventRecord(j1, ks);
    if (crc_after_sha && kc == s) {
        hipStreamWaitEvent(s, j1, 0);
        if (!r) r = run_items(D, items, sums_dev, kc);
    } else {
        if (!r) r = run_items(D, items, sums_dev, kc);
        hipStreamWaitEvent(s, j1, 0);
        if (kc != s) {
            hipEventRecord(j2, kc);
            hipStreamWaitEvent(s, j2, 0);
        }
    }
    hipEventDestroy(fork);
    hipEventDestroy(j1);
    hipEventDestroy(j2);
    return r;
}

int krk_metainfo_digest_chunks_dev(const krk_chunk* chunks, uint64_t n, uint32_t* state_dev, uint32_t* sums_dev,
                                   uint8_t* digests_dev, void* stream) {
    KRK_DEVICE(D);
    int r = validate_chunks(chunks, n);
    if (r || !n) return r;
    KRK_CHECK(state_dev && sums_dev && digests_dev, KRK_EINVAL, "chunks_dev: null output");
    ItemBuilder B;
    return chunks_step(D, chunks, n, state_dev, sums_dev, digests_dev, pick(D, stream), B);
}

int krk_metainfo_digest_chunks_dev_on(const krk_chunk* chunks, uint64_t n, uint32_t* state_dev, uint32_t* sums_dev,
                                      uint8_t* digests_dev, void* stream, void* sha_stream) {
    KRK_DEVICE(D);
    int r = validate_chunks(chunks, n);
    if (r || !n) return r;
    KRK_CHECK(state_dev && sums_dev && digests_dev, KRK_EINVAL, "chunks_dev: null output");
    ItemBuilder B;
    return chunks_step(D, chunks, n, state_dev, sums_dev, digests_dev, pick(D, stream), B,
                       static_cast<hipStream_t>(sha_stream));
}

int krk_metainfo_digest_chunks_dev_after(const krk_chunk* chunks, uint64_t n, uint32_t* state_dev, uint32_t* sums_dev,
                                         uint8_t* digests_dev, void* stream, void* sha_stream) {
    KRK_DEVICE(D);
    int r = validate_chunks(chunks, n);
    if (r || !n) return r;
    KRK_CHECK(state_dev && sums_dev && digests_dev && sha_stream, KRK_EINVAL, "chunks_dev_after: null argument");
    ItemBuilder B;
    return chunks_step(D, chunks, n, state_dev, sums_dev, digests_dev, pick(D, stream), B,
                       static_cast<hipStream_t>(sha_stream), /*crc_after_sha=*/true);
}

// The piece CRCs of device chunks alone (no SHA-256): the tail bytes of chains whose
// SHA-256 a host thread finishes (the windowed tail handoff, kraken_amd/windowed.py) still
// get their piece sums on the GPU, XOR-accumulated like a window's.
int krk_chunks_crc_dev(const krk_chunk* chunks, uint64_t n, uint32_t* sums_dev, void* stream) {
    KRK_DEVICE(D);
    int r = validate_chunks(chunks, n, /*crc_only=*/true);
    if (r || !n) return r;
    KRK_CHECK(sums_dev, KRK_EINVAL, "chunks_crc_dev: sums_dev is NULL");
    ItemBuilder B;
    CrcBatch items;
    for (uint64_t i = 0; i < n; ++i)
        if (chunks[i].length)
            B.add(items, reinterpret_cast<uint64_t>(chunks[i].data), chunks[i].offset,
                  chunks[i].offset + chunks[i].length, chunks[i].blob_length, (uint64_t)chunks[i].piece_length,
                  chunks[i].sums_offset);
    return run_items(D, items, sums_dev, pick(D, stream));
}

// krk_metainfo_digest_host: windows.cpp

int krk_verify_pieces_dev(const krk_blob* blob, const uint32_t* expected_host, uint8_t* ok_out_host, void* stream) {
    KRK_CHECK(blob && expected_host && ok_out_host, KRK_EINVAL, "verify: null argument");
    KRK_DEVICE(D);
    hipStream_t s = pick(D, stream);
    krk_blob b = *blob;
    b.sums_offset = 0;
    const uint64_t np = krk_num_pieces(b.length, b.piece_length);
    int r = validate_blobs(&b, 1);
    if (r || !np) return r;
    uint32_t* d_sums = nullptr;
    uint8_t* d_ok = nullptr;
    KRK_HIP(scratch_alloc(D, reinterpret_cast<void**>(&d_sums), np * 4, s));
    KRK_HIP(scratch_alloc(D, reinterpret_cast<void**>(&d_ok), np, s));
    r = piece_sums_dev(D, &b, 1, d_sums, s);
    void* d_exp = nullptr;
    if (!r) r = upload(D, expected_host, np * 4, &d_exp, s);
    if (!r) {
        hipError_t e = launch_crc_verify(d_sums, static_cast<const uint32_t*>(d_exp), d_ok, (uint32_t)np, s);
        if (e != hipSuccess) { set_error(KRK_EHIP, "verify launch: %s", launch_error_text(e)); r = KRK_EHIP; }
    }
    if (hipStreamSynchronize(s) != hipSuccess && !r) { set_error(KRK_EHIP, "verify sync"); r = KRK_EHIP; }
    if (!r && hipMemcpy(ok_out_host, d_ok, np, hipMemcpyDeviceToHost) != hipSuccess) r = KRK_EHIP;
    scratch_free(D, d_sums, s);
    scratch_free(D, d_ok, s);
    if (d_exp) scratch_free(D, d_exp, s);
    if (hipStreamSynchronize(s) != hipSuccess && !r) { set_error(KRK_EHIP, "verify sync"); r = KRK_EHIP; }
    return r;
}

int krk_verify_pieces_host(const uint8_t* const* data, const uint64_t* lengths, const uint32_t* expected,
                           uint64_t n, uint8_t* ok_out) {
    if (!n) return KRK_OK;
    KRK_CHECK(data && lengths && expected && ok_out, KRK_EINVAL, "verify_pieces_host: null argument");
    // Each piece is a one-piece blob; an empty piece sums to 0 (crc32 of nothing).
    std::vector<krk_blob> blobs(n);
    for (uint64_t i = 0; i < n; ++i)
        blobs[i] = krk_blob{data[i], lengths[i], (int64_t)std::max<uint64_t>(lengths[i], 1), i};
    std::vector<uint32_t> sums(n, 0);
    int r = krk_piece_sums_host(blobs.data(), n, sums.data());
    if (r) return r;
    for (uint64_t i = 0; i < n; ++i) ok_out[i] = sums[i] == expected[i];
    return KRK_OK;
}

// ---------------------------------------------------------------- HRW
static int hexv(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

// A ring's node table (label bytes, label offsets, weights) and, for the Locations
// table, the healthy flags: ONE upload (one copy on the stream instead of four).
struct DevNodes {
    void* pack = nullptr;
    const uint8_t* labels = nullptr;
    const uint64_t* off = nullptr;
    const int64_t* w = nullptr;
    const uint8_t* healthy = nullptr;
};

static int upload_nodes(Device* D, const krk_nodes* nodes, DevNodes& dn, hipStream_t s,
                        const uint8_t* healthy = nullptr) {
    KRK_CHECK(nodes && nodes->n_nodes > 0 && nodes->label_off && nodes->weights, KRK_EINVAL,
              "nodes: empty or null");
    KRK_CHECK(nodes->n_nodes <= 4096, KRK_EINVAL, "more than 4096 nodes");
    const uint64_t N = nodes->n_nodes, lb = nodes->label_off[N];
    KRK_CHECK(lb == 0 || nodes->labels, KRK_EINVAL, "nodes: labels are null");
    const size_t o_w = (N + 1) * 8, o_lab = o_w + N * 8, o_h = o_lab + lb;  // 8-byte parts first
    std::vector<uint8_t> pk(o_h + (healthy ? N : 0) + 1, 0);
    memcpy(pk.data(), nodes->label_off, (N + 1) * 8);
    memcpy(pk.data() + o_w, nodes->weights, N * 8);
    if (lb) memcpy(pk.data() + o_lab, nodes->labels, lb);
    if (healthy) memcpy(pk.data() + o_h, healthy, N);
    int r = upload(D, pk.data(), pk.size(), &dn.pack, s);
    if (r) return r;
    const uint8_t* b = static_cast<const uint8_t*>(dn.pack);
    dn.off = reinterpret_cast<const uint64_t*>(b);
    dn.w = reinterpret_cast<const int64_t*>(b + o_w);
    dn.labels = b + o_lab;
    dn.healthy = healthy ? b + o_h : nullptr;
    return KRK_OK;
}

static void free_nodes(Device* D, DevNodes& dn, hipStream_t s) {
    if (dn.pack) scratch_free(D, dn.pack, s);
    dn = DevNodes();
}

// Order + Locations table for nk decoded keys already on the device; result rows
// on the device.
static int hrw_table_dev(Device* D, const void* d_kb, const void* d_koff, const void* d_bad, uint64_t nk,
                         const krk_nodes* nodes, const uint8_t* healthy, int32_t max_replica, uint32_t row_out,
                         int32_t** d_locs, uint8_t** d_counts, hipStream_t s) {
    const uint32_t N = nodes->n_nodes;
    DevNodes dn;
    int r = upload_nodes(D, nodes, dn, s, healthy);
    int32_t* d_order = nullptr;
    if (!r && scratch_alloc(D, reinterpret_cast<void**>(&d_order), nk * N * 4, s) != hipSuccess) r = KRK_ENOMEM;
    if (!r && scratch_alloc(D, reinterpret_cast<void**>(d_locs), nk * row_out * 4, s) != hipSuccess) r = KRK_ENOMEM;
    if (!r && scratch_alloc(D, reinterpret_cast<void**>(d_counts), nk, s) != hipSuccess) r = KRK_ENOMEM;
    if (!r) {
        HrwArgs a{static_cast<const uint8_t*>(d_kb), static_cast<const uint64_t*>(d_koff), nk, dn.labels, dn.off,
                  dn.w, N, N, static_cast<const uint8_t*>(d_bad), d_order, nullptr};
        hipError_t e = timed(K_HRW, s, [&] { return launch_hrw_order(a, s); });
        if (e == hipSuccess)
            e = timed(K_FILTER, s, [&] {
                return launch_ring_filter(d_order, nk, N, dn.healthy, max_replica, row_out, *d_locs, *d_counts, s);
            });
        if (e != hipSuccess) { set_error(KRK_EHIP, "hrw launch: %s", launch_error_text(e)); r = KRK_EHIP; }
    }
    free_nodes(D, dn, s);
    if (d_order) scratch_free(D, d_order, s);
    return r;
}

// The same for keys given on the host.
static int hrw_table(Device* D, const std::vector<uint8_t>& kb, const std::vector<uint64_t>& koff,
                     const std::vector<uint8_t>& bad, const krk_nodes* nodes, const uint8_t* healthy,
                     int32_t max_replica, uint32_t row_out, int32_t** d_locs, uint8_t** d_counts,
                     hipStream_t s) {
    void *d_kb = nullptr, *d_koff = nullptr, *d_bad = nullptr;
    int r = upload(D, kb.data(), kb.size(), &d_kb, s);
    if (!r) r = upload(D, koff.data(), koff.size() * 8, &d_koff, s);
    if (!r) r = upload(D, bad.data(), bad.size(), &d_bad, s);
    if (!r) r = hrw_table_dev(D, d_kb, d_koff, d_bad, koff.size() - 1, nodes, healthy, max_replica, row_out,
                              d_locs, d_counts, s);
    for (void* p : {d_kb, d_koff, d_bad})
        if (p) scratch_free(D, p, s);
    return r;
}

int krk_hrw_ordered(const char* keys, const uint64_t* key_off, uint64_t n_keys, const krk_nodes* nodes,
                    uint32_t n_out, int32_t* order_out, double* scores_out) {
    if (!n_keys) return KRK_OK;
    KRK_CHECK(keys && key_off && order_out, KRK_EINVAL, "hrw_ordered: null argument");
    // rows are n_out wide (-1 padded past the node count); bounded like the node count
    KRK_CHECK(n_out <= 4096, KRK_EINVAL, "n_out %u exceeds 4096", n_out);
    KRK_DEVICE(D);
    hipStream_t s = D->s_main;
    // hex.DecodeString per key (rendezvous.go:154-157).
    std::vector<uint8_t> kb;
    std::vector<uint64_t> koff(n_keys + 1, 0);
    std::vector<uint8_t> bad(n_keys, 0);
    bool any_bad = false;
    for (uint64_t i = 0; i < n_keys; ++i) {
        const char* k = keys + key_off[i];
        const uint64_t len = key_off[i + 1] - key_off[i];
        koff[i] = kb.size();
        bool ok = (len % 2) == 0;
        for (uint64_t q = 0; ok && q + 1 < len; q += 2) {
            const int a = hexv(k[q]), b = hexv(k[q + 1]);
            if (a < 0 || b < 0) { ok = false; break; }
            kb.push_back((uint8_t)(a << 4 | b));
        }
        if (!ok) { kb.resize(koff[i]); bad[i] = 1; any_bad = true; }
    }
    koff[n_keys] = kb.size();
    if (kb.empty()) kb.push_back(0);
    DevNodes dn;
    int r = upload_nodes(D, nodes, dn, s);
    const uint32_t N = nodes ? nodes->n_nodes : 0;
    void *d_kb = nullptr, *d_koff = nullptr, *d_bad = nullptr;
    int32_t* d_order = nullptr;
    double* d_sc = nullptr;
    if (!r) r = upload(D, kb.data(), kb.size(), &d_kb, s);
    if (!r) r = upload(D, koff.data(), koff.size() * 8, &d_koff, s);
    if (!r) r = upload(D, bad.data(), bad.size(), &d_bad, s);
    if (!r && scratch_alloc(D, reinterpret_cast<void**>(&d_order), n_keys * n_out * 4 + 4, s) != hipSuccess) r = KRK_ENOMEM;
    if (!r && scores_out && scratch_alloc(D, reinterpret_cast<void**>(&d_sc), n_keys * N * 8, s) != hipSuccess)
        r = KRK_ENOMEM;
    if (!r) {
        HrwArgs a{static_cast<const uint8_t*>(d_kb), static_cast<const uint64_t*>(d_koff), n_keys, dn.labels, dn.off,
                  dn.w, N, n_out, static_cast<const uint8_t*>(d_bad), d_order, d_sc};
        hipError_t e = n_out ? timed(K_HRW, s, [&] { return launch_hrw_order(a, s); }) : hipSuccess;
        if (e != hipSuccess) { set_error(KRK_EHIP, "hrw launch: %s", launch_error_text(e)); r = KRK_EHIP; }
    }
    // Copy-out: drain the stream, then blocking copies into the caller's (pageable) memory.
    if (hipStreamSynchronize(s) != hipSuccess && !r) { set_error(KRK_EHIP, "hrw sync"); r = KRK_EHIP; }
    if (!r && n_out && hipMemcpy(order_out, d_order, n_keys * n_out * 4, hipMemcpyDeviceToHost) != hipSuccess)
        r = KRK_EHIP;
    if (!r && scores_out && hipMemcpy(scores_out, d_sc, n_keys * N * 8, hipMemcpyDeviceToHost) != hipSuccess)
        r = KRK_EHIP;
    free_nodes(D, dn, s);
    for (void* p : {d_kb, d_koff, d_bad, static_cast<void*>(d_order), static_cast<void*>(d_sc)})
        if (p) scratch_free(D, p, s);
    if (hipStreamSynchronize(s) != hipSuccess && !r) { set_error(KRK_EHIP, "hrw sync"); r = KRK_EHIP; }
    if (!r && any_bad) {
        set_error(KRK_EHEX, "invalid hex key: Score is NaN");
        return KRK_EHEX;
    }
    return r;
}

int krk_hrw_uint64_to_float64(const uint8_t* sums8, uint64_t n, int rehash, double* out) {
    if (!n) return KRK_OK;
    KRK_CHECK(sums8 && out, KRK_EINVAL, "hrw_uint64_to_float64: null argument");
    KRK_DEVICE(D);
    hipStream_t s = D->s_main;
    std::vector<uint64_t> v(n);
    for (uint64_t i = 0; i < n; ++i) {  // binary.BigEndian.Uint64
        uint64_t x = 0;
        for (int k = 0; k < 8; ++k) x = x << 8 | sums8[8 * i + k];
        v[i] = x;
    }
    void* d_v = nullptr;
    double* d_o = nullptr;
    int r = upload(D, v.data(), n * 8, &d_v, s);
    if (!r && scratch_alloc(D, &d_o, n * 8, s) != hipSuccess) r = KRK_ENOMEM;
    if (!r) {
        hipError_t e = launch_u64_to_f64(static_cast<const uint64_t*>(d_v), n, rehash, d_o, s);
        if (e != hipSuccess) { set_error(KRK_EHIP, "u64_to_f64 launch: %s", launch_error_text(e)); r = KRK_EHIP; }
    }
    if (hipStreamSynchronize(s) != hipSuccess && !r) { set_error(KRK_EHIP, "u64_to_f64 sync"); r = KRK_EHIP; }
    if (!r && hipMemcpy(out, d_o, n * 8, hipMemcpyDeviceToHost) != hipSuccess) r = KRK_EHIP;
    if (d_v) scratch_free(D, d_v, s);
    if (d_o) scratch_free(D, d_o, s);
    return r;
}

static void shard_keys(std::vector<uint8_t>& kb, std::vector<uint64_t>& koff, const std::vector<uint32_t>& shards) {
    kb.resize(shards.size() * 2);
    koff.resize(shards.size() + 1);
    for (size_t i = 0; i < shards.size(); ++i) {
        kb[2 * i] = (uint8_t)(shards[i] >> 8);
        kb[2 * i + 1] = (uint8_t)shards[i];
        koff[i] = 2 * i;
    }
    koff[shards.size()] = kb.size();
}

int krk_ring_locations(const uint8_t* digests32, uint64_t n, const krk_nodes* nodes, const uint8_t* healthy,
                       int32_t max_replica, int32_t* locs_out, uint8_t* counts_out) {
    if (!n) return KRK_OK;
    KRK_CHECK(digests32 && healthy && locs_out && counts_out, KRK_EINVAL, "ring_locations: null argument");
    KRK_DEVICE(D);
    hipStream_t s = D->s_main;
    const uint32_t row_out = (uint32_t)std::max<int32_t>(1, max_replica);
    // Only the shards present: Locations depends on d only through ShardID.
    std::vector<int32_t> row_of(65536, -1);
    std::vector<uint32_t> shards;
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t sh = (uint32_t)digests32[32 * i] << 8 | digests32[32 * i + 1];
        if (row_of[sh] < 0) { row_of[sh] = (int32_t)shards.size(); shards.push_back(sh); }
    }
    std::vector<uint8_t> kb, bad(shards.size(), 0);
    std::vector<uint64_t> koff;
    shard_keys(kb, koff, shards);
    int32_t* d_locs = nullptr;
    uint8_t* d_counts = nullptr;
    int r = hrw_table(D, kb, koff, bad, nodes, healthy, max_replica, row_out, &d_locs, &d_counts, s);
    std::vector<int32_t> tl(shards.size() * row_out);
    std::vector<uint8_t> tc(shards.size());
    if (hipStreamSynchronize(s) != hipSuccess && !r) { set_error(KRK_EHIP, "ring sync"); r = KRK_EHIP; }
    if (!r && hipMemcpy(tl.data(), d_locs, tl.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) r = KRK_EHIP;
    if (!r && hipMemcpy(tc.data(), d_counts, tc.size(), hipMemcpyDeviceToHost) != hipSuccess) r = KRK_EHIP;
    if (d_locs) scratch_free(D, d_locs, s);
    if (d_counts) scratch_free(D, d_counts, s);
    if (hipStreamSynchronize(s) != hipSuccess && !r) { set_error(KRK_EHIP, "ring sync"); r = KRK_EHIP; }
    if (r) return r;
    for (uint64_t i = 0; i < n; ++i) {
        const int32_t row = row_of[(uint32_t)digests32[32 * i] << 8 | digests32[32 * i + 1]];
        memcpy(locs_out + i * row_out, tl.data() + (uint64_t)row * row_out, row_out * 4);
        counts_out[i] = tc[row];
    }
    return KRK_OK;
}

}  // extern "C"

// The 65,536-row owner table (one row per ShardID) on the device: d_tl rows of row_out
// node indices (-1 padded), d_tc counts.  Released by the caller with scratch_free.
static int shard_owner_table(Device* D, const krk_nodes* nodes, const uint8_t* healthy, int32_t max_replica,
                             uint32_t row_out, int32_t** d_tl, uint8_t** d_tc, hipStream_t s) {
    std::call_once(D->shard_once, [D] {
        std::vector<uint32_t> shards(65536);
        std::iota(shards.begin(), shards.end(), 0u);
        std::vector<uint8_t> kb, bad(65536, 0);
        std::vector<uint64_t> koff;
        shard_keys(kb, koff, shards);
        if (hipMalloc(&D->shard_kb, kb.size()) != hipSuccess || hipMalloc(&D->shard_koff, koff.size() * 8) != hipSuccess ||
            hipMalloc(&D->shard_bad, bad.size()) != hipSuccess ||
            hipMemcpy(D->shard_kb, kb.data(), kb.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(D->shard_koff, koff.data(), koff.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(D->shard_bad, bad.data(), bad.size(), hipMemcpyHostToDevice) != hipSuccess)
            D->shard_rc = KRK_ENOMEM;
    });
    KRK_CHECK(D->shard_rc == KRK_OK, D->shard_rc, "shard key table allocation failed");
    return hrw_table_dev(D, D->shard_kb, D->shard_koff, D->shard_bad, 65536, nodes, healthy, max_replica, row_out,
                         d_tl, d_tc, s);
}

// The shard owner tables of the last few memberships a device served (ring.Refresh caches
// its hrw in the reference, lib/hashring/ring.go:141-165; Locations never recomputes it):
// keyed by the exact membership bytes (labels, weights, health, MaxReplica).  A table is
// built once on the caller's stream (ready event); later callers wait for that event and
// record a per-stream "used" event, and an evicted table's blocks go back to the scratch
// cache stream-ordered behind every stream that used it.
namespace krk {
struct OwnerTable {
    std::vector<uint8_t> key;
    int32_t* tl = nullptr;
    uint8_t* tc = nullptr;
    uint32_t* tp = nullptr;  // packed rows (launch_pack_owner_rows) when N <= 255 and row <= 3
    hipEvent_t ready = nullptr;
    std::vector<std::pair<hipStream_t, hipEvent_t>> used;
    uint64_t stamp = 0;
    int inflight = 0;  // callers between owner_table() and owner_used(): not evictable
};
struct OwnerTables {
    std::vector<OwnerTable> e;
    uint64_t clock = 0;
};
}  // namespace krk
static constexpr size_t kOwnerTables = 8;

static std::vector<uint8_t> owner_key(const krk_nodes* nodes, const uint8_t* healthy, int32_t max_replica) {
    const uint32_t N = nodes->n_nodes;
    std::vector<uint8_t> k;
    auto put = [&k](const void* p, size_t n) {
        const uint8_t* b = static_cast<const uint8_t*>(p);
        k.insert(k.end(), b, b + n);
    };
    put(&N, 4);
    put(&max_replica, 4);
    put(nodes->label_off, (N + 1) * 8);
    put(nodes->labels + nodes->label_off[0], nodes->label_off[N] - nodes->label_off[0]);
    put(nodes->weights, N * 8);
    put(healthy, N);
    return k;
}

static void owner_release(Device* D, OwnerTable& t, hipStream_t s) {
    for (auto& u : t.used) {
        hipStreamWaitEvent(s, u.second, 0);
        hipEventDestroy(u.second);
    }
    if (t.ready) hipEventDestroy(t.ready);
    if (t.tl) scratch_free(D, t.tl, s);
    if (t.tc) scratch_free(D, t.tc, s);
    if (t.tp) scratch_free(D, t.tp, s);
    const int inflight = t.inflight;
    t = OwnerTable{};
    t.inflight = inflight;
}

// Device pointers of the owner table of (nodes, healthy, max_replica), usable on stream s
// once the call returns (s waits for its build); the caller's use is recorded after its
// launch with owner_used(), which every successful call must be followed by.  Slots are
// stable: a failed build leaves its slot empty instead of erasing it, and a slot
// with a caller between the two calls is never evicted (the cache grows past kOwnerTables
// rather than release a table a launch is about to read).
static int owner_table(Device* D, const krk_nodes* nodes, const uint8_t* healthy, int32_t max_replica,
                       uint32_t row_out, int32_t** d_tl, uint8_t** d_tc, uint32_t** d_tp, size_t* slot,
                       hipStream_t s) {
    std::vector<uint8_t> key = owner_key(nodes, healthy, max_replica);
    std::lock_guard<std::mutex> g(D->owners_mu);
    if (!D->owners) D->owners = new OwnerTables();
    OwnerTables& C = *D->owners;
    for (size_t i = 0; i < C.e.size(); ++i)
        if (C.e[i].key == key) {
            KRK_HIP(hipStreamWaitEvent(s, C.e[i].ready, 0));
            C.e[i].stamp = ++C.clock;
            C.e[i].inflight++;
            *d_tl = C.e[i].tl;
            *d_tc = C.e[i].tc;
            *d_tp = C.e[i].tp;
            *slot = i;
            return KRK_OK;
        }
    size_t i = C.e.size();
    for (size_t j = 0; j < C.e.size(); ++j)  // an empty slot (a failed build) first
        if (C.e[j].key.empty() && !C.e[j].inflight) {
            i = j;
            break;
        }
    if (i == C.e.size() && C.e.size() >= kOwnerTables) {  // else the least recently used idle one goes
        for (size_t j = 0; j < C.e.size(); ++j)
            if (!C.e[j].inflight && (i == C.e.size() || C.e[j].stamp < C.e[i].stamp)) i = j;
        if (i < C.e.size()) owner_release(D, C.e[i], s);
    }
    if (i == C.e.size()) C.e.emplace_back();
    OwnerTable& t = C.e[i];
    int r = shard_owner_table(D, nodes, healthy, max_replica, row_out, &t.tl, &t.tc, s);
    if (!r && nodes->n_nodes <= 255 && row_out <= 3 &&
        (scratch_alloc(D, &t.tp, 65536 * sizeof(uint32_t), s) != hipSuccess ||
         launch_pack_owner_rows(t.tl, t.tc, row_out, t.tp, s) != hipSuccess)) {
        set_error(KRK_EHIP, "ring owner table: packed rows");
        r = KRK_EHIP;
    }
    if (!r && (hipEventCreateWithFlags(&t.ready, hipEventDisableTiming) != hipSuccess ||
               hipEventRecord(t.ready, s) != hipSuccess)) {
        set_error(KRK_EHIP, "ring owner table: event");
        r = KRK_EHIP;
    }
    if (r) {
        owner_release(D, t, s);  // the slot stays, empty (key cleared), for the next build
        return r;
    }
    t.key = std::move(key);
    t.stamp = ++C.clock;
    t.inflight++;
    *d_tl = t.tl;
    *d_tc = t.tc;
    *d_tp = t.tp;
    *slot = i;
    return KRK_OK;
}

void krk::owner_tables_teardown(Device& D) {
    if (!D.owners) return;
    for (OwnerTable& t : D.owners->e) owner_release(&D, t, D.s_main);
    hipStreamSynchronize(D.s_main);
    delete D.owners;
    D.owners = nullptr;
}

static void owner_used(Device* D, size_t slot, hipStream_t s) {
    std::lock_guard<std::mutex> g(D->owners_mu);
    OwnerTable& t = D->owners->e[slot];
    t.inflight--;
    for (auto& u : t.used)
        if (u.first == s) {
            hipEventRecord(u.second, s);
            return;
        }
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess && hipEventRecord(ev, s) == hipSuccess)
        t.used.push_back({s, ev});
    else if (ev) {
        hipEventDestroy(ev);
        hipStreamSynchronize(s);  // no event to order the release behind: the use is done now
    }
}

// Where the placement kernels may write [p, p + n): device memory, or page-locked host
// memory the GPU maps at its host address (krk_host_alloc / hipHostMalloc / registered:
// the gather then writes the owner lists over PCIe and the caller needs no copy-back).
// Pageable memory, or a mapping at another address, is refused -- the kernel would fault.
static bool device_writable(const void* p, uint64_t n) {
    auto ok_at = [](const void* q) {
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        // device memory, managed / unified memory, or page-locked host memory
        // the GPU maps at its host address
        if (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged || a.type == hipMemoryTypeUnified)
            return true;
        return a.type == hipMemoryTypeHost && a.devicePointer == q;
    };
    return ok_at(p) && (n <= 1 || ok_at(static_cast<const uint8_t*>(p) + n - 1));
}

template <typename T>
static int ring_locations_dev(const uint8_t* digests32_dev, uint64_t n, const krk_nodes* nodes,
                              const uint8_t* healthy, int32_t max_replica, T* locs_dev, uint8_t* counts_dev,
                              void* stream) {
    if (!n) return KRK_OK;
    KRK_CHECK(digests32_dev && healthy && locs_dev && counts_dev && nodes, KRK_EINVAL,
              "ring_locations_dev: null argument");
    KRK_CHECK(sizeof(T) != 1 || nodes->n_nodes <= 255, KRK_ERANGE,
              "ring_locations_u8_dev: %u nodes do not fit 8-bit owner indices (<= 255)", nodes->n_nodes);
    KRK_DEVICE(D);
    hipStream_t s = pick(D, stream);
    const uint32_t row_out = (uint32_t)std::max<int32_t>(1, max_replica);
    KRK_CHECK(device_writable(locs_dev, n * row_out * sizeof(T)) && device_writable(counts_dev, n), KRK_EINVAL,
              "ring_locations_dev: locs and counts must be device memory or page-locked host memory");
    int32_t* d_tl = nullptr;
    uint8_t* d_tc = nullptr;
    uint32_t* d_tp = nullptr;
    size_t slot = 0;
    int r = owner_table(D, nodes, healthy, max_replica, row_out, &d_tl, &d_tc, &d_tp, &slot, s);
    if (!r) {
        hipError_t e = timed(K_GATHER, s, [&] {
            if constexpr (sizeof(T) == 1) {
                // word stores need word-aligned outputs and a 2-byte aligned digest array
                const bool words = d_tp && !((uintptr_t)digests32_dev & 1) && !((uintptr_t)locs_dev & 3) &&
                                   !((uintptr_t)counts_dev & 3);
                if (words) return launch_shard_gather_packed(digests32_dev, n, d_tp, row_out, locs_dev, counts_dev, s);
                return launch_shard_gather_u8(digests32_dev, n, d_tl, d_tc, row_out, locs_dev, counts_dev, s);
            } else
                return launch_shard_gather(digests32_dev, n, d_tl, d_tc, row_out, locs_dev, counts_dev, s);
        });
        owner_used(D, slot, s);
        if (e != hipSuccess) { set_error(KRK_EHIP, "gather launch: %s", launch_error_text(e)); r = KRK_EHIP; }
    }
    return r;
}

extern "C" {

int krk_ring_owner_table(const krk_nodes* nodes, const uint8_t* healthy, int32_t max_replica, int32_t* locs_out,
                         uint8_t* counts_out) {
    KRK_CHECK(nodes && healthy && locs_out && counts_out, KRK_EINVAL, "ring_owner_table: null argument");
    KRK_DEVICE(D);
    hipStream_t s = D->s_main;
    const uint32_t row_out = (uint32_t)std::max<int32_t>(1, max_replica);
    int32_t* d_tl = nullptr;
    uint8_t* d_tc = nullptr;
    int r = shard_owner_table(D, nodes, healthy, max_replica, row_out, &d_tl, &d_tc, s);
    if (hipStreamSynchronize(s) != hipSuccess && !r) { set_error(KRK_EHIP, "owner table sync"); r = KRK_EHIP; }
    if (!r && (hipMemcpy(locs_out, d_tl, size_t(65536) * row_out * 4, hipMemcpyDeviceToHost) != hipSuccess ||
               hipMemcpy(counts_out, d_tc, 65536, hipMemcpyDeviceToHost) != hipSuccess)) {
        set_error(KRK_EHIP, "owner table copy");
        r = KRK_EHIP;
    }
    if (d_tl) scratch_free(D, d_tl, s);
    if (d_tc) scratch_free(D, d_tc, s);
    return r;
}

int krk_ring_locations_dev(const uint8_t* digests32_dev, uint64_t n, const krk_nodes* nodes,
                           const uint8_t* healthy, int32_t max_replica, int32_t* locs_dev, uint8_t* counts_dev,
                           void* stream) {
    return ring_locations_dev(digests32_dev, n, nodes, healthy, max_replica, locs_dev, counts_dev, stream);
}

int krk_ring_locations_u8_dev(const uint8_t* digests32_dev, uint64_t n, const krk_nodes* nodes,
                              const uint8_t* healthy, int32_t max_replica, uint8_t* locs_dev, uint8_t* counts_dev,
                              void* stream) {
    return ring_locations_dev(digests32_dev, n, nodes, healthy, max_replica, locs_dev, counts_dev, stream);
}

// ---------------------------------------------------------------- synthetic data
int krk_synth_fill_dev(uint8_t* dst_dev, uint64_t blob_idx, uint64_t offset, uint64_t n, int variant, void* stream) {
    if (!n) return KRK_OK;
    KRK_CHECK(dst_dev, KRK_EINVAL, "dst is NULL");
    KRK_DEVICE(D);
    hipStream_t s = pick(D, stream);
    const uint64_t GAMMA = 0x9E3779B97F4A7C15ULL;
    auto mix = [](uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    };
    const uint64_t seed = mix((0x4B52414B454EULL ^ blob_idx) + GAMMA);
    hipError_t e = timed(K_SYNTH, s, [&] { return launch_synth_fill(dst_dev, seed, offset, n, variant, s); });
    KRK_CHECK(e == hipSuccess, KRK_EHIP, "synth launch: %s", launch_error_text(e));
    return KRK_OK;
}

int krk_synth_fill_chunks_dev(const krk_chunk* chunks, uint64_t n, int variant, void* stream) {
    if (!n) return KRK_OK;
    KRK_CHECK(chunks, KRK_EINVAL, "chunks is NULL");
    KRK_CHECK(n <= 0xFFFFFFFFull / 16, KRK_EINVAL, "too many chunks");
    KRK_DEVICE(D);
    hipStream_t s = pick(D, stream);
    const uint64_t GAMMA = 0x9E3779B97F4A7C15ULL;
    auto mix = [](uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    };
    std::vector<SynthChunk> sc;
    sc.reserve(n);
    for (uint64_t i = 0; i < n; ++i) {
        if (!chunks[i].length) continue;
        KRK_CHECK(chunks[i].data, KRK_EINVAL, "chunk %llu: data is NULL", (unsigned long long)i);
        sc.push_back({const_cast<uint8_t*>(chunks[i].data), mix((0x4B52414B454EULL ^ chunks[i].blob) + GAMMA),
                      chunks[i].offset, chunks[i].length});
    }
    if (sc.empty()) return KRK_OK;
    void* d_sc = nullptr;
    int r = upload(D, sc.data(), sc.size() * sizeof(SynthChunk), &d_sc, s);
    if (r) return r;
    hipError_t e = timed(K_SYNTH, s, [&] {
        return launch_synth_fill_chunks(static_cast<const SynthChunk*>(d_sc), (uint32_t)sc.size(), variant, s);
    });
    scratch_free(D, d_sc, s);
    KRK_CHECK(e == hipSuccess, KRK_EHIP, "synth launch: %s", launch_error_text(e));
    return KRK_OK;
}

// ---------------------------------------------------------------- memory helpers
int krk_dev_alloc(uint64_t bytes, void** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_DEVICE(D);
    (void)D;
    hipError_t e = hipMalloc(out, bytes ? bytes : 1);
    KRK_CHECK(e == hipSuccess, KRK_ENOMEM, "hipMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(e));
    return KRK_OK;
}
int krk_dev_free(void* p) {
    KRK_HIP(hipFree(p));
    return KRK_OK;
}
// Page-locked host memory for receive buffers and staged results.  Large buffers are
// anonymous mappings in transparent huge pages registered with HIP (pages placed by the
// default policy as the registration faults them in): the GPU's DMA reads them at the same
// rate as hipHostMalloc memory (57.2-57.6 GB/s) and host threads read them as fast as
// pageable memory (the library's host CRC: 216 vs 218 GB/s pageable, against 166 for
// hipHostMalloc blocks on the same box; interleaving the pages over the NUMA nodes cost as
// much, 165; tools/micro/host_mem_probe.cpp, profiles/r04/host_mem_probe*.jsonl).  Small
// buffers stay hipHostMalloc (one registration per call costs more than it saves).
namespace {
std::mutex g_host_mu;
std::unordered_map<void*, size_t> g_host_maps;  // registered mappings: address -> length
std::map<uintptr_t, size_t> g_host_ranges;      // every live krk_host_alloc block: start -> length

}  // namespace

extern "C++" {
namespace krk {
bool lib_pinned_range(const void* p, uint64_t n) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> g(g_host_mu);
    auto it = g_host_ranges.upper_bound(a);
    if (it == g_host_ranges.begin()) return false;
    --it;
    return a >= it->first && a + n <= it->first + it->second;
}
bool lib_pinned_block(const void* p, uint64_t n, uintptr_t* base) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> g(g_host_mu);
    auto it = g_host_ranges.upper_bound(a);
    if (it == g_host_ranges.begin()) return false;
    --it;
    if (a < it->first || a + n > it->first + it->second) return false;
    *base = it->first;
    return true;
}
}  // namespace krk
}
int krk_host_alloc(uint64_t bytes, void** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_DEVICE(D);
    (void)D;
    constexpr uint64_t kLarge = 2ull << 20;
    if (bytes >= kLarge) {
        const size_t len = (bytes + kLarge - 1) & ~(kLarge - 1);
        void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p != MAP_FAILED) {
            madvise(p, len, MADV_HUGEPAGE);
            if (hipHostRegister(p, len, hipHostRegisterDefault) == hipSuccess) {
                std::lock_guard<std::mutex> g(g_host_mu);
                g_host_maps[p] = len;
                g_host_ranges[reinterpret_cast<uintptr_t>(p)] = len;
                *out = p;
                return KRK_OK;
            }
            (void)hipGetLastError();
            munmap(p, len);
        }
    }
    hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
    KRK_CHECK(e == hipSuccess, KRK_ENOMEM, "hipHostMalloc(%llu): %s", (unsigned long long)bytes,
              hipGetErrorString(e));
    std::lock_guard<std::mutex> g(g_host_mu);
    g_host_ranges[reinterpret_cast<uintptr_t>(*out)] = bytes ? bytes : 1;
    return KRK_OK;
}
int krk_host_alloc_dma(uint64_t bytes, void** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_DEVICE(D);
    (void)D;
    hipError_t e = hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault);
    KRK_CHECK(e == hipSuccess, KRK_ENOMEM, "hipHostMalloc(%llu): %s", (unsigned long long)bytes,
              hipGetErrorString(e));
    std::lock_guard<std::mutex> g(g_host_mu);
    g_host_ranges[reinterpret_cast<uintptr_t>(*out)] = bytes ? bytes : 1;
    return KRK_OK;
}
int krk_host_free(void* p) {
    size_t len = 0;
    {
        std::lock_guard<std::mutex> g(g_host_mu);
        g_host_ranges.erase(reinterpret_cast<uintptr_t>(p));
        auto it = g_host_maps.find(p);
        if (it != g_host_maps.end()) {
            len = it->second;
            g_host_maps.erase(it);
        }
    }
    if (len) {
        const hipError_t e = hipHostUnregister(p);
        munmap(p, len);
        KRK_HIP(e);
        return KRK_OK;
    }
    KRK_HIP(hipHostFree(p));
    return KRK_OK;
}
int krk_memcpy_h2d(void* dst, const void* src, uint64_t n) {
    KRK_DEVICE(D);
    (void)D;
    KRK_HIP(hipMemcpy(dst, src, n, hipMemcpyHostToDevice));
    return KRK_OK;
}
int krk_memcpy_d2h(void* dst, const void* src, uint64_t n) {
    KRK_DEVICE(D);
    (void)D;
    KRK_HIP(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost));
    return KRK_OK;
}
int krk_memcpy_d2h_async(void* dst, const void* src, uint64_t n, void* stream) {
    KRK_DEVICE(D);
    KRK_HIP(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, pick(D, stream)));
    return KRK_OK;
}
int krk_stream_create(void** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_DEVICE(D);
    (void)D;
    hipStream_t s;
    KRK_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *out = s;
    return KRK_OK;
}
int krk_device_pci_bus_id(char* out, uint32_t cap) {
    KRK_CHECK(out && cap >= 16, KRK_EINVAL, "device_pci_bus_id: a buffer of at least 16 bytes");
    KRK_DEVICE(D);
    KRK_HIP(hipDeviceGetPCIBusId(out, (int)cap, D->id));
    return KRK_OK;
}
int krk_device_cus(int* out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_DEVICE(D);
    *out = D->cus;
    return KRK_OK;
}
int krk_stream_create_prio(int priority, void** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_DEVICE(D);
    (void)D;
    int least = 0, greatest = 0;  // HIP: numerically lower = higher priority
    KRK_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    const int p = priority < 0 ? greatest : priority > 0 ? least : (least + greatest) / 2;
    hipStream_t s;
    KRK_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, p));
    *out = s;
    return KRK_OK;
}
int krk_stream_destroy(void* s) {
    KRK_CHECK(s, KRK_EINVAL, "stream is NULL");
    const hipStream_t hs = static_cast<hipStream_t>(s);
    // The library state tied to the stream lives on the stream's own device, which need not
    // be this thread's.
    hipDevice_t owner = t_dev;
    KRK_HIP(hipStreamGetDevice(hs, &owner));
    const int saved = t_dev;
    int drc = KRK_OK;
    if (Device* D = device_id((int)owner, &drc)) forget_stream(D, hs);
    device_id(saved, &drc);  // the calling thread's current device is unchanged
    KRK_HIP(hipStreamDestroy(hs));
    return KRK_OK;
}
int krk_stream_sync(void* s) {
    KRK_DEVICE(D);
    KRK_HIP(hipStreamSynchronize(pick(D, s)));
    return KRK_OK;
}

int krk_event_create(void** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_DEVICE(D);
    (void)D;
    hipEvent_t e;
    // blocking sync: a host thread waiting for a window (tens of ms) sleeps instead of
    // spinning a core of the process's CPU budget, which its hash threads need
    KRK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming | hipEventBlockingSync));
    *out = e;
    return KRK_OK;
}
int krk_event_record(void* ev, void* stream) {
    KRK_CHECK(ev, KRK_EINVAL, "event is NULL");
    KRK_DEVICE(D);
    KRK_HIP(hipEventRecord(static_cast<hipEvent_t>(ev), pick(D, stream)));
    return KRK_OK;
}
int krk_event_query(void* ev, int* done) {
    KRK_CHECK(ev && done, KRK_EINVAL, "event_query: null argument");
    const hipError_t e = hipEventQuery(static_cast<hipEvent_t>(ev));
    KRK_CHECK(e == hipSuccess || e == hipErrorNotReady, KRK_EHIP, "event query: %s", hipGetErrorString(e));
    if (e == hipErrorNotReady) (void)hipGetLastError();
    *done = e == hipSuccess;
    return KRK_OK;
}
int krk_event_create_polling(void** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_DEVICE(D);
    (void)D;
    hipEvent_t e;
    KRK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *out = e;
    return KRK_OK;
}
int krk_stream_wait_event(void* stream, void* ev) {
    KRK_CHECK(ev, KRK_EINVAL, "event is NULL");
    KRK_DEVICE(D);
    KRK_HIP(hipStreamWaitEvent(pick(D, stream), static_cast<hipEvent_t>(ev), 0));
    return KRK_OK;
}
int krk_event_sync(void* ev) {
    KRK_CHECK(ev, KRK_EINVAL, "event is NULL");
    KRK_HIP(hipEventSynchronize(static_cast<hipEvent_t>(ev)));
    return KRK_OK;
}
int krk_event_destroy(void* ev) {
    if (ev) hipEventDestroy(static_cast<hipEvent_t>(ev));
    return KRK_OK;
}

int krk_set_timing(int on) {
    g_timing.store(on != 0);
    return KRK_OK;
}
int krk_kernel_stats(const char* kernel, uint64_t* launches, double* total_ms) {
    KRK_CHECK(kernel, KRK_EINVAL, "kernel is NULL");
    drain_timing();
    std::lock_guard<std::mutex> g(g_tmu);
    for (int k = 0; k < K_N; ++k)
        if (strcmp(kernel, kKernNames[k]) == 0) {
            if (launches) *launches = g_cnt[k];
            if (total_ms) *total_ms = g_ms[k];
            return KRK_OK;
        }
    set_error(KRK_EINVAL, "unknown kernel '%s'", kernel);
    return KRK_EINVAL;
}
int krk_sha_lanes_per_stream(uint64_t n_streams, int* lanes) {
    KRK_CHECK(lanes, KRK_EINVAL, "lanes is NULL");
    KRK_CHECK(n_streams <= 0xffffffffull, KRK_ERANGE, "too many streams");
    KRK_DEVICE(D);
    (void)D;
    *lanes = sha_lanes_for((uint32_t)n_streams);
    return KRK_OK;
}
int krk_device_clock_mhz(void* stream, double* mhz) {
    KRK_CHECK(mhz, KRK_EINVAL, "mhz is NULL");
    KRK_DEVICE(D);
    hipStream_t s = pick(D, stream);
    uint64_t* d_out = nullptr;
    KRK_HIP(scratch_alloc(D, &d_out, 32, s));
    uint64_t h[3] = {0, 0, 0};
    hipError_t e = launch_clock_probe(1u << 20, d_out, s);
    if (e == hipSuccess) e = hipMemcpyAsync(h, d_out, 24, hipMemcpyDeviceToHost, s);
    scratch_free(D, d_out, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    KRK_CHECK(e == hipSuccess, KRK_EHIP, "clock probe: %s", launch_error_text(e));
    KRK_CHECK(h[1] > 0, KRK_EHIP, "clock probe: no realtime ticks");
    *mhz = (double)h[0] / (double)h[1] * 100.0;
    return KRK_OK;
}

int krk_set_sha_plan(int plan) {
    KRK_CHECK(sha_plan_valid(plan), KRK_EINVAL, "unknown SHA-256 launch plan %d", plan);
    set_sha_plan(plan);
    return KRK_OK;
}
int krk_reset_kernel_stats(void) {
    drain_timing();
    std::lock_guard<std::mutex> g(g_tmu);
    for (int k = 0; k < K_N; ++k) { g_ms[k] = 0; g_cnt[k] = 0; }
    int cur = 0;
    hipGetDevice(&cur);
    for (int d = 0; d < kMaxDevs; ++d)
        if (g_origin[d]) {
            hipSetDevice(d);
            hipEventDestroy(g_origin[d]);
            g_origin[d] = nullptr;
        }
    hipSetDevice(cur);
    g_timeline.clear();
    return KRK_OK;
}
int krk_kernel_timeline(const char* kernel, krk_launch_rec* out, uint64_t cap, uint64_t* n) {
    KRK_CHECK(kernel && n, KRK_EINVAL, "kernel or n is NULL");
    int want = -1;
    for (int k = 0; k < K_N; ++k)
        if (strcmp(kernel, kKernNames[k]) == 0) want = k;
    KRK_CHECK(want >= 0, KRK_EINVAL, "unknown kernel '%s'", kernel);
    drain_timing();
    std::lock_guard<std::mutex> g(g_tmu);
    uint64_t m = 0;
    for (const auto& r : g_timeline) {
        if (r.k != want) continue;
        if (out && m < cap) out[m] = {r.dev, r.plan, r.units, r.t0, r.t1};
        ++m;
    }
    *n = m;
    return KRK_OK;
}
int krk_sha_plan_for(uint64_t n_streams, int* plan) {
    KRK_CHECK(plan, KRK_EINVAL, "plan is NULL");
    KRK_CHECK(n_streams <= 0xffffffffull, KRK_ERANGE, "too many streams");
    KRK_DEVICE(D);
    (void)D;
    *plan = sha_plan_for((uint32_t)n_streams);
    return KRK_OK;
}

}  // extern "C"
