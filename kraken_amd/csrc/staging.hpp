// staging.hpp -- internal to libkraken_hip: the pinned staging windows of the host
// paths (host buffers and files -> pinned host window -> device window -> kernels), and
// the host-side fills of a window (copies, file reads) spread over the host pool.
#pragma once
#include <errno.h>
#include <fcntl.h>
#include <linux/aio_abi.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <unordered_map>

#include "runtime.hpp"

namespace krk {

// Device allocations of one host-path call, freed on every return path (hipFree
// waits for the device, so work still queued on them on an error path is drained).
struct DevMem {
    std::vector<void*> ps;
    ~DevMem() {
        for (void* p : ps) hipFree(p);
    }
    template <class T>
    hipError_t alloc(T** p, size_t n) {
        void* v = nullptr;
        const hipError_t e = hipMalloc(&v, n);
        if (e == hipSuccess) ps.push_back(v);
        *p = static_cast<T*>(v);
        return e;
    }
};

// ------------------------------------------------------------------ host staging pipeline
// One pinned host window and one device window of the ring; window k is refilled only
// after the kernels that consumed it (events) have finished.
struct Window {
    uint8_t* host = nullptr;
    uint8_t* dev = nullptr;
    size_t cap = 0;
    hipEvent_t copied = nullptr;    // the H2D out of `host` has finished: host buffer reusable
    hipEvent_t consumed = nullptr;  // single-stream users: all work reading `dev` has finished
    hipEvent_t done[2] = {nullptr, nullptr};  // kernels reading `dev`, one event per kernel stream
    bool inflight = false, copying = false;
    bool done_pending[2] = {false, false};
};

// A window of page-locked chunks goes to the device as one hipMemcpyAsync a chunk when it has
// few enough chunks that the calls stay well under the window's transfer.  Windows of
// thousands of chunks stage instead: measured on MI355X, one hipMemcpyBatchAsync of a
// window's 14,336 pinned chunks ran at 4.3 GB/s against 50 GB/s staged (profiles/r04).
constexpr size_t kDirectMaxCalls = 64;

// A ring of pinned host windows and device windows.  The host side of window k is
// refilled once its H2D is done; the H2D into its device side waits (on the copy
// stream only) for the kernels that read the previous contents, so the upload of
// window k+1 overlaps the kernels of window k.
struct CopyTask {
    uint8_t* dst;
    const uint8_t* src;
    size_t n;
};

// KRK_STAGING_WINDOWS (2..4, default 3): windows in the ring; with more, a window's host copy
// or file reads may run further ahead of the upload and kernels of the earlier ones.  C2's
// end-to-end leg on MI355X: 47.4 GB/s with 2, 54.3 with 3, 53.1 with 4 (H2D 56.5 / 56.5 /
// 53.5 measured beside each; profiles/r04/e2e_staging_windows_*.json).
constexpr int kMaxWindows = 4;
inline int staging_windows() {
    static const int n = [] {
        const char* v = KRK_OP_ENV("KRK_STAGING_WINDOWS");
        const int x = v ? atoi(v) : 3;
        return std::min(kMaxWindows, std::max(2, x));
    }();
    return n;
}

struct Pipeline {
    Window w[kMaxWindows];
    int n = 2;  // windows in use
    int next(int k) const { return (k + 1) % n; }
    ~Pipeline() {
        for (auto& x : w) {
            if (x.inflight) hipEventSynchronize(x.consumed);
            if (x.copying) hipEventSynchronize(x.copied);
            for (int i = 0; i < 2; ++i)
                if (x.done_pending[i]) hipEventSynchronize(x.done[i]);
            if (x.host) hipHostFree(x.host);
            if (x.dev) hipFree(x.dev);
            if (x.copied) hipEventDestroy(x.copied);
            if (x.consumed) hipEventDestroy(x.consumed);
            for (auto e : x.done)
                if (e) hipEventDestroy(e);
        }
    }
    int init(size_t cap) {
        n = staging_windows();
        for (int i = 0; i < n; ++i) {
            Window& x = w[i];
            x.cap = cap;
            KRK_HIP(hipHostMalloc(reinterpret_cast<void**>(&x.host), cap, hipHostMallocDefault));
            KRK_HIP(hipMalloc(reinterpret_cast<void**>(&x.dev), cap));
            KRK_HIP(hipEventCreateWithFlags(&x.copied, hipEventDisableTiming));
            KRK_HIP(hipEventCreateWithFlags(&x.consumed, hipEventDisableTiming));
            for (auto& e : x.done) KRK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        return KRK_OK;
    }
    // Host side of window k is free for refilling.
    int acquire(int k) {
        if (w[k].inflight) {
            KRK_HIP(hipEventSynchronize(w[k].consumed));
            w[k].inflight = false;
        }
        if (w[k].copying) {
            KRK_HIP(hipEventSynchronize(w[k].copied));
            w[k].copying = false;
        }
        return KRK_OK;
    }
    // Upload n bytes of window k on cp, after the kernels that read its last contents.
    hipError_t h2d(int k, size_t n, hipStream_t cp) {
        Window& x = w[k];
        for (int i = 0; i < 2; ++i)
            if (x.done_pending[i]) {
                hipError_t e = hipStreamWaitEvent(cp, x.done[i], 0);
                if (e != hipSuccess) return e;
                x.done_pending[i] = false;
            }
        hipError_t e = hipMemcpyAsync(x.dev, x.host, n, hipMemcpyHostToDevice, cp);
        if (e == hipSuccess) e = hipEventRecord(x.copied, cp);
        if (e == hipSuccess) x.copying = true;
        return e;
    }
    // The caller's pinned bytes DMA'd straight into device window k (tasks' dst are
    // device addresses in it), after the kernels that read its last contents.
    hipError_t h2d_direct(int k, const std::vector<CopyTask>& tasks, hipStream_t cp) {
        Window& x = w[k];
        for (int i = 0; i < 2; ++i)
            if (x.done_pending[i]) {
                hipError_t e = hipStreamWaitEvent(cp, x.done[i], 0);
                if (e != hipSuccess) return e;
                x.done_pending[i] = false;
            }
        for (const auto& t : tasks) {
            hipError_t e = hipMemcpyAsync(t.dst, t.src, t.n, hipMemcpyHostToDevice, cp);
            if (e != hipSuccess) return e;
        }
        hipError_t e = hipEventRecord(x.copied, cp);
        if (e == hipSuccess) x.copying = true;
        return e;
    }
    // The caller's page-locked bytes gathered into device window k by ONE gather launch on
    // cp (spans' dst are device addresses in it), after the kernels that read its last
    // contents.
    int h2d_gather(Device* D, int k, const std::vector<GatherSpan>& spans, hipStream_t cp) {
        Window& x = w[k];
        for (int i = 0; i < 2; ++i)
            if (x.done_pending[i]) {
                KRK_HIP(hipStreamWaitEvent(cp, x.done[i], 0));
                x.done_pending[i] = false;
            }
        const int r = run_gather(D, spans, cp);
        if (r) return r;
        KRK_HIP(hipEventRecord(x.copied, cp));
        x.copying = true;
        return KRK_OK;
    }
    // Kernel stream ks (slot 0 or 1) has enqueued everything that reads window k.
    hipError_t release(int k, int slot, hipStream_t ks) {
        hipError_t e = hipEventRecord(w[k].done[slot], ks);
        if (e == hipSuccess) w[k].done_pending[slot] = true;
        return e;
    }
};

// KRK_TRACE=1: host-side phase times of the windowed host paths, to stderr.
inline bool trace_on() {
    static const bool on = KRK_OP_ENV("KRK_TRACE") && atoi(KRK_OP_ENV("KRK_TRACE")) > 0;
    return on;
}
inline double wall_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline size_t window_bytes() {
    const char* v = KRK_OP_ENV("KRK_WINDOW_MB");
    size_t mb = v ? strtoull(v, nullptr, 10) : 512;
    if (mb < 1) mb = 1;
    return mb << 20;
}

// The device's persistent staging windows (grown to at least `cap`) for one host-path
// call; a concurrent second caller, or a call wanting windows above 1 GiB, gets
// private windows (freed when the call returns) instead.
struct StagingLease {
    Device* D = nullptr;
    Pipeline* p = nullptr;
    std::unique_ptr<Pipeline> own;
    bool locked = false;
    ~StagingLease() {
        if (locked) D->staging_mu.unlock();
    }
};

inline int lease_staging(Device* D, size_t cap, StagingLease& L) {
    L.D = D;
    constexpr size_t kKeepMax = size_t(1) << 30;  // windows kept across calls: at most 4 x 1 GiB pinned
    if (cap <= kKeepMax && D->staging_mu.try_lock()) {
        L.locked = true;
        if (!D->staging || D->staging->w[0].cap < cap) {
            delete D->staging;  // its destructor drains the old windows' events
            D->staging = nullptr;
            auto p = std::make_unique<Pipeline>();
            // kept windows grow in 32 MiB steps with 32 MiB of headroom: a batch whose chunk
            // placement pads a little more (O_DIRECT's 4 KiB places: 512 MiB + 4 KiB x live)
            // must not re-pin three windows (~0.6 s) after one that padded less
            constexpr size_t kStep = size_t(32) << 20;
            int r = p->init(std::min(kKeepMax, (cap + kStep - 1) / kStep * kStep + kStep));
            if (r) return r;
            D->staging = p.release();
        }
        L.p = D->staging;
        return KRK_OK;
    }
    L.own = std::make_unique<Pipeline>();
    L.p = L.own.get();
    return L.own->init(cap);
}

// Whether [p, p + n) is page-locked host memory (krk_host_alloc / hipHostMalloc).  A range
// inside a krk_host_alloc block is answered from the library's own table (thousands of
// receive-buffer pieces a batch: a HIP pointer query each cost ~3 us).  Pageable
// memory is an expected "invalid value" here: not left pending on the thread (the next
// launch would report it as an unchecked earlier error).
bool lib_pinned_range(const void* p, uint64_t n);  // runtime.cpp: inside one live krk_host_alloc block

inline bool host_pinned(const void* p, uint64_t n) {
    if (lib_pinned_range(p, n)) return true;  // the library's own blocks: no HIP query
    auto pinned_at = [](const void* q) {
        hipPointerAttribute_t a{};
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        return a.type == hipMemoryTypeHost;
    };
    return pinned_at(p) && (n <= 1 || pinned_at(static_cast<const uint8_t*>(p) + n - 1));
}

// Whether the GPU addresses page-locked host memory at p at the host address itself (the
// gather kernel reads it there).
inline bool mapped_at_host_address(const void* p) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.devicePointer == p;
}

// The live krk_host_alloc block holding [p, p + n): its base in *base (runtime.cpp).
bool lib_pinned_block(const void* p, uint64_t n, uintptr_t* base);

// Whether the gather may read EVERY blob of a batch at its host address (the
// first blob alone was checked, and a batch mixing krk_host_alloc blocks with other
// page-locked mappings whose device address differs would have faulted the gather).  A
// krk_host_alloc block is queried once per call; other memory at both ends of each blob.
class MappedAtHost {
  public:
    bool operator()(const void* p, uint64_t n) {
        if (!n) return true;
        uintptr_t base = 0;
        if (lib_pinned_block(p, n, &base)) {
            auto it = blocks_.find(base);
            if (it == blocks_.end()) it = blocks_.emplace(base, mapped_at_host_address(reinterpret_cast<void*>(base))).first;
            return it->second;
        }
        return mapped_at_host_address(p) && (n == 1 || mapped_at_host_address(static_cast<const uint8_t*>(p) + n - 1));
    }

  private:
    std::unordered_map<uintptr_t, bool> blocks_;
};

// Host -> pinned staging copies of one window, split over the calling thread and the host
// pool's idle threads (one host thread's memcpy is well below the PCIe rate).
// KRK_COPY_THREADS overrides the split.

inline unsigned copy_threads() {
    const char* v = KRK_AB_ENV("KRK_COPY_THREADS");
    if (v) return std::max(1u, (unsigned)strtoul(v, nullptr, 10));
    return std::max(1u, std::min(16u, (unsigned)host_threads_for_call()));
}

inline void par_copy(const std::vector<CopyTask>& tasks) {
    size_t total = 0;
    for (const auto& t : tasks) total += t.n;
    const unsigned T = copy_threads();
    if (T == 1 || total < (8u << 20)) {
        for (const auto& t : tasks) memcpy(t.dst, t.src, t.n);
        return;
    }
    // Cut the concatenated byte range into T equal spans.
    auto run = [&](size_t lo, size_t hi) {
        size_t pos = 0;
        for (const auto& t : tasks) {
            const size_t a = std::max(lo, pos), b = std::min(hi, pos + t.n);
            if (a < b) memcpy(t.dst + (a - pos), t.src + (a - pos), b - a);
            pos += t.n;
            if (pos >= hi) break;
        }
    };
    // spans on the calling thread and the host pool's idle threads
    const size_t span = (total + T - 1) / T;
    host_parallel_for(T, (int)T - 1, [&](size_t i) { run(i * span, std::min(total, (i + 1) * span)); });
}

// File -> pinned window reads of one window, split over the copy threads at
// 1 MiB-aligned spans (O_DIRECT needs block-aligned offsets and lengths; every
// task starts 4 KiB-aligned in both the file and the window).
struct ReadTask {
    int fd;
    uint64_t off;   // file offset
    uint8_t* dst;
    size_t n;       // bytes wanted (O_DIRECT reads round the last block up)
    size_t blob;    // index into the caller's files (for the error message)
    std::atomic<uint64_t>* ra = nullptr;  // the file's readahead mark (hinted up to), or null
    uint64_t flen = 0;                    // the file's length (readahead stops there)
};

// Per-file readahead of the page-cache reads (KRK_FILE_READAHEAD_MB; default 0 = off).
// A window holds one chunk of every live file -- ~136 KiB each at 3,826 live files -- and the
// kernel's readahead turns that into ~128 KiB disk requests; the box's disk reads 13.9 GB/s at
// 128 KiB requests, 18.0 at 1 MiB and 21.9 at 8 MiB (16 threads, tools/micro/disk_probe,
// profiles/r05/disk_probe.jsonl), and neither more threads nor per-chunk WILLNEED hints
// move it.  So each file's reads run R bytes ahead of its chunks as POSIX_FADV_WILLNEED in
// R-sized pieces: one large request a file every R bytes, landing in the page cache while the
// windows before it are read, and the chunk reads copy from the cache.  Measured against no
// hint on four boxes' cold 32 GiB legs (profiles/r05/bench_files*.json): 2 MiB ahead ran
// 0.91-1.07x, 8 MiB 0.91-1.00x -- no effect beyond the disk's run-to-run noise, so it is off
// by default and the knob stays for disks where request size is the whole story.
inline uint64_t file_readahead_bytes() {
    const char* v = KRK_AB_ENV("KRK_FILE_READAHEAD_MB");
    return (v ? strtoull(v, nullptr, 10) : 0) << 20;
}

// Returns -1 on success, else the index of the failed task; err = its errno (0 = EOF).
inline long par_read(const std::vector<ReadTask>& tasks, bool direct, int* err) {
    // Spans are cut in a stream of the tasks laid end to end, each padded to 4 KiB
    // when direct, so every span boundary falls on a block boundary of its task.
    auto padded = [direct](size_t n) { return direct ? (n + 4095) & ~size_t(4095) : n; };
    size_t total = 0;
    for (const auto& t : tasks) total += padded(t.n);
    std::atomic<long> bad{-1};
    std::atomic<int> bad_errno{0};
    const uint64_t R = direct ? 0 : file_readahead_bytes();
    auto run = [&](size_t lo, size_t hi) {
        size_t pos = 0;
        for (size_t i = 0; i < tasks.size() && pos < hi; pos += padded(tasks[i].n), ++i) {
            const ReadTask& t = tasks[i];
            size_t a = std::max(lo, pos), b = std::min(hi, pos + t.n);
            if (a >= b) continue;
            a -= pos;
            b -= pos;
            if (R && t.ra) {  // keep the file hinted R bytes past this read, R bytes a hint
                const uint64_t want = std::min(t.flen, t.off + b + R);
                uint64_t mark = t.ra->load(std::memory_order_relaxed);
                while (mark < want) {
                    const uint64_t to = std::min(t.flen, mark + R);
                    if (t.ra->compare_exchange_weak(mark, to)) {
                        posix_fadvise(t.fd, (off_t)mark, (off_t)(to - mark), POSIX_FADV_WILLNEED);
                        mark = to;
                    }
                }
            }
            while (a < b) {
                size_t want = b - a;
                if (direct) want = (want + 4095) & ~size_t(4095);
                const ssize_t got = pread(t.fd, t.dst + a, want, (off_t)(t.off + a));
                if (got < 0 && errno == EINTR) continue;
                if (got <= 0) {
                    long expect = -1;
                    bad.compare_exchange_strong(expect, (long)i);
                    bad_errno.store(got < 0 ? errno : 0);
                    return;
                }
                a += (size_t)got;
            }
        }
    };
    const unsigned T = (total < (8u << 20)) ? 1 : copy_threads();
    constexpr size_t kAlign = size_t(1) << 20;
    const size_t span = std::max(kAlign, ((total + T - 1) / T + kAlign - 1) & ~(kAlign - 1));
    const size_t spans = (total + span - 1) / span;
    host_parallel_for(spans, (int)spans - 1, [&](size_t i) { run(i * span, std::min(total, (i + 1) * span)); });
    *err = bad_errno.load();
    return bad.load();
}

// O_DIRECT reads of one window through Linux AIO: ONE thread submits every chunk
// (io_submit, up to kAioDepth in flight) and reaps them (io_getevents), so the disk sees a
// deep queue of requests without a thread blocked on each, and the bytes land in the pinned
// window by the disk's DMA with no page-cache copy.  On the GPU box's disk, a window of
// 3,826 chunks of 136 KiB: 16.2-16.4 GB/s from one thread against 11.7 for 16 threads'
// page-cache preads of the same chunks and 18.2 for 16 threads' 1 MiB whole-file reads
// (tools/micro/disk_probe.cpp, profiles/r05/disk_probe_aio.jsonl).  Tasks start 4 KiB-
// aligned in file and window; lengths are read rounded up to the block.  Returns -1 on
// success, else the index of a failed task with *err its errno (0 = unexpected EOF);
// -2 when AIO is unavailable (the caller reads synchronously).
inline bool use_aio() {  // KRK_FILE_AIO=0: O_DIRECT chunks by synchronous preads (A/B)
    const char* v = KRK_OP_ENV("KRK_FILE_AIO");
    return !(v && v[0] == '0');
}
// AIO contexts are kept for the process and reused: io_destroy waits out an RCU grace
// period, and destroying one per file batch cost ~0.35 s a call on the GPU box (a cold
// 32 GiB pass spent 2.03 s in its window loop and 2.39 s in the call).
class AioContexts {
  public:
    static AioContexts& get() {
        static AioContexts* p = new AioContexts();  // leaked at exit with its contexts
        return *p;
    }
    aio_context_t take(unsigned depth) {
        {
            std::lock_guard<std::mutex> g(mu_);
            if (!free_.empty()) {
                const aio_context_t c = free_.back();
                free_.pop_back();
                return c;
            }
        }
        aio_context_t c = 0;
        return syscall(SYS_io_setup, depth, &c) == 0 ? c : 0;
    }
    void give(aio_context_t c) {
        std::lock_guard<std::mutex> g(mu_);
        free_.push_back(c);
    }

  private:
    std::mutex mu_;
    std::vector<aio_context_t> free_;
};

class AioReader {
  public:
    static constexpr unsigned kAioDepth = 256;
    ~AioReader() {
        if (ctx_ && !broken_) AioContexts::get().give(ctx_);  // nothing in flight: every read was reaped
    }
    long read(const std::vector<ReadTask>& tasks, int* err) {
        *err = 0;
        if (tasks.empty()) return -1;
        if (!ctx_ && (failed_ || !(ctx_ = AioContexts::get().take(kAioDepth)))) {
            failed_ = true;
            return -2;
        }
        std::vector<iocb> cb(kAioDepth);
        std::vector<iocb*> ptr(kAioDepth);
        std::vector<io_event> ev(kAioDepth);
        std::vector<unsigned> free_slot(kAioDepth);
        std::vector<size_t> task_of(kAioDepth);
        for (unsigned q = 0; q < kAioDepth; ++q) free_slot[q] = kAioDepth - 1 - q;
        size_t next = 0, inflight = 0;
        long bad = -1;
        while ((next < tasks.size() && bad < 0) || inflight) {
            int nsub = 0;
            while (bad < 0 && next < tasks.size() && !free_slot.empty()) {
                const unsigned q = free_slot.back();
                free_slot.pop_back();
                const ReadTask& t = tasks[next];
                iocb& c = cb[q];
                memset(&c, 0, sizeof c);
                c.aio_data = q;
                c.aio_lio_opcode = IOCB_CMD_PREAD;
                c.aio_fildes = (uint32_t)t.fd;
                c.aio_buf = reinterpret_cast<uint64_t>(t.dst);
                c.aio_nbytes = (t.n + 4095) & ~size_t(4095);
                c.aio_offset = (int64_t)t.off;
                task_of[q] = next++;
                ptr[nsub++] = &c;
            }
            if (nsub) {
                long r = syscall(SYS_io_submit, ctx_, nsub, ptr.data());
                if (r < 0) r = 0;  // nothing went: the slots come back below
                for (int k = (int)r; k < nsub; ++k) {  // not submitted: read them synchronously
                    const unsigned q = (unsigned)ptr[k]->aio_data;
                    if (bad < 0 && !sync_read(tasks[task_of[q]], err)) bad = (long)task_of[q];
                    free_slot.push_back(q);
                }
                inflight += (size_t)r;
            }
            if (!inflight) continue;
            long got = syscall(SYS_io_getevents, ctx_, 1, (long)kAioDepth, ev.data(), nullptr);
            if (got < 0) {
                if (errno == EINTR) continue;
                *err = errno;
                broken_ = true;  // requests may still be in flight: the context is never reused
                return bad >= 0 ? bad : 0;  // fail the window
            }
            for (long e = 0; e < got; ++e) {
                const unsigned q = (unsigned)ev[e].data;
                const ReadTask& t = tasks[task_of[q]];
                const int64_t res = ev[e].res;
                if (bad < 0) {
                    if (res < 0) {
                        *err = (int)-res;
                        bad = (long)task_of[q];
                    } else if ((uint64_t)res < t.n && (res & 4095)) {  // the file ended inside the block
                        *err = 0;
                        bad = (long)task_of[q];
                    } else if ((uint64_t)res < t.n) {  // short on a block edge: the rest synchronously
                        ReadTask rest = t;
                        rest.off += (uint64_t)res;
                        rest.dst += res;
                        rest.n -= (size_t)res;
                        if (!sync_read(rest, err)) bad = (long)task_of[q];
                    }
                }
                free_slot.push_back(q);
            }
            inflight -= (size_t)got;
        }
        return bad;
    }

  private:
    aio_context_t ctx_ = 0;
    bool failed_ = false, broken_ = false;
    // pread until t.n bytes are in (block-rounded requests); false + *err on failure or EOF
    static bool sync_read(const ReadTask& t, int* err) {
        size_t a = 0;
        while (a < t.n) {
            const ssize_t got = pread(t.fd, t.dst + a, ((t.n - a) + 4095) & ~size_t(4095), (off_t)(t.off + a));
            if (got < 0 && errno == EINTR) continue;
            if (got <= 0) {
                *err = got < 0 ? errno : 0;
                return false;
            }
            a += (size_t)got;
        }
        return true;
    }
};

}  // namespace krk
