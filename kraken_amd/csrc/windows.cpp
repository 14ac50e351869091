// windows.cpp -- host-resident batches through the pinned staging windows:
// the upload / cache-fill verify of origin/blobserver/uploader.go:74-94 and
// lib/store/ca_store.go:99-135 (Digester over the bytes) fused with the metainfo of
// lib/metainfogen/generator.go:41-58 (piece CRCs of the same bytes), so each byte is read
// once -- from the caller's buffers (krk_metainfo_digest_host) or from the cache files
// themselves (krk_metainfo_digest_files) -- and crosses PCIe once, where the reference
// reads every upload twice.
//
// The window schedule (the C3 machinery of kraken_amd/windowed.py, here in C++): every live
// blob advances by the same chunk per window (about W bytes a window), SHA-256 chained
// through per-blob midstates in HBM and the chunk's piece CRCs XOR-accumulated into its
// pieces (CRC-32 is linear, so any cut is legal).  At most `cap` blobs are live, admitted
// longest first so the longest chain starts in window 0: by default 7/8 of the largest
// stream count the SHA-256 launch plan still runs on two lanes a stream (14,336 on 256
// CUs), which keeps every window on a multi-lane plan and leaves an eighth of the CUs free
// of SHA workgroups for the window's CRC launch, queued beside it on another stream
// (profiles/r02/c3_live_cap.jsonl).  The host's work per window is O(live).
#include <dirent.h>
#include <sys/mman.h>
#include <sys/resource.h>

#include <condition_variable>
#include <deque>
#include <thread>

#include "host_register.hpp"
#include "runtime.hpp"
#include "staging.hpp"

namespace krk {

// ----------------------------------------------------------------- the window schedule
struct WinChunk {
    uint32_t blob;
    uint64_t off, len;
};

class WindowSched {
  public:
    // blobs: the windowed blobs' indices into lens; chunks a multiple of `align` bytes
    // (64: SHA-256 blocks; 4 KiB for O_DIRECT file reads) except each blob's last.
    WindowSched(const uint64_t* lens, std::vector<uint32_t> blobs, uint64_t W, uint64_t cap, uint64_t align = 64)
        : L_(lens), W_(W), cap_(std::max<uint64_t>(cap, 1)), align_(std::max<uint64_t>(align, 64)), queue_(std::move(blobs)) {
        std::stable_sort(queue_.begin(), queue_.end(), [&](uint32_t a, uint32_t b) { return L_[a] > L_[b]; });
    }
    // The next window's chunks (in admission order); false once every blob is done.
    bool next(std::vector<WinChunk>& out) {
        out.clear();
        while (live_.size() < cap_ && q_ < queue_.size()) live_.push_back({queue_[q_++], 0});
        if (live_.empty()) return false;
        max_live_ = std::max<uint64_t>(max_live_, live_.size());
        const uint64_t c = std::max(align_, std::min(max_chunk_, W_ / live_.size()) / align_ * align_);
        size_t keep = 0;
        for (size_t k = 0; k < live_.size(); ++k) {
            auto [b, pos] = live_[k];
            const uint64_t take = std::min(c, L_[b] - pos);
            out.push_back({b, pos, take});
            pos += take;
            if (pos < L_[b]) live_[keep++] = {b, pos};
        }
        live_.resize(keep);
        return true;
    }
    uint64_t max_live() const { return max_live_; }
    // At most `c` bytes a chunk (rounded down to the alignment): the windows stay short once
    // few blobs are live (the tail handoff hands chains over at window boundaries).
    void set_max_chunk(uint64_t c) { max_chunk_ = std::max<uint64_t>(c, 1); }
    // Take blob b out of the schedule (its chain continues elsewhere): a live blob's slot goes
    // to the next waiting blob at the next window; a waiting one is never admitted.  *done:
    // the bytes the windows gave it (0 for a waiting blob).
    bool drop(uint32_t b, uint64_t* done) {
        for (size_t k = 0; k < live_.size(); ++k)
            if (live_[k].first == b) {
                *done = live_[k].second;
                live_.erase(live_.begin() + (long)k);
                return true;
            }
        for (size_t k = q_; k < queue_.size(); ++k)
            if (queue_[k] == b) {
                *done = 0;
                queue_.erase(queue_.begin() + (long)k);
                return true;
            }
        return false;
    }

  private:
    const uint64_t* L_;
    uint64_t W_, cap_, align_;
    std::vector<uint32_t> queue_;
    size_t q_ = 0;
    std::vector<std::pair<uint32_t, uint64_t>> live_;  // blob, bytes done
    uint64_t max_live_ = 0;
    uint64_t max_chunk_ = UINT64_MAX;
};

// Live streams per window on device D: 7/8 of the largest stream count whose SHA-256 launch
// still runs two (or eight) lanes a stream, a multiple of the two-pair workgroup's 64.
uint64_t window_stream_cap(Device* D) {
    (void)D;  // the plan reads the current device's CU count
    uint64_t lo = 1, hi = uint64_t(1) << 30;
    if (sha_lanes_for((uint32_t)hi) >= 2) return (hi * 7 / 8) / 64 * 64;
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) / 2;
        (sha_lanes_for((uint32_t)mid) >= 2 ? lo : hi) = mid;
    }
    return std::max<uint64_t>(64, (lo * 7 / 8) / 64 * 64);
}

namespace {

// Where a window's bytes come from: the caller's buffers or the cache files.
struct Filler {
    virtual ~Filler() = default;
    // bytes [off, off + len) of blob b into dst (host, pinned); the whole window at once
    struct Task {
        uint32_t b;
        uint64_t off, len;
        uint8_t* dst;
    };
    virtual int fill(const std::vector<Task>& tasks) = 0;
    // The source is page-locked: its chunks can be DMA'd straight into the device window.
    virtual const uint8_t* pinned_src(uint32_t /*blob*/, uint64_t /*off*/) const { return nullptr; }
    virtual bool pinned_all() const { return false; }
    // ... and the GPU addresses it at the host address (the gather reads it there)
    virtual bool pinned_mapped() const { return false; }
    // The caller's pageable bytes made page-locked for the gather (host_register.hpp), or null.
    virtual HostRegistry* registry() { return nullptr; }
    virtual const uint8_t* src(uint32_t /*blob*/, uint64_t /*off*/) const { return nullptr; }
};

struct MemFiller : Filler {
    const krk_blob* blobs;
    bool pinned = false;  // every windowed blob page-locked (krk_host_alloc): no staging copy
    bool mapped = false;  // ... at device addresses equal to the host ones
    std::unique_ptr<HostRegistry> reg;  // pageable blobs registered for the gather
    hipStream_t gather_stream = nullptr;  // where the gathers ran (drained before unregistering)
    explicit MemFiller(const krk_blob* b) : blobs(b) {}
    ~MemFiller() override {
        if (reg) reg->finish(gather_stream);
    }
    const uint8_t* pinned_src(uint32_t b, uint64_t off) const override { return pinned ? blobs[b].data + off : nullptr; }
    bool pinned_all() const override { return pinned; }
    bool pinned_mapped() const override { return mapped; }
    HostRegistry* registry() override { return reg.get(); }
    const uint8_t* src(uint32_t b, uint64_t off) const override { return blobs[b].data + off; }
    int fill(const std::vector<Task>& tasks) override {
        std::vector<CopyTask> c;
        c.reserve(tasks.size());
        for (const Task& t : tasks)
            if (t.len) c.push_back({t.dst, blobs[t.b].data + t.off, (size_t)t.len});
        par_copy(c);
        return KRK_OK;
    }
};

// A blob's file is opened at its first chunk and closed after its last; live blobs <= the
// descriptor budget (the window cap is capped by it), so no descriptor is reopened.
struct FileFiller : Filler {
    const krk_file_blob* files;
    bool direct;
    std::vector<int> fd;
    std::vector<char> is_direct;
    std::unique_ptr<std::atomic<uint64_t>[]> ra;  // each file's readahead mark (par_read)
    AioReader aio;                                  // the O_DIRECT chunks of a window
    FileFiller(const krk_file_blob* f, uint64_t n, bool want_direct)
        : files(f), direct(want_direct), fd(n, -1), is_direct(n, 0), ra(new std::atomic<uint64_t>[n]()) {}
    ~FileFiller() override {
        for (int x : fd)
            if (x >= 0) close(x);
    }
    int open_file(uint32_t i) {
        if (fd[i] >= 0) return KRK_OK;
        int x = -1;
        if (direct) {
            x = open(files[i].path, O_RDONLY | O_DIRECT | O_CLOEXEC);
            is_direct[i] = x >= 0;
        }
        if (x < 0) x = open(files[i].path, O_RDONLY | O_CLOEXEC);
        KRK_CHECK(x >= 0, KRK_EIO, "open %s: %s", files[i].path, strerror(errno));
        fd[i] = x;
        return KRK_OK;
    }
    int fill(const std::vector<Task>& tasks) override {
        std::vector<ReadTask> plain, odirect;
        for (const Task& t : tasks) {
            // every file is opened, an empty one too: Generate / verify open the file and
            // fail on a missing one
            int r = open_file(t.b);
            if (r) return r;
            if (!t.len) continue;
            (is_direct[t.b] ? odirect : plain)
                .push_back({fd[t.b], t.off, t.dst, (size_t)t.len, (size_t)t.b, &ra[t.b], files[t.b].length});
        }
        for (int pass = 0; pass < 2; ++pass) {
            const auto& rt = pass ? odirect : plain;
            if (rt.empty()) continue;
            int e = 0;
            long bad = pass == 1 && use_aio() ? aio.read(rt, &e) : -2;
            if (bad == -2) bad = par_read(rt, pass == 1, &e);
            if (bad >= 0) {
                const char* path = files[rt[bad].blob].path;
                if (e) set_error(KRK_EIO, "read blob: %s: %s", path, strerror(e));
                else set_error(KRK_EIO, "read blob: %s: unexpected EOF", path);
                return KRK_EIO;
            }
        }
        for (const Task& t : tasks)  // a blob's last chunk: its file is done
            if (t.off + t.len == files[t.b].length && fd[t.b] >= 0) {
                close(fd[t.b]);
                fd[t.b] = -1;
            }
        return KRK_OK;
    }
};

// File descriptors the file batches may hold open, shared by the whole process (ADVICE r04:
// every *_multi worker and every concurrent caller took the whole remaining budget for
// itself): the soft RLIMIT_NOFILE less the descriptors open at first use and a reserve for
// the rest of the process, handed out in leases.  A call waits only while every descriptor
// is leased, and then takes at least one.
class FdPool {
  public:
    uint64_t acquire(uint64_t want) {
        std::unique_lock<std::mutex> g(mu_);
        if (!init_) {
            free_ = total_ = initial_budget();
            init_ = true;
        }
        cv_.wait(g, [&] { return free_ > 0; });
        const uint64_t take = std::max<uint64_t>(1, std::min(want, free_));
        free_ -= take;
        return take;
    }
    void release(uint64_t n) {
        {
            std::lock_guard<std::mutex> g(mu_);
            free_ += n;
        }
        cv_.notify_all();
    }
    uint64_t total() {
        std::lock_guard<std::mutex> g(mu_);
        return init_ ? total_ : initial_budget();
    }

  private:
    static uint64_t initial_budget() {
        if (const char* e = KRK_OP_ENV("KRK_FD_BUDGET"))  // tests: a small budget without touching the rlimit
            if (strtoull(e, nullptr, 10) > 0) return strtoull(e, nullptr, 10);
        struct rlimit rl {};
        if (getrlimit(RLIMIT_NOFILE, &rl) != 0 || rl.rlim_cur == RLIM_INFINITY) return uint64_t(1) << 20;
        uint64_t open_now = 0;
        if (DIR* d = opendir("/proc/self/fd")) {
            while (readdir(d)) ++open_now;
            closedir(d);
        }
        const uint64_t reserve = 64 + open_now;
        return rl.rlim_cur > reserve + 16 ? rl.rlim_cur - reserve : 16;
    }
    std::mutex mu_;
    std::condition_variable cv_;
    bool init_ = false;
    uint64_t free_ = 0, total_ = 0;
};
FdPool& fd_pool() {
    static FdPool* p = new FdPool();  // leaked: used until exit
    return *p;
}
struct FdLease {
    uint64_t n;
    explicit FdLease(uint64_t want) : n(fd_pool().acquire(want)) {}
    ~FdLease() { fd_pool().release(n); }
    FdLease(const FdLease&) = delete;
    FdLease& operator=(const FdLease&) = delete;
};

struct CallStats {
    uint64_t max_live = 0;
    int windows = 0;
    int direct_windows = 0;  // windows DMA'd straight from the caller's page-locked memory
    int gather_windows = 0;  // windows gathered by the GPU from page-locked / registered caller memory
    uint64_t host_blobs = 0;
    uint64_t registered_bytes = 0;  // caller bytes registered for the gather
    double register_s = 0;          // helper-thread seconds spent registering them
    // the window loop's wall seconds and where it waited: for a free window (acquire), filling
    // windows from the source (fill: staging copies or file reads), enqueueing copies + kernels
    double loop_s = 0, acquire_s = 0, fill_s = 0, enqueue_s = 0;
    double resident = -1;  // file batches: the page-cache resident share of the sampled files
    bool direct_reads = false;  // file batches: read with O_DIRECT
    uint64_t live_at_copyout = 0;  // registry segments still registered when the results were copied out
};
thread_local CallStats t_last_call;


// The windows of one host-resident batch: the blobs not in `skip`, chunk by chunk, into the
// device's staging windows and through both kernels.  d_sums / d_dig / d_state indexed like
// the caller's blobs (sums by sums_off).  Asynchronous on the device's streams; returns once
// the last window is queued (the caller synchronises s_main / s_a / s_b).
int windows_pass(Device* D, uint64_t n, const uint64_t* lens, const int64_t* plens, const uint64_t* soff,
                 const std::vector<char>& skip, Filler& filler, uint64_t align, uint64_t cap, uint32_t* d_sums,
                 uint8_t* d_dig, uint32_t* d_state, CallStats* st, bool crc = true) {
    std::vector<uint32_t> blobs;
    for (uint64_t i = 0; i < n; ++i)
        if (!skip[i]) blobs.push_back((uint32_t)i);
    st->max_live = 0;
    st->windows = st->direct_windows = st->gather_windows = 0;
    st->loop_s = st->acquire_s = st->fill_s = st->enqueue_s = 0;
    st->direct_reads = false;
    if (blobs.empty()) return KRK_OK;
    const size_t W = window_bytes();
    const uint64_t live_cap = std::min<uint64_t>(cap, blobs.size());
    WindowSched sched(lens, blobs, W, live_cap, align);
    const size_t place = std::max<uint64_t>(align == 64 ? 16 : align, 16);  // chunk start alignment in the window
    // a window holds about W bytes, but never less than one minimum chunk (the schedule's
    // alignment) a live blob, each rounded up to `place` (a small KRK_WINDOW_MB
    // or a large KRK_LIVE_CAP made live x 64 > W + 16 x live)
    const uint64_t span = std::max<uint64_t>(W, live_cap * std::max<uint64_t>(align, 64)) + place * live_cap;
    StagingLease lease;
    int r = lease_staging(D, span, lease);
    if (r) return r;
    Pipeline& pl = *lease.p;
    hipStream_t cp = D->s_main, ks = D->s_a, kc = D->s_b;
    std::vector<WinChunk> win;
    // the gather (gather.hip): page-locked caller memory goes up in one launch a window, read
    // by the GPU -- pinned blobs as they are, pageable ones once the registry has registered
    // the pages the window reads (a dry run of the same schedule tells it which, when)
    HostRegistry* reg = filler.registry();
    if (reg) {
        WindowSched dry(lens, blobs, W, live_cap, align);
        for (int w = 0; dry.next(win); ++w)
            for (const WinChunk& c : win) reg->need(w, filler.src(c.blob, c.off), c.len);
        reg->start(std::min(4, std::max(1, host_threads_for_call() / 4)));
    }
    bool gather_ok = reg != nullptr || (filler.pinned_all() && filler.pinned_mapped());
    // The next window is built (schedule step, fill tasks, SHA jobs, CRC items) on a helper
    // thread while this one fills and enqueues the current one: with 14,336 live blobs the
    // build is ~1.7 ms a window, 16 % of a page-cache files pass that was fill-bound.  Window
    // wi always lands in staging slot wi % pl.n (Pipeline::next), so its addresses are known
    // ahead.
    struct Built {
        std::vector<Filler::Task> tasks;
        std::vector<ShaJob> jobs;
        CrcBatch items;
        size_t fill = 0;
        double build_s = 0;
    };
    std::mutex bmu;
    std::condition_variable bcv;
    std::deque<Built> ready;
    bool built_all = false, stop_build = false;
    constexpr size_t kBuildAhead = 2;
    std::thread builder([&] {
        ItemBuilder B;
        std::vector<WinChunk> win;
        for (int bi = 0;; ++bi) {
            {
                std::unique_lock<std::mutex> lk(bmu);
                bcv.wait(lk, [&] { return stop_build || ready.size() < kBuildAhead; });
                if (stop_build) return;
            }
            const double tb = wall_s();
            if (!sched.next(win)) break;
            Window& w = pl.w[bi % pl.n];
            Built bt;
            bt.tasks.reserve(win.size());
            bt.jobs.reserve(win.size());
            for (const WinChunk& c : win) {
                const uint64_t L = lens[c.blob];
                const uint64_t dev = reinterpret_cast<uint64_t>(w.dev + bt.fill);
                bt.tasks.push_back({c.blob, c.off, c.len, w.host + bt.fill});  // an empty blob too (its file is opened)
                if (c.len && crc) B.add(bt.items, dev, c.off, c.off + c.len, L, (uint64_t)plens[c.blob], soff[c.blob]);
                ShaJob j{};
                j.ptr = dev;
                j.len = c.len;
                j.prefix = c.off;
                j.out = c.blob;
                j.flags = (c.off + c.len == L ? kShaFinal : 0) | (c.off ? kShaFromState : 0);
                memcpy(j.h, kIV, sizeof kIV);
                bt.jobs.push_back(j);
                bt.fill += (c.len + place - 1) / place * place;
            }
            bt.build_s = wall_s() - tb;
            std::lock_guard<std::mutex> g(bmu);
            ready.push_back(std::move(bt));
            bcv.notify_all();
        }
        std::lock_guard<std::mutex> g(bmu);
        built_all = true;
        bcv.notify_all();
    });
    struct BuilderJoin {
        std::thread& t;
        std::mutex& mu;
        std::condition_variable& cv;
        bool& stop;
        ~BuilderJoin() {
            {
                std::lock_guard<std::mutex> g(mu);
                stop = true;
            }
            cv.notify_all();
            if (t.joinable()) t.join();
        }
    } builder_join{builder, bmu, bcv, stop_build};
    int k = 0, wi = 0;
    double t_acq = 0, t_build = 0, t_fill = 0, t_enq = 0, t_wait_build = 0;
    const double t0 = wall_s();
    while (!r) {
        Built bt;
        {
            const double tw = wall_s();
            std::unique_lock<std::mutex> lk(bmu);
            bcv.wait(lk, [&] { return !ready.empty() || built_all; });
            if (ready.empty()) break;  // every window built and run
            bt = std::move(ready.front());
            ready.pop_front();
            bcv.notify_all();
            t_wait_build += wall_s() - tw;
        }
        t_build += bt.build_s;
        const double ta = wall_s();
        r = pl.acquire(k);
        if (r) break;
        if (reg && wi >= pl.n) reg->copied(wi - pl.n);  // acquire waited for that window's copy
        const double tb = wall_s();
        t_acq += tb - ta;
        Window& w = pl.w[k];
        const std::vector<Filler::Task>& tasks = bt.tasks;
        const size_t fill = bt.fill;
        if (fill > w.cap) {  // the lease covers every window the schedule can build
            set_error(KRK_EINVAL, "metainfo windows: window of %zu bytes exceeds the %zu-byte staging lease", fill,
                      (size_t)w.cap);
            r = KRK_EINVAL;
            break;
        }
        const double tc = wall_s();
        // page-locked sources go straight from the caller's memory into the device window: a
        // DMA a chunk for a few wide chunks, else one gather launch (pinned blobs, or pageable
        // ones once registered); the others through the pinned host window
        const bool direct = !tasks.empty() && filler.pinned_all() && tasks.size() <= kDirectMaxCalls;
        const bool gather = !direct && !tasks.empty() && gather_ok && (!reg || (gather_ok = reg->ready(wi)));
        std::vector<CopyTask> dma;
        std::vector<GatherSpan> spans;
        if (direct) {
            dma.reserve(tasks.size());
            for (const Filler::Task& t : tasks)
                if (t.len) dma.push_back({w.dev + (t.dst - w.host), filler.pinned_src(t.b, t.off), (size_t)t.len});
        } else if (gather) {
            spans.reserve(tasks.size());
            for (const Filler::Task& t : tasks)
                if (t.len) spans.push_back({w.dev + (t.dst - w.host), filler.src(t.b, t.off), t.len});
        } else {
            r = filler.fill(tasks);
            if (r) break;
        }
        const double td = wall_s();
        t_fill += td - tc;
        ++st->windows;
        st->direct_windows += direct;
        st->gather_windows += gather;
        hipError_t up = hipSuccess;
        if (gather) {
            r = pl.h2d_gather(D, k, spans, cp);
            if (r) break;
        } else {
            up = direct ? pl.h2d_direct(k, dma, cp) : pl.h2d(k, fill, cp);
        }
        if (up != hipSuccess || hipStreamWaitEvent(ks, w.copied, 0) != hipSuccess ||
            (crc && hipStreamWaitEvent(kc, w.copied, 0) != hipSuccess)) {
            set_error(KRK_EHIP, "metainfo windows: staging copy failed");
            r = KRK_EHIP;
            break;
        }
        r = run_jobs(D, bt.jobs, d_dig, d_state, ks);
        if (!r && crc) r = run_items(D, bt.items, d_sums, kc);
        if (r) break;
        // the device window is free again once both kernels have read it
        pl.release(k, 0, ks);
        if (crc) pl.release(k, 1, kc);
        t_enq += wall_s() - td;
        k = pl.next(k);
        ++wi;
    }
    {
        std::lock_guard<std::mutex> g(bmu);
        stop_build = true;
    }
    bcv.notify_all();
    builder.join();
    st->max_live = sched.max_live();
    st->loop_s = wall_s() - t0;
    st->acquire_s = t_acq;
    st->fill_s = t_fill;
    st->enqueue_s = t_enq;
    if (reg) {
        st->registered_bytes = reg->registered_bytes();
        st->register_s = reg->register_seconds();
    }
    if (trace_on())
        fprintf(stderr,
                "krk_trace windows: windows=%d W=%zu max_live=%llu loop=%.3fs acquire=%.3fs build=%.3fs (ahead; "
                "waited %.3fs) fill=%.3fs enqueue=%.3fs\n",
                st->windows, W, (unsigned long long)st->max_live, wall_s() - t0, t_acq, t_build, t_wait_build, t_fill,
                t_enq);
    return r;
}

// KRK_HOST_GATHER: 0 = host-buffer calls always stage; 1 = gather pageable blobs too
// (registered for the call: host_register.hpp); unset (AUTO) = gather page-locked blobs'
// wide windows, stage pageable ones.  Measured on MI355X, C2 end to end
// (profiles/r05/bench_c2.json): pageable 100 MiB blobs registered and gathered 27.3 GB/s
// (3.8 s a pass with the registrations already made, 8.2 s registering 100 GB of fresh 4 KiB
// pages at ~20 GB/s -- registration does not scale with threads), staged 52.3 GB/s; pinned
// blobs (the files leg's krk_host_alloc sources) gathered 58.0 GB/s at 0.034 CPU-s/GB,
// staged 54.9 at 0.134.  The GPU reads 4 KiB-page registrations far slower than the
// library's huge-page pinned blocks, so AUTO registers nothing.
std::atomic<int> g_host_gather{-2};  // -2: not read yet; krk_set_host_gather
int host_gather_mode() {
    int m = g_host_gather.load(std::memory_order_relaxed);
    if (m != -2) return m;
    const char* e = KRK_OP_ENV("KRK_HOST_GATHER");
    int expect = -2;
    g_host_gather.compare_exchange_strong(expect, e ? (atoi(e) > 0 ? 1 : 0) : -1);
    return g_host_gather.load();
}

// The MemFiller of a host-buffer call: page-locked blobs DMA'd or gathered as they are,
// pageable ones registered for the gather (KRK_HOST_GATHER) or staged.
void setup_mem_filler(MemFiller& f, const krk_blob* blobs, uint64_t n, const std::vector<char>& on_host, Device* D) {
    // KRK_PINNED_DIRECT=0 stages pinned sources too (A/B)
    static const bool allow_direct = !KRK_AB_ENV("KRK_PINNED_DIRECT") || atoi(KRK_AB_ENV("KRK_PINNED_DIRECT")) != 0;
    const int gm = host_gather_mode();
    f.pinned = allow_direct;
    uint64_t first = n;
    for (uint64_t i = 0; i < n; ++i) {
        if (on_host[i] || !blobs[i].length) continue;
        if (first == n) first = i;
        if (f.pinned && !host_pinned(blobs[i].data, blobs[i].length)) f.pinned = false;
    }
    if (first == n) return;
    f.mapped = f.pinned && gm != 0;  // every windowed blob at its host address
    MappedAtHost at_host;
    for (uint64_t i = first; f.mapped && i < n; ++i)
        if (!on_host[i]) f.mapped = at_host(blobs[i].data, blobs[i].length);
    if (!f.pinned && gm == 1) {
        std::vector<std::pair<uintptr_t, uintptr_t>> ranges;
        for (uint64_t i = 0; i < n; ++i)
            if (!on_host[i] && blobs[i].length) {
                const uintptr_t a = reinterpret_cast<uintptr_t>(blobs[i].data);
                ranges.push_back({a, a + blobs[i].length});
            }
        f.reg = std::make_unique<HostRegistry>(std::move(ranges));
        f.gather_stream = D->s_main;  // windows_pass's copy stream
    }
}

// Every host-buffer entry point, once its streams have drained and before any copy-out: the
// registry's helpers stopped and every caller range it registered released.  A HIP copy whose
// destination starts in a registered page and runs past it is refused ("copy-out failed:
// invalid argument"): the registry rounds each blob out to whole pages,
// so with the last windows' segments still registered an output array -- or any heap buffer
// -- sharing a page with a small blob was such a destination.  The count left registered is
// kept for krk_windows_last_copyout (0 by construction).
void release_caller_pages(MemFiller& f, CallStats* st) {
    if (!f.reg) return;
    f.reg->finish(f.gather_stream);
    st->live_at_copyout = f.reg->live_segments();
}

// A call's results to the caller's host memory, refused (not attempted) while the call still
// holds a registration touching the destination's pages.
int copy_out(void* dst, const void* src_dev, size_t n, const HostRegistry* reg, const char* what) {
    if (!n) return KRK_OK;
    KRK_CHECK(!reg || !reg->overlaps_live(dst, n), KRK_EINVAL,
              "%s copy-out: destination shares a page the call still holds registered", what);
    const hipError_t e = hipMemcpy(dst, src_dev, n, hipMemcpyDeviceToHost);
    KRK_CHECK(e == hipSuccess, KRK_EHIP, "%s copy-out failed: %s", what, hipGetErrorString(e));
    return KRK_OK;
}

// KRK_LIVE_CAP: overrides the window's live-stream cap (tests, sweeps).
uint64_t live_cap_for(Device* D) {
    const char* e = KRK_OP_ENV("KRK_LIVE_CAP");
    const uint64_t v = e ? strtoull(e, nullptr, 10) : 0;
    return v ? v : window_stream_cap(D);
}

// A file batch read O_DIRECT (cold: bound by the disk) needs no more live files than it takes
// the windows' SHA-256 streams to outrun the host link -- h2d over the eight-lane per-stream
// rate, ~970 on MI355X, rounded up to 64: every live file beyond that only shrinks each
// file's chunk of a window, and so the disk's requests.  Cold 32 GiB leg on one box
// (profiles/r06/bench_files_live.json): 3,734 live 12.4 GB/s, 2,048 14.7, 1,024 15.2, 512
// 15.2, 256 13.5 (the streams bind there), the reference's two reads 14.3.  KRK_LIVE_CAP wins.
uint64_t direct_live_cap(Device* D) {
    if (KRK_OP_ENV("KRK_LIVE_CAP")) return live_cap_for(D);
    const Rates R = planner_rates(D);
    const double per_stream = R.stream[0] > 0 ? R.stream[0] : 58e6;
    const double link = R.h2d > 0 ? R.h2d : 56e9;
    const uint64_t need = (uint64_t)(link / per_stream) + 1;
    return std::min(live_cap_for(D), std::max<uint64_t>(256, (need + 63) / 64 * 64));
}


}  // namespace

}  // namespace krk

using namespace krk;

// The device results, the host offload's results and the caller's arrays of one call.
namespace {
struct Outputs {
    uint8_t* d_dig = nullptr;
    uint32_t *d_state = nullptr, *d_sums = nullptr;
    DevMem mem;
    int alloc(uint64_t n, uint64_t hi) {
        KRK_HIP(mem.alloc(&d_dig, n * 32));
        KRK_HIP(mem.alloc(&d_state, n * 32));
        KRK_HIP(mem.alloc(&d_sums, std::max<uint64_t>(hi, 1) * 4));
        KRK_HIP(hipMemset(d_sums, 0, std::max<uint64_t>(hi, 1) * 4));
        return KRK_OK;
    }
};
}  // namespace

extern "C" {

int krk_window_stream_cap(uint64_t* cap) {
    KRK_CHECK(cap, KRK_EINVAL, "cap is NULL");
    KRK_DEVICE(D);
    *cap = window_stream_cap(D);
    return KRK_OK;
}

struct krk_window_sched {
    std::vector<uint64_t> lens;
    std::unique_ptr<WindowSched> s;
    std::vector<WinChunk> win;
};

int krk_window_sched_new(const uint64_t* lengths, uint64_t n, uint64_t window_bytes, uint64_t live_cap,
                         krk_window_sched** out) {
    KRK_CHECK(out && (n == 0 || lengths), KRK_EINVAL, "window_sched_new: null argument");
    KRK_CHECK(window_bytes >= 64 && live_cap >= 1, KRK_EINVAL, "window bytes >= 64 and live cap >= 1");
    KRK_CHECK(n <= 0xFFFFFFFFull, KRK_EINVAL, "more than 2^32 blobs");
    auto* w = new krk_window_sched();
    w->lens.assign(lengths, lengths + n);
    std::vector<uint32_t> all(n);
    for (uint64_t i = 0; i < n; ++i) all[i] = (uint32_t)i;
    w->s = std::make_unique<WindowSched>(w->lens.data(), std::move(all), window_bytes, live_cap);
    *out = w;
    return KRK_OK;
}

int krk_window_sched_next(krk_window_sched* w, uint32_t* blobs, uint64_t* offsets, uint64_t* lengths, uint64_t cap,
                          uint64_t* n_out) {
    KRK_CHECK(w && n_out, KRK_EINVAL, "window_sched_next: null argument");
    if (!w->s->next(w->win)) {
        *n_out = 0;
        return KRK_OK;
    }
    *n_out = w->win.size();
    KRK_CHECK(w->win.size() <= cap, KRK_ERANGE, "window has %zu chunks, capacity %llu", w->win.size(),
              (unsigned long long)cap);
    for (size_t k = 0; k < w->win.size(); ++k) {
        if (blobs) blobs[k] = w->win[k].blob;
        if (offsets) offsets[k] = w->win[k].off;
        if (lengths) lengths[k] = w->win[k].len;
    }
    return KRK_OK;
}

int krk_window_sched_drop(krk_window_sched* w, uint32_t blob, uint64_t* offset) {
    KRK_CHECK(w && offset, KRK_EINVAL, "window_sched_drop: null argument");
    KRK_CHECK(w->s->drop(blob, offset), KRK_EINVAL, "window_sched_drop: blob %u is neither live nor waiting", blob);
    return KRK_OK;
}

int krk_window_sched_set_chunk_cap(krk_window_sched* w, uint64_t max_chunk) {
    KRK_CHECK(w && max_chunk >= 64, KRK_EINVAL, "window_sched_set_chunk_cap: null schedule or cap < 64");
    w->s->set_max_chunk(max_chunk);
    return KRK_OK;
}

void krk_window_sched_free(krk_window_sched* w) { delete w; }

int krk_metainfo_digest_host(const krk_blob* blobs, uint64_t n, uint32_t* sums_host, uint8_t* digests_host) {
    KRK_DEVICE(D);
    int r = validate_blobs(blobs, n);
    if (r) return r;
    if (!n) return KRK_OK;
    KRK_CHECK(digests_host, KRK_EINVAL, "digests_host is NULL");
    uint64_t lo, hi;
    sums_span(blobs, n, &lo, &hi);
    KRK_CHECK(hi == lo || sums_host, KRK_EINVAL, "sums_host is NULL");
    std::vector<uint64_t> lens(n), soff(n);
    std::vector<int64_t> plens(n);
    for (uint64_t i = 0; i < n; ++i) {
        lens[i] = blobs[i].length;
        plens[i] = blobs[i].piece_length;
        soff[i] = blobs[i].sums_offset;
    }
    // SHA-256 host offload (KRK_OFFLOAD_AUTO by default): the planner's blobs are hashed and
    // piece-summed in place on host threads and never cross the host link.
    std::vector<char> on_host(n, 0);
    std::vector<uint32_t> host;
    const int off_t = offload_threads(kOffHostWhole);
    if (off_t > 0) {
        host = offload_plan(lens.data(), n, off_t, planner_rates(D), nullptr, nullptr, kOffHostWhole);
        for (uint32_t i : host) on_host[i] = 1;
    }
    Outputs o;
    r = o.alloc(n, hi);
    if (r) return r;
    std::vector<uint8_t> host_dig(32 * host.size());
    std::vector<uint64_t> host_sums_off(host.size() + 1, 0);
    for (size_t j = 0; j < host.size(); ++j)
        host_sums_off[j + 1] = host_sums_off[j] + krk_num_pieces(lens[host[j]], plens[host[j]]);
    std::vector<uint32_t> host_sums(host_sums_off.back());
    std::thread host_th;
    if (!host.empty())
        host_th = std::thread([&] {
            std::vector<const uint8_t*> p(host.size());
            std::vector<uint64_t> l(host.size()), pl(host.size());
            std::vector<uint32_t*> so(host.size());
            for (size_t j = 0; j < host.size(); ++j) {
                p[j] = blobs[host[j]].data;
                l[j] = lens[host[j]];
                pl[j] = (uint64_t)plens[host[j]];
                so[j] = host_sums.data() + host_sums_off[j];
            }
            offload_whole_host(p, l, pl, so, off_t, host_dig.data());
        });
    struct Joiner {
        std::thread& t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } joiner{host_th};
    // The copy threads and the offload's threads share the process's CPU budget: above it
    // a CPU quota throttles the whole process.
    struct ShareGuard {
        int saved;
        ~ShareGuard() { t_host_share = saved; }
    } share_guard{t_host_share};
    if (!host.empty()) t_host_share = std::max(4, host_threads_for_call() - off_t);
    MemFiller filler(blobs);
    setup_mem_filler(filler, blobs, n, on_host, D);
    CallStats st;
    r = windows_pass(D, n, lens.data(), plens.data(), soff.data(), on_host, filler, 64, live_cap_for(D), o.d_sums,
                     o.d_dig, o.d_state, &st);
    if (!r && (hipStreamSynchronize(D->s_a) != hipSuccess || hipStreamSynchronize(D->s_b) != hipSuccess ||
               hipStreamSynchronize(D->s_main) != hipSuccess)) {
        set_error(KRK_EHIP, "metainfo_digest_host: sync failed");
        r = KRK_EHIP;
    }
    release_caller_pages(filler, &st);
    if (!r) r = copy_out(digests_host, o.d_dig, n * 32, filler.reg.get(), "digest");
    if (!r && hi > lo) r = copy_out(sums_host + lo, o.d_sums + lo, (hi - lo) * 4, filler.reg.get(), "sums");
    if (host_th.joinable()) host_th.join();
    for (size_t q = 0; !r && q < host.size(); ++q) {
        memcpy(digests_host + 32 * (size_t)host[q], &host_dig[32 * q], 32);
        if (host_sums_off[q + 1] > host_sums_off[q])
            memcpy(sums_host + soff[host[q]], &host_sums[host_sums_off[q]], (host_sums_off[q + 1] - host_sums_off[q]) * 4);
    }
    st.host_blobs = host.size();
    t_last_call = st;
    return r;
}

// Whole-blob SHA-256 of host buffers (the Digester over many uploads at once): the same
// windows and schedule as krk_metainfo_digest_host without the CRC launches, and the
// planner's blobs hashed in place on host threads (KRK_OFFLOAD_HOST_SHA).
int krk_sha256_host(const uint8_t* const* data_host, const uint64_t* lengths, uint64_t n, uint8_t* digests_host) {
    KRK_DEVICE(D);
    if (!n) return KRK_OK;
    KRK_CHECK(data_host && lengths && digests_host, KRK_EINVAL, "sha256_host: null argument");
    for (uint64_t i = 0; i < n; ++i)
        KRK_CHECK(lengths[i] == 0 || data_host[i], KRK_EINVAL, "blob %llu: data is NULL", (unsigned long long)i);
    std::vector<krk_blob> blobs(n);
    std::vector<int64_t> plens(n, 1);
    std::vector<uint64_t> soff(n, 0);
    for (uint64_t i = 0; i < n; ++i) blobs[i] = krk_blob{data_host[i], lengths[i], 1, 0};
    std::vector<char> on_host(n, 0);
    std::vector<uint32_t> host;
    const int off_t = offload_threads(kOffHostSha);
    if (off_t > 0) {
        host = offload_plan(lengths, n, off_t, planner_rates(D), nullptr, nullptr, kOffHostSha);
        for (uint32_t i : host) on_host[i] = 1;
    }
    uint8_t* d_dig = nullptr;
    uint32_t* d_state = nullptr;
    DevMem mem;
    KRK_HIP(mem.alloc(&d_dig, n * 32));
    KRK_HIP(mem.alloc(&d_state, n * 32));
    std::vector<uint8_t> host_dig(32 * host.size());
    std::thread host_th;
    if (!host.empty())
        host_th = std::thread([&] {
            std::vector<const uint8_t*> p(host.size());
            std::vector<uint64_t> l(host.size());
            for (size_t j = 0; j < host.size(); ++j) {
                p[j] = data_host[host[j]];
                l[j] = lengths[host[j]];
            }
            offload_hash_host(p, l, off_t, host_dig.data());
        });
    struct Joiner {
        std::thread& t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } joiner{host_th};
    struct ShareGuard {
        int saved;
        ~ShareGuard() { t_host_share = saved; }
    } share_guard{t_host_share};
    if (!host.empty()) t_host_share = std::max(4, host_threads_for_call() - off_t);
    MemFiller filler(blobs.data());
    setup_mem_filler(filler, blobs.data(), n, on_host, D);
    CallStats st;
    int r = windows_pass(D, n, lengths, plens.data(), soff.data(), on_host, filler, 64, live_cap_for(D), nullptr,
                         d_dig, d_state, &st, /*crc=*/false);
    if (!r && (hipStreamSynchronize(D->s_a) != hipSuccess || hipStreamSynchronize(D->s_main) != hipSuccess)) {
        set_error(KRK_EHIP, "sha256_host: sync failed");
        r = KRK_EHIP;
    }
    release_caller_pages(filler, &st);
    if (!r) r = copy_out(digests_host, d_dig, n * 32, filler.reg.get(), "digest");
    if (host_th.joinable()) host_th.join();
    for (size_t q = 0; !r && q < host.size(); ++q) memcpy(digests_host + 32 * (size_t)host[q], &host_dig[32 * q], 32);
    st.host_blobs = host.size();
    t_last_call = st;
    return r;
}

// The page-cache resident share of a file batch, from up to 64 evenly spaced files' first
// 16 MiB (mmap + mincore: no page is read).  -1 when none could be sampled.
static double files_resident_fraction(const krk_file_blob* files, uint64_t n) {
    const uint64_t step = std::max<uint64_t>(1, n / 64);
    const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
    uint64_t in = 0, all = 0;
    std::vector<unsigned char> vec;
    for (uint64_t i = 0; i < n; i += step) {
        const size_t len = (size_t)std::min<uint64_t>(files[i].length, 16ull << 20);
        if (!len) continue;
        const int fd = open(files[i].path, O_RDONLY | O_CLOEXEC);
        if (fd < 0) continue;  // the pass reports it
        void* m = mmap(nullptr, len, PROT_READ, MAP_SHARED, fd, 0);
        close(fd);
        if (m == MAP_FAILED) continue;
        vec.assign((len + pg - 1) / pg, 0);
        if (mincore(m, len, vec.data()) == 0) {
            for (unsigned char c : vec) in += c & 1;
            all += vec.size();
        }
        munmap(m, len);
    }
    return all ? (double)in / (double)all : -1.0;
}

int krk_metainfo_digest_files(const krk_file_blob* files, uint64_t n, uint32_t* sums_host, uint8_t* digests_host) {
    KRK_DEVICE(D);
    if (!n) return KRK_OK;
    KRK_CHECK(files && digests_host, KRK_EINVAL, "metainfo_digest_files: null argument");
    std::vector<uint64_t> lens(n), soff(n);
    std::vector<int64_t> plens(n);
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint64_t i = 0; i < n; ++i) {
        KRK_CHECK(files[i].path, KRK_EINVAL, "file %llu: path is NULL", (unsigned long long)i);
        KRK_CHECK(files[i].piece_length > 0, KRK_EINVAL, "piece length must be positive");
        lens[i] = files[i].length;
        plens[i] = files[i].piece_length;
        soff[i] = files[i].sums_offset;
        const uint64_t np = krk_num_pieces(lens[i], plens[i]);
        KRK_CHECK(soff[i] + np <= 0xFFFFFFFFull, KRK_EINVAL, "sums index exceeds 2^32 in one call");
        if (np) {
            lo = std::min(lo, soff[i]);
            hi = std::max(hi, soff[i] + np);
        }
    }
    if (lo > hi) lo = hi = 0;
    KRK_CHECK(hi == lo || sums_host, KRK_EINVAL, "sums_host is NULL");
    // Host offload (AUTO by default): the planner's files are read, hashed and piece-summed
    // by host threads in one pass each and never cross the host link.
    // A batch mostly out of the page cache (the residency sample) is bound by the disk,
    // wherever its bytes are hashed: under AUTO, host threads would read the same disk and
    // take CPU from the window readers (cold 32 GiB leg: AUTO 13.4 GB/s against 14.8
    // GPU-only, profiles/r05/bench_files.json), so such a batch stays on the windows -- and
    // is read with O_DIRECT (below).
    std::vector<char> on_host(n, 0);
    std::vector<uint32_t> host;
    int off_t = offload_threads(kOffHostWhole);
    const double resident = files_resident_fraction(files, n);
    const bool cold = resident >= 0 && resident < 0.5;
    if (cold && offload_auto()) off_t = 0;
    if (off_t > 0) {
        host = offload_plan(lens.data(), n, off_t, planner_rates(D), nullptr, nullptr, kOffHostFiles);
        for (uint32_t i : host) on_host[i] = 1;
    }
    Outputs o;
    int r = o.alloc(n, hi);
    if (r) return r;
    std::vector<uint8_t> host_dig(32 * host.size());
    std::vector<uint64_t> host_sums_off(host.size() + 1, 0);
    for (size_t j = 0; j < host.size(); ++j)
        host_sums_off[j + 1] = host_sums_off[j] + krk_num_pieces(lens[host[j]], plens[host[j]]);
    std::vector<uint32_t> host_sums(host_sums_off.back());
    int host_rc = KRK_OK;
    std::string host_err;
    std::thread host_th;
    if (!host.empty())
        host_th = std::thread([&] {
            std::vector<const char*> p(host.size());
            std::vector<uint64_t> l(host.size()), pl(host.size());
            std::vector<uint32_t*> so(host.size());
            for (size_t j = 0; j < host.size(); ++j) {
                p[j] = files[host[j]].path;
                l[j] = lens[host[j]];
                pl[j] = (uint64_t)plens[host[j]];
                so[j] = host_sums.data() + host_sums_off[j];
            }
            host_rc = offload_whole_files(p, l, pl, so, off_t, host_dig.data());
            if (host_rc) host_err = t_err;
        });
    struct Joiner {
        std::thread& t;
        ~Joiner() {
            if (t.joinable()) t.join();
        }
    } joiner{host_th};
    struct ShareGuard {
        int saved;
        ~ShareGuard() { t_host_share = saved; }
    } share_guard{t_host_share};
    if (!host.empty()) t_host_share = std::max(4, host_threads_for_call() - off_t);
    // O_DIRECT reads (Linux AIO, a window's chunks queued at once): KRK_FILE_DIRECT=1 / 0
    // force them on / off; by default a cold batch takes them (no page-cache copy, a deep
    // disk queue from one thread: 16.3 GB/s against 11.7 for 16 threads' page-cache preads
    // of the same window chunks, profiles/r05/disk_probe_aio.jsonl) and a cached one reads
    // the page cache.
    const char* fd_env = KRK_OP_ENV("KRK_FILE_DIRECT");
    const bool direct = fd_env ? atoi(fd_env) > 0 : cold;
    FileFiller filler(files, n, direct);
    CallStats st;
    // at most as many live blobs as this call holds file descriptors (a lease of the
    // process's budget, shared with every other file batch running now)
    FdLease fds(std::min<uint64_t>(direct ? direct_live_cap(D) : live_cap_for(D), n));
    r = windows_pass(D, n, lens.data(), plens.data(), soff.data(), on_host, filler, direct ? 4096 : 64, fds.n,
                     o.d_sums, o.d_dig, o.d_state, &st);
    st.resident = resident;
    st.direct_reads = direct;
    // drain what was queued even after a read error (the windows' kernels read the buffers)
    const bool synced = hipStreamSynchronize(D->s_a) == hipSuccess && hipStreamSynchronize(D->s_b) == hipSuccess &&
                        hipStreamSynchronize(D->s_main) == hipSuccess;
    if (!r && !synced) {
        set_error(KRK_EHIP, "metainfo_digest_files: sync failed");
        r = KRK_EHIP;
    }
    if (!r && hipMemcpy(digests_host, o.d_dig, n * 32, hipMemcpyDeviceToHost) != hipSuccess) {
        set_error(KRK_EHIP, "digest copy-out failed");
        r = KRK_EHIP;
    }
    if (!r && hi > lo && hipMemcpy(sums_host + lo, o.d_sums + lo, (hi - lo) * 4, hipMemcpyDeviceToHost) != hipSuccess) {
        set_error(KRK_EHIP, "sums copy-out failed");
        r = KRK_EHIP;
    }
    if (host_th.joinable()) host_th.join();
    if (!r && host_rc) {
        t_err = host_err;
        r = host_rc;
    }
    for (size_t q = 0; !r && q < host.size(); ++q) {
        memcpy(digests_host + 32 * (size_t)host[q], &host_dig[32 * q], 32);
        if (host_sums_off[q + 1] > host_sums_off[q])
            memcpy(sums_host + soff[host[q]], &host_sums[host_sums_off[q]], (host_sums_off[q + 1] - host_sums_off[q]) * 4);
    }
    st.host_blobs = host.size();
    t_last_call = st;
    return r;
}

int krk_windows_last_call(uint64_t* max_live, int* windows, uint64_t* host_blobs) {
    if (max_live) *max_live = t_last_call.max_live;
    if (windows) *windows = t_last_call.windows;
    if (host_blobs) *host_blobs = t_last_call.host_blobs;
    return KRK_OK;
}

int krk_windows_last_copyout(uint64_t* live_registered) {
    KRK_CHECK(live_registered, KRK_EINVAL, "live_registered is NULL");
    *live_registered = t_last_call.live_at_copyout;
    return KRK_OK;
}

int krk_windows_last_direct(int* direct_windows) {
    KRK_CHECK(direct_windows, KRK_EINVAL, "direct_windows is NULL");
    *direct_windows = t_last_call.direct_windows;
    return KRK_OK;
}

int krk_set_host_gather(int mode) {
    KRK_CHECK(mode >= -1 && mode <= 1, KRK_EINVAL, "host gather mode %d outside -1 (auto), 0, 1", mode);
    g_host_gather.store(mode);
    return KRK_OK;
}

int krk_windows_last_gather(int* gather_windows, uint64_t* registered_bytes, double* register_seconds) {
    if (gather_windows) *gather_windows = t_last_call.gather_windows;
    if (registered_bytes) *registered_bytes = t_last_call.registered_bytes;
    if (register_seconds) *register_seconds = t_last_call.register_s;
    return KRK_OK;
}

int krk_windows_last_phases(double* loop_s, double* acquire_s, double* fill_s, double* enqueue_s,
                            double* resident, int* direct_reads) {
    if (resident) *resident = t_last_call.resident;
    if (direct_reads) *direct_reads = t_last_call.direct_reads ? 1 : 0;
    if (loop_s) *loop_s = t_last_call.loop_s;
    if (acquire_s) *acquire_s = t_last_call.acquire_s;
    if (fill_s) *fill_s = t_last_call.fill_s;
    if (enqueue_s) *enqueue_s = t_last_call.enqueue_s;
    return KRK_OK;
}

}  // extern "C"
