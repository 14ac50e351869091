// engine.cpp -- the per-device submission engine behind the streaming entry points
// (krk_digester_*, krk_piece_stream_*, krk_crc32_update).
//
// The reference calls these from many goroutines at once (SURVEY.md 8(b)
// "Threading": origin/blobserver/uploader.go:75 and lib/store/ca_store.go:119 run a
// Digester per upload / cache fill, lib/torrent/storage/agentstorage/torrent.go:182
// a PieceHash per received piece).  One launch per call would serialise them and
// leave the chip empty, so every device context owns:
//
//  * a pool of fixed-size pinned staging slots, each with a device mirror, under a
//    HARD pinned-bytes cap (KRK_SLOT_POOL_MB, krk_engine_set_pool_cap): a caller copies
//    its bytes into a slot on its own thread and issues the slot's H2D on the engine's
//    copy stream; at the cap it waits for a release (backpressure).  Slots are held
//    only by requests in flight, which the engine always completes -- an owner keeps
//    its partial data in its own host buffer between calls -- so the wait ends;
//  * two queues (SHA-256, CRC-32), each with a dispatcher thread that coalesces the
//    pending requests into ONE launch and a completer thread that retires launches in
//    order, so up to kMaxInflight launches per queue are on the device at once and the
//    host's job building, result copies and wake-ups overlap the kernels.
//
// SHA-256 (Digester): every GPU digester owns a row of the engine's HBM state table
// (8 words) and digest table (32 B).  A request's job starts from that row
// (kShaFromState, or the IV for the first request) and writes it back, so a
// digester's requests chain through the device in stream order: the dispatcher takes
// at most one request per digester per launch and may launch the next batch behind the
// running one without waiting for its results.  It forms that next batch once every
// digester of the running batch has its next request queued, or shortly before the
// running batch is due to end (estimated from the measured per-byte time of earlier
// batches), so a digester whose next request arrives a little late still makes the
// next launch.  Only final requests copy anything back (their digests).
//
// CRC-32 (PieceHash / piece streams): requests carry no state: each piece portion is
// hashed as an independent message and the owner's piece sums are folded on the
// completer thread with the GF(2) combine crc(A||B) = crc(A) * x^(8|B|) ^ crc(B)
// (crc_math.hpp), in submission order, so any number of a stream's requests may share
// a launch and a stream's piece end need not be known when its bytes are submitted.
//
// Host crossovers: a digester created while few digesters are live
// runs SHA-NI on its caller's thread (one core ~2 GB/s vs one GPU stream ~59 MB/s);
// crc32.Update calls of at most KRK_CRC_HOST_MAX bytes run on the caller's thread
// (no PCIe round trip for a small write).  Both are product code (host_meta.cpp).
#include <sched.h>

#include <chrono>
#include <condition_variable>
#include <deque>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "runtime.hpp"

namespace krk {

void host_sha256_blocks(uint32_t h[8], const uint8_t* p, size_t nblocks);
void host_sha256_final(const uint32_t h[8], uint64_t absorbed, const uint8_t* tail, size_t n, uint8_t out[32]);
uint32_t host_crc32_update(uint32_t crc, const uint8_t* p, size_t n);

namespace {

using Clock = std::chrono::steady_clock;

// a knob's value (KRK_OP_ENV / KRK_AB_ENV, knobs.hpp) as a positive size, else dflt
size_t env_size(const char* v, size_t dflt) {
    if (!v || !*v) return dflt;
    const unsigned long long x = strtoull(v, nullptr, 10);
    return x ? (size_t)x : dflt;
}

// ------------------------------------------------------------------ slots
struct Slot {
    uint8_t* host = nullptr;      // pinned, mapped into the device's address space
    const uint8_t* mapped = nullptr;  // `host` as the device addresses it (zero-copy reads)
    uint8_t* dev = nullptr;       // device mirror (CRC requests are copied here)
    hipEvent_t h2d = nullptr;  // the last H2D of this slot
};

class SlotPool {
  public:
    size_t S = 0;  // bytes per slot (multiple of 64)

    int numa = -1;  // the node the slots' pinned pages come from (-1: wherever the growing thread runs)

    void init(size_t slot_bytes, size_t cap_bytes, int numa_node = -1) {
        S = slot_bytes;
        numa = numa_node;
        set_cap(cap_bytes);
    }

    // The hard cap on pinned bytes (at least one chunk).  Lowering it never frees
    // slots already allocated; it stops further growth.
    void set_cap(size_t cap_bytes) {
        {
            std::lock_guard<std::mutex> g(mu_);
            cap_ = std::max(cap_bytes, S * kPerChunk);
        }
        cv_.notify_all();
    }

    // A free slot: grows the pool one chunk at a time while under the cap, else waits
    // for a release (backpressure).  Call with the owning device current.
    Slot* acquire(int* rc) {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            if (!free_.empty()) {
                Slot* s = free_.back();
                free_.pop_back();
                *rc = KRK_OK;
                return s;
            }
            if (allocated_ + S * kPerChunk <= cap_) {
                *rc = grow();
                if (*rc) return nullptr;
                continue;
            }
            ++waits_;
            cv_.wait(lk);
        }
    }

    // A slot for an owner to fill in place between calls, only while more than `reserve`
    // slots stay free or growable: the reserve is left to submissions (which block), so
    // slots held by idle owners can never starve the requests that release slots.
    Slot* try_acquire(size_t reserve) {
        std::lock_guard<std::mutex> g(mu_);
        const size_t growable = cap_ > allocated_ ? (cap_ - allocated_) / S : 0;
        if (free_.size() + growable <= reserve) return nullptr;
        if (free_.empty() && grow() != KRK_OK) return nullptr;
        Slot* s = free_.back();
        free_.pop_back();
        return s;
    }
    size_t reserve() {
        std::lock_guard<std::mutex> g(mu_);
        return std::max<size_t>(kPerChunk, cap_ / S / 4);
    }

    void release(Slot* s) {
        if (!s) return;
        {
            std::lock_guard<std::mutex> g(mu_);
            free_.push_back(s);
        }
        cv_.notify_one();
    }

    size_t pinned_bytes() {
        std::lock_guard<std::mutex> g(mu_);
        return allocated_;
    }
    size_t cap() {
        std::lock_guard<std::mutex> g(mu_);
        return cap_;
    }
    uint64_t waits() {
        std::lock_guard<std::mutex> g(mu_);
        return waits_;
    }

    void destroy() {
        std::lock_guard<std::mutex> g(mu_);
        for (auto& c : chunks_)
            for (int i = 0; i < kPerChunk; ++i)
                if (c[i].h2d) {
                    hipEventSynchronize(c[i].h2d);
                    hipEventDestroy(c[i].h2d);
                }
        for (void* p : host_) hipHostFree(p);
        for (void* p : dev_) hipFree(p);
        chunks_.clear();
        host_.clear();
        dev_.clear();
        free_.clear();
        allocated_ = 0;
    }

  private:
    static constexpr int kPerChunk = 16;
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<Slot*> free_;
    std::vector<std::unique_ptr<Slot[]>> chunks_;
    std::vector<void*> host_, dev_;
    size_t allocated_ = 0;
    size_t cap_ = 0;
    uint64_t waits_ = 0;

    // With mu_ held.  Everything is created before anything is published, and a
    // failure undoes what this call made: the pool never holds a half-built chunk.
    int grow() {
        const size_t bytes = S * kPerChunk;
        hipEvent_t ev[kPerChunk] = {};
        for (int i = 0; i < kPerChunk; ++i) {
            const hipError_t e = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
            if (e != hipSuccess) {
                for (int j = 0; j < i; ++j) hipEventDestroy(ev[j]);
                set_error(KRK_EHIP, "engine: slot events: %s", hipGetErrorString(e));
                return KRK_EHIP;
            }
        }
        void *h = nullptr, *d = nullptr, *hm = nullptr;
        // coherent: the SHA-256 kernel reads a slot straight over PCIe (no H2D copy), and a
        // reused slot must never be served from a stale GPU cache line
        on_numa_node(numa, [&] {
            if (hipHostMalloc(&h, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) h = nullptr;
            else memset(h, 0, bytes);  // first touch on that node
        });
        if (h && hipHostGetDevicePointer(&hm, h, 0) != hipSuccess) hm = nullptr;
        if (h && hm && hipMalloc(&d, bytes) != hipSuccess) d = nullptr;
        if (!h || !hm || !d) {
            if (h) hipHostFree(h);
            for (auto& e : ev) hipEventDestroy(e);
            set_error(KRK_ENOMEM, "engine: %s staging slots (%zu bytes)", h ? "device" : "pinned host", bytes);
            return KRK_ENOMEM;
        }
        std::unique_ptr<Slot[]> c(new Slot[kPerChunk]);
        for (int i = 0; i < kPerChunk; ++i) {
            c[i].host = static_cast<uint8_t*>(h) + i * S;
            c[i].mapped = static_cast<const uint8_t*>(hm) + i * S;
            c[i].dev = static_cast<uint8_t*>(d) + i * S;
            c[i].h2d = ev[i];
            free_.push_back(&c[i]);
        }
        host_.push_back(h);
        dev_.push_back(d);
        chunks_.push_back(std::move(c));
        allocated_ += bytes;
        return KRK_OK;
    }
};

// ------------------------------------------------------------------ requests
struct Waiter {
    std::mutex mu;
    std::condition_variable cv;
};

struct Req {
    Slot* slot = nullptr;  // released when the request completes
    uint64_t len = 0;
    uint64_t seq = 0;             // order of the slot's H2D on the copy stream
    const void* owner = nullptr;  // ordering key (SHA: one request per owner per launch)
    Waiter* w = nullptr;
    Clock::time_point t_submit;
    // SHA: the owner's state-table row, bytes absorbed before this request; final =
    // pad and write the digest (the state row is left as it was: no reset).
    uint32_t row = 0;
    uint64_t prefix = 0;
    bool final = false;
    uint8_t digest[32] = {};
    // CRC: stream offset of the slot's first byte and the piece length (0: the request
    // is one portion); crcs[k] = crc32 of portion k as an independent message.
    uint64_t off = 0;
    uint64_t P = 0;
    std::vector<uint32_t> crcs;
    void (*on_done)(Req*) = nullptr;  // runs on the completer thread, in FIFO order
    void* ctx = nullptr;
    int rc = KRK_OK;
    std::string err;
    bool done = false;
};

constexpr int kMaxInflight = 8;           // result buffers per queue (launches on the device at once <= this)
int g_inflight = 3;                       // launches per queue on the device at once (KRK_ENGINE_INFLIGHT)
// Requests per digester / piece stream in flight (KRK_OWNER_INFLIGHT).  With 512 KiB
// slots a launch of 256 streams is ~9 ms, so 8 in flight keep ~70 ms of each owner's
// bytes ahead of the device: an owner whose writer thread was descheduled for a while
// still makes the next launch.
size_t g_owner_inflight = 8;
constexpr uint32_t kStateRows = 65536;    // GPU digesters per device (state + digest rows)
constexpr uint64_t kMaxCrcBatchBytes = 4ull << 30;

struct Inflight {
    std::vector<Req*> batch;
    hipEvent_t done = nullptr;
    int rc = KRK_OK;
    std::string err;
    int out_i = -1;  // the queue's pinned result buffer this launch writes
    hipEvent_t gathered = nullptr;  // kSrcGather: the batch's slots are in their device mirrors
    uint64_t max_len = 0;
    Clock::time_point t_launch;
    char reason = '-';                    // trace: why the batch was formed
    size_t depth = 0, left_queued = 0;    // trace: launches on the device, requests left
    int64_t missing = 0;
    double est = 0;                       // trace: the per-byte time estimate when formed
    // SHA: digest rows [row0, row0 + nrows) copied back (final requests)
    uint32_t row0 = 0, nrows = 0;
    // CRC: request i's portion CRCs at base[i] .. base[i + 1] of the results
    std::vector<uint64_t> base;
    uint64_t total = 0;
};

struct Queue {
    std::mutex mu;
    std::condition_variable cv;       // dispatcher: requests, a retired launch, stop
    std::condition_variable cv_done;  // completer: a launch to retire
    std::deque<Req*> q;
    std::deque<Inflight*> inflight;   // launch order
    bool stop = false, disp_exited = false;
    bool dispatching = false;  // a batch is between take_batch and publish (one at a time: stream order = owner order)
    std::thread th, th_done;
    hipStream_t s = nullptr;
    uint8_t* out[kMaxInflight] = {};  // pinned result buffers, grown on demand
    size_t out_cap[kMaxInflight] = {};
    bool out_busy[kMaxInflight] = {};
    std::vector<uint8_t*> retired;    // grown-out result buffers
    // SHA coalescing: per owner, requests queued and non-final requests in launches on
    // the device; `missing` counts owners with requests on the device but none queued
    // (and no final request formed: a digester that asked for its digest is not
    // expected back).  A new batch is formed early only when missing == 0.
    struct Own {
        int queued = 0, flying = 0;
        bool closed = false;
    };
    bool coalesce = false;  // the SHA queue
    std::unordered_map<const void*, Own> own;
    int64_t missing = 0;
    Clock::time_point due;                        // expected end of the last launch
    Clock::time_point last_arrival;               // an owner with nothing on the device queued a request
    Clock::time_point last_done;                  // when the previous launch retired
    double ns_per_byte = 1e9 / 59e6;              // per-stream SHA time, EMA of measured launches
};

}  // namespace

struct Engine {
    Device* D = nullptr;
    int dev = 0;
    SlotPool pool;
    hipStream_t s_copy = nullptr;
    std::mutex copy_mu;
    uint64_t copy_seq = 0;
    Queue sha, crc;
    uint32_t* d_state = nullptr;  // kStateRows x 8 words
    uint8_t* d_digest = nullptr;  // kStateRows x 32 B
    std::mutex row_mu;
    std::vector<uint32_t> free_rows;
    // Host buffers (pool.S bytes, pageable) that digesters and piece streams fill between
    // submissions, recycled so that a new owner's first bytes do not page-fault a fresh
    // 2 MiB allocation (256 new uploads: half a GiB of first-touch faults).
    std::mutex pend_mu;
    std::vector<std::unique_ptr<uint8_t[]>> pend_free;
    uint32_t next_row = 0;
    uint64_t coalesce_us = 30000;  // idle device: the longest the first request waits for company
    uint64_t quiet_us = 10000;     // ... or this long with no new owner (KRK_SHA_QUIET_US)
    uint64_t fail_crc_at = 0;     // fault injection for tests: the n-th CRC launch fails (0 = never)
    bool trace = false;           // KRK_ENGINE_TRACE: one stderr line per SHA launch
    // Where the kernels read a request's slot (KRK_ENGINE_SLOT_SRC):
    //  kSrcZeroCopy (default): the SHA-256 kernel loads the pinned slot itself over PCIe
    //    (CRC requests: DMA'd at submission);
    //  kSrcGather: one gather launch per batch copies every slot of the batch into its device
    //    mirror (gather.hip) on the engine's gather stream, and the kernels read HBM;
    //  kSrcDma: one H2D DMA per slot on the copy stream at submission.
    // Measured on MI355X, same box, bench.py --workload engine (profiles/r05/bench_engine_*.json):
    // zero-copy 14.1 / 29.6 / 21.6 GB/s at 256 / 640 / 1,024 digesters, gather 12.0 / 20.6 /
    // 20.4 -- a batch is formed only when its owners are back, just before the running one
    // ends, so its gather cannot overlap the previous kernel and adds its time to every batch.
    int src = 1;
    hipStream_t s_gather = nullptr;
    std::mutex gather_mu;
    bool caller_runs = true;      // the submission completing a coalescing set launches it (KRK_ENGINE_CALLER_RUNS=0: off)
    Clock::time_point t0 = Clock::now();
    uint64_t crc_launches = 0;
    std::atomic<uint64_t> sha_batches{0}, sha_jobs{0}, crc_batches{0}, crc_reqs{0};
    std::atomic<int64_t> live_digesters{0};  // GPU digesters placed on this engine
};

namespace {

constexpr int kSrcGather = 0, kSrcZeroCopy = 1, kSrcDma = 2;
static_assert(kSrcZeroCopy == 1, "Engine::src default");

// Whether a request's slot is DMA'd to its device mirror at submission (stage()).
bool stages_on_submit(const Engine* E, bool sha) {
    return E->src == kSrcDma || (!sha && E->src == kSrcZeroCopy);
}

// kSrcGather: every slot of the batch into its device mirror in ONE gather launch on the
// engine's gather stream; the queue's stream waits for it (f->gathered).
int gather_batch(Engine* E, Queue& Q, Inflight* f) {
    std::vector<GatherSpan> spans;
    for (const Req* r : f->batch)
        if (r->slot && r->len) spans.push_back({r->slot->dev, r->slot->mapped, r->len});
    if (spans.empty()) return KRK_OK;
    std::lock_guard<std::mutex> g(E->gather_mu);
    int rc = run_gather(E->D, spans, E->s_gather);
    if (rc) return rc;
    KRK_HIP(hipEventCreateWithFlags(&f->gathered, hipEventDisableTiming));
    KRK_HIP(hipEventRecord(f->gathered, E->s_gather));
    KRK_HIP(hipStreamWaitEvent(Q.s, f->gathered, 0));
    return KRK_OK;
}

void finish(Req* r, int rc, const std::string& err) {
    r->rc = rc;
    if (rc != KRK_OK) r->err = err;
    if (r->on_done) r->on_done(r);
    std::lock_guard<std::mutex> g(r->w->mu);
    r->done = true;
    r->w->cv.notify_all();
}

int grow_out(Queue& Q, int i, size_t n) {
    if (Q.out_cap[i] >= n) return KRK_OK;
    // freeing pinned memory waits for the whole device: the old buffer is kept until teardown
    if (Q.out[i]) Q.retired.push_back(Q.out[i]);
    Q.out[i] = nullptr;
    Q.out_cap[i] = 0;
    size_t cap = 1 << 20;
    while (cap < n) cap <<= 1;
    KRK_HIP(hipHostMalloc(reinterpret_cast<void**>(&Q.out[i]), cap, hipHostMallocDefault));
    Q.out_cap[i] = cap;
    return KRK_OK;
}

// The copy stream's H2D of every request of a batch is done once the last-staged one is
// (one stream, copies in seq order): one wait instead of one per request.
int wait_staged(Queue& Q, const std::vector<Req*>& batch) {
    const Req* last = nullptr;
    for (const Req* r : batch)
        if (r->slot && r->len && (!last || r->seq > last->seq)) last = r;
    if (last) KRK_HIP(hipStreamWaitEvent(Q.s, last->slot->h2d, 0));
    return KRK_OK;
}

// One multi-stream SHA-256 launch: job i runs from its owner's state row (or the IV)
// and writes the row back (non-final) or the owner's digest row (final).
int launch_sha(Engine* E, Inflight* f) {
    Device* D = E->D;
    Queue& Q = E->sha;
    const size_t n = f->batch.size();
    std::vector<ShaJob> jobs(n);
    uint32_t lo = UINT32_MAX, hi = 0;
    for (size_t i = 0; i < n; ++i) {
        Req* r = f->batch[i];
        ShaJob& j = jobs[i];
        j = ShaJob{};
        // zero-copy: the producer waves load the pinned slot over PCIe; otherwise the slot's
        // device mirror (gathered in this batch's gather launch, or DMA'd at submission)
        j.ptr = reinterpret_cast<uint64_t>(r->slot ? (E->src == kSrcZeroCopy ? r->slot->mapped : r->slot->dev)
                                                   : reinterpret_cast<const uint8_t*>(E->d_state));
        j.len = r->len;
        j.prefix = r->prefix;
        j.out = r->row;
        j.flags = (r->final ? kShaFinal : 0) | (r->prefix ? kShaFromState : 0);
        memcpy(j.h, kIV, 32);
        f->max_len = std::max<uint64_t>(f->max_len, r->len);
        if (r->final) lo = std::min(lo, r->row), hi = std::max(hi, r->row);
    }
    int rc = E->src == kSrcGather ? gather_batch(E, Q, f) : E->src == kSrcDma ? wait_staged(Q, f->batch) : KRK_OK;
    if (!rc) rc = run_jobs(D, jobs, E->d_digest, E->d_state, Q.s);
    if (!rc && lo <= hi) {
        f->row0 = lo;
        f->nrows = hi - lo + 1;
        rc = grow_out(Q, f->out_i, 32ull * f->nrows);
        if (!rc && hipMemcpyAsync(Q.out[f->out_i], E->d_digest + 32ull * lo, 32ull * f->nrows, hipMemcpyDeviceToHost,
                                  Q.s) != hipSuccess) {
            set_error(KRK_EHIP, "engine: SHA digest copy");
            rc = KRK_EHIP;
        }
    }
    return rc;
}

void complete_sha(Engine* E, Inflight* f) {
    if (f->rc) return;
    for (Req* r : f->batch)
        if (r->final) memcpy(r->digest, E->sha.out[f->out_i] + 32ull * (r->row - f->row0), 32);
    E->sha_batches.fetch_add(1, std::memory_order_relaxed);
    E->sha_jobs.fetch_add(f->batch.size(), std::memory_order_relaxed);
}

// Portions of stream bytes [a, a+len) cut at multiples of P (P == 0: one portion).
struct Portions {
    uint64_t first_end;  // end of the first portion
    uint64_t f0, f1;     // whole pieces [f0, f1) strictly inside
    bool head, tail;     // a partial portion before / after the whole pieces
    uint64_t count;
};

Portions portions(uint64_t a, uint64_t len, uint64_t P) {
    Portions p{};
    const uint64_t b = a + len;
    if (!len) return p;
    if (P == 0) {
        p.head = true;
        p.first_end = b;
        p.count = 1;
        return p;
    }
    p.f0 = (a + P - 1) / P;
    p.f1 = b / P;
    if (p.f1 < p.f0) {  // inside one piece, touching neither boundary
        p.head = true;
        p.first_end = b;
        p.f0 = p.f1 = 0;
        p.count = 1;
        return p;
    }
    p.head = a < p.f0 * P;
    p.tail = b > p.f1 * P;
    p.first_end = p.head ? p.f0 * P : a;
    p.count = (p.head ? 1 : 0) + (p.f1 - p.f0) + (p.tail ? 1 : 0);
    return p;
}

int launch_crc(Engine* E, Inflight* f) {
    Device* D = E->D;
    Queue& Q = E->crc;
    ItemBuilder B;
    CrcBatch cb;
    auto& batch = f->batch;
    f->base.assign(batch.size() + 1, 0);
    uint64_t total = 0;
    for (size_t i = 0; i < batch.size(); ++i) {
        Req* r = batch[i];
        f->base[i] = total;
        const Portions p = portions(r->off, r->len, r->P);
        total += p.count;
        f->max_len = std::max<uint64_t>(f->max_len, r->len);
        if (!p.count) continue;
        const uint64_t dev = reinterpret_cast<uint64_t>(r->slot->dev);
        const uint64_t a = r->off, b = r->off + r->len;
        uint64_t idx = f->base[i];
        auto part = [&](uint64_t s, uint64_t e) {  // a portion hashed as its own message
            B.piece(cb.items, dev + (s - a), s, e, s, e, (uint32_t)idx++, 0xFFFFFFFFu);
        };
        if (p.head) part(a, p.first_end);
        if (p.f1 > p.f0) {
            B.run(cb, dev + (p.f0 * r->P - a), p.f0, p.f1, r->P, idx - p.f0);
            idx += p.f1 - p.f0;
        }
        if (p.tail) part(std::max(a, p.f1 * r->P), b);
    }
    f->base[batch.size()] = total;
    f->total = total;
    if (total >= (1ull << 32)) {
        set_error(KRK_EINVAL, "engine: more than 2^32 CRC portions in one batch");
        return KRK_EINVAL;
    }
    if (!total) return KRK_OK;
    int rc = E->src == kSrcGather ? gather_batch(E, Q, f) : wait_staged(Q, batch);
    if (rc) return rc;
    uint32_t* d_sums = nullptr;
    KRK_HIP(scratch_alloc(D, &d_sums, total * 4, Q.s));
    if (hipMemsetAsync(d_sums, 0, total * 4, Q.s) != hipSuccess) {
        set_error(KRK_EHIP, "engine: CRC sums clear");
        rc = KRK_EHIP;
    }
    if (!rc) rc = run_items(D, cb, d_sums, Q.s);
    if (!rc) rc = grow_out(Q, f->out_i, total * 4);
    if (!rc && hipMemcpyAsync(Q.out[f->out_i], d_sums, total * 4, hipMemcpyDeviceToHost, Q.s) != hipSuccess) {
        set_error(KRK_EHIP, "engine: CRC result copy");
        rc = KRK_EHIP;
    }
    scratch_free(D, d_sums, Q.s);
    return rc;
}

void complete_crc(Engine* E, Inflight* f) {
    if (f->rc) return;
    const uint32_t* res = reinterpret_cast<const uint32_t*>(E->crc.out[f->out_i]);
    for (size_t i = 0; i < f->batch.size(); ++i) f->batch[i]->crcs.assign(res + f->base[i], res + f->base[i + 1]);
    E->crc_batches.fetch_add(1, std::memory_order_relaxed);
    E->crc_reqs.fetch_add(f->batch.size(), std::memory_order_relaxed);
}

// Owner bookkeeping for the SHA coalescing (with Q.mu held): apply `f` to o's counts
// and keep Q.missing = #owners with requests on the device, none queued, not closed.
template <class F>
void own_update(Queue& Q, const void* o, F&& f) {
    Queue::Own& w = Q.own[o];
    const bool before = w.flying > 0 && w.queued == 0 && !w.closed;
    f(w);
    const bool after = w.flying > 0 && w.queued == 0 && !w.closed;
    Q.missing += (after ? 1 : 0) - (before ? 1 : 0);
    if (w.queued == 0 && w.flying == 0) Q.own.erase(o);
}

// Every owner with requests on the device has its next request queued; on an idle
// device, every live GPU digester of the engine has one queued.
bool expected_present(const Queue& Q, int64_t live) {
    if (Q.q.empty()) return false;
    if (Q.inflight.empty()) return live > 0 && (int64_t)Q.own.size() >= live;
    return Q.missing == 0;
}

// With Q->mu held and no dispatch in progress: the next batch (SHA: the oldest request of
// each owner, FIFO -- its state row chains through the launches, which run one after the
// other on the queue's stream; CRC: up to kMaxCrcBatchBytes), marked as being dispatched.
Inflight* take_batch(Queue* Q, bool sha, char reason) {
    auto* f = new Inflight();
    if (sha) {
        std::unordered_set<const void*> seen;
        for (auto it = Q->q.begin(); it != Q->q.end() && f->batch.size() < kStateRows;) {
            if (seen.insert((*it)->owner).second) {
                Req* r = *it;
                f->batch.push_back(r);
                own_update(*Q, r->owner, [&](Queue::Own& w) {
                    --w.queued;
                    if (r->final) w.closed = true;
                });
                it = Q->q.erase(it);
            } else {
                ++it;
            }
        }
    } else {
        uint64_t bytes = 0;
        while (!Q->q.empty() && (f->batch.empty() || bytes + Q->q.front()->len <= kMaxCrcBatchBytes)) {
            bytes += Q->q.front()->len;
            f->batch.push_back(Q->q.front());
            Q->q.pop_front();
        }
    }
    f->reason = reason;
    f->depth = Q->inflight.size();
    f->left_queued = Q->q.size();
    f->missing = Q->missing;
    f->est = Q->ns_per_byte;
    for (int i = 0; i < kMaxInflight; ++i)
        if (!Q->out_busy[i]) {
            Q->out_busy[i] = true;
            f->out_i = i;
            break;
        }
    Q->dispatching = true;
    return f;
}

// Without the lock: launch f on the queue's stream and record its completion event.
void launch_batch(Engine* E, Queue* Q, Inflight* f, bool sha) {
    // A caller's thread may run this (submit): the launch goes to the engine's device, and
    // the caller's current device -- HIP's and the library's (t_dev, which the launch timing
    // records) -- is restored afterwards.
    int hip_saved = -1;
    if (hipGetDevice(&hip_saved) != hipSuccess) hip_saved = -1;
    const int t_saved = t_dev;
    struct Restore {
        int hip, t;
        ~Restore() {
            t_dev = t;
            if (hip >= 0) hipSetDevice(hip);
        }
    } restore{hip_saved, t_saved};
    hipSetDevice(E->dev);
    t_dev = E->dev;
    f->t_launch = Clock::now();
    if (sha && E->trace)
        fprintf(stderr, "krk_engine sha t=%.3fms abs=%.3fms n=%zu why=%c depth=%zu left_queued=%zu missing=%lld est=%.2fns/B\n",
                std::chrono::duration<double, std::milli>(f->t_launch - E->t0).count(),
                std::chrono::duration<double, std::milli>(f->t_launch.time_since_epoch()).count(), f->batch.size(),
                f->reason, f->depth, f->left_queued, (long long)f->missing, f->est);
    if (!sha && ++E->crc_launches == E->fail_crc_at) {
        set_error(KRK_EHIP, "engine: injected failure of CRC launch %llu (fault injection, diag build)",
                  (unsigned long long)E->crc_launches);
        f->rc = KRK_EHIP;
    } else {
        f->rc = sha ? launch_sha(E, f) : launch_crc(E, f);
    }
    if (!f->rc) {
        if (hipEventCreateWithFlags(&f->done, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(f->done, Q->s) != hipSuccess) {
            set_error(KRK_EHIP, "engine: launch event");
            f->rc = KRK_EHIP;
        }
    }
    if (f->rc) f->err = t_err;
}

// With Q->mu held: f joins the launches on the device; the next dispatch may start.
void publish(Queue* Q, Inflight* f, bool sha) {
    if (sha) {
        for (const Req* r : f->batch)
            if (!r->final) own_update(*Q, r->owner, [](Queue::Own& w) { ++w.flying; });
        const auto start = std::max(f->t_launch, Q->inflight.empty() ? f->t_launch : Q->due);
        Q->due = start + std::chrono::nanoseconds((int64_t)(Q->ns_per_byte * (double)f->max_len));
    }
    Q->inflight.push_back(f);
    Q->dispatching = false;
}

void dispatcher(Engine* E, Queue* Q, bool sha) {
    hipSetDevice(E->dev);
    t_dev = E->dev;
    for (;;) {
        Inflight* f = nullptr;
        {
            std::unique_lock<std::mutex> lk(Q->mu);
            Q->cv.wait(lk, [&] {
                return (Q->stop && Q->q.empty() && !Q->dispatching) ||
                       (!Q->q.empty() && !Q->dispatching && Q->inflight.size() < (size_t)g_inflight);
            });
            if (Q->q.empty()) {  // stop requested and drained
                Q->disp_exited = true;
                Q->cv_done.notify_all();
                return;
            }
            char reason = '-';
            if (sha) {
                // Coalesce: on an idle device the first request waits coalesce_us for
                // company; behind running launches, the next batch is formed once every
                // owner with requests on the device has its next request queued, or ~1 ms
                // before the last launch is due to end.  (Forming it as soon as SOME owners
                // are back splits the owners into groups that alternate between launches:
                // each would then run at a fraction of the per-stream rate.)  The submission
                // that completes the set usually launches the batch itself (submit()).
                reason = 'T';
                for (;;) {
                    if (Q->stop || expected_present(*Q, E->live_digesters.load(std::memory_order_relaxed))) {  // every owner on the device is back
                        reason = Q->stop ? 'S' : 'P';
                        break;
                    }
                    // idle device: wait until every live GPU digester has a request queued, or
                    // 10 ms pass with no new owner, at most coalesce_us after the first request,
                    // so that uploads that start together also start on the device together
                    // (a digester that misses the first launch runs a whole launch behind)
                    const auto until =
                        Q->inflight.empty()
                            ? std::min(Q->q.front()->t_submit + std::chrono::microseconds(E->coalesce_us),
                                       Q->last_arrival + std::chrono::microseconds(E->quiet_us))
                            : Q->due - std::chrono::milliseconds(1);
                    if (Clock::now() >= until) break;
                    Q->cv.wait_until(lk, until);
                    if (Q->q.empty() || Q->dispatching) break;
                }
                // a caller dispatched meanwhile, or took every request
                if (Q->q.empty() || Q->dispatching || Q->inflight.size() >= (size_t)g_inflight) continue;
            }
            f = take_batch(Q, sha, reason);
        }
        launch_batch(E, Q, f, sha);
        {
            std::lock_guard<std::mutex> g(Q->mu);
            publish(Q, f, sha);
        }
        Q->cv.notify_all();
        Q->cv_done.notify_one();
    }
}

// Retires launches in order: waits for the device, hands results to the requests,
// releases their slots and wakes their owners.
void completer(Engine* E, Queue* Q, bool sha) {
    hipSetDevice(E->dev);
    t_dev = E->dev;
    for (;;) {
        Inflight* f = nullptr;
        {
            std::unique_lock<std::mutex> lk(Q->mu);
            Q->cv_done.wait(lk, [&] { return !Q->inflight.empty() || Q->disp_exited; });
            if (Q->inflight.empty()) return;
            f = Q->inflight.front();
        }
        if (!f->rc && f->done && hipEventSynchronize(f->done) != hipSuccess) {
            set_error(KRK_EHIP, "engine: %s batch failed", sha ? "SHA" : "CRC");
            f->rc = KRK_EHIP;
            f->err = t_err;
        }
        const auto t_done = Clock::now();
        if (sha && E->trace)
            fprintf(stderr, "krk_engine sha_done abs=%.3fms n=%zu\n",
                    std::chrono::duration<double, std::milli>(t_done.time_since_epoch()).count(), f->batch.size());
        if (sha) complete_sha(E, f);
        else complete_crc(E, f);
        {
            // bookkeeping first: once finished, a request (and its owner) may be freed
            std::lock_guard<std::mutex> g(Q->mu);
            Q->inflight.pop_front();
            if (f->out_i >= 0) Q->out_busy[f->out_i] = false;
            if (sha) {
                for (const Req* r : f->batch)
                    if (!r->final) own_update(*Q, r->owner, [](Queue::Own& w) { --w.flying; });
                if (!f->rc && f->max_len >= (256u << 10)) {  // per-stream time of this launch
                    const auto start = std::max(f->t_launch, Q->last_done);
                    const double ns =
                        (double)std::chrono::duration_cast<std::chrono::nanoseconds>(t_done - start).count();
                    Q->ns_per_byte = 0.7 * Q->ns_per_byte + 0.3 * (ns / (double)f->max_len);
                }
            }
            Q->last_done = t_done;
        }
        for (Req* r : f->batch) {
            E->pool.release(r->slot);
            finish(r, f->rc, f->err);
        }
        if (f->done) hipEventDestroy(f->done);
        if (f->gathered) hipEventDestroy(f->gathered);
        Q->cv.notify_all();
        delete f;
    }
}

int engine_start(Engine* E) {
    // 512 KiB slots (KRK_SLOT_KB / KRK_SLOT_MB): a digester that misses a launch falls one
    // launch behind for good, so the launch should be short; 256 concurrent digesters from
    // native threads, same box, interleaved (tests/native/digesters.cpp): 2 MiB slots with 4
    // in flight 8.8-12.6 GB/s, 512 KiB with 8 in flight 11.1-14.2 GB/s (zero-copy).
    const size_t slot = KRK_AB_ENV("KRK_SLOT_KB")   ? (env_size(KRK_AB_ENV("KRK_SLOT_KB"), 512) << 10)
                        : KRK_AB_ENV("KRK_SLOT_MB") ? (env_size(KRK_AB_ENV("KRK_SLOT_MB"), 2) << 20)
                                                    : (512u << 10);
    // KRK_SLOT_NUMA: "gpu" = the device's NUMA node, N = node N, unset = no binding
    int numa = -1;
    if (const char* nm = KRK_AB_ENV("KRK_SLOT_NUMA")) numa = strcmp(nm, "gpu") == 0 ? device_numa_node(E->dev) : atoi(nm);
    E->pool.init((slot + 63) & ~size_t(63), env_size(KRK_OP_ENV("KRK_SLOT_POOL_MB"), 4096) << 20, numa);
    g_owner_inflight = std::max<size_t>(2, env_size(KRK_AB_ENV("KRK_OWNER_INFLIGHT"), 8));
    g_inflight = (int)std::min<size_t>(kMaxInflight, std::max<size_t>(1, env_size(KRK_AB_ENV("KRK_ENGINE_INFLIGHT"), 3)));
    E->coalesce_us = env_size(KRK_AB_ENV("KRK_SHA_COALESCE_US"), 30000);
    // 10 ms: 256 writers starting together reach their first full slot over 5-25 ms on a
    // CPU-quota box; with 3 ms a third of the rounds launched before all were in and ran 3-4
    // launches more (profiles/r03/engine_quiet_ab.jsonl: median 13.94 -> 14.16 GB/s, every
    // round 33 launches).  A GPU Digester carries >= 512 KiB a request, ~9 ms of a stream.
    E->quiet_us = env_size(KRK_AB_ENV("KRK_SHA_QUIET_US"), 10000);
    E->fail_crc_at = env_size(KRK_AB_ENV("KRK_ENGINE_FAIL_CRC_LAUNCH"), 0);
    E->trace = env_size(KRK_OP_ENV("KRK_ENGINE_TRACE"), 0) != 0;
    if (const char* z = KRK_AB_ENV("KRK_SHA_ZERO_COPY")) E->src = atoi(z) ? kSrcZeroCopy : kSrcDma;  // round-4 knob
    if (const char* m = KRK_AB_ENV("KRK_ENGINE_SLOT_SRC"))
        E->src = !strcmp(m, "gather") ? kSrcGather : !strcmp(m, "dma") ? kSrcDma : kSrcZeroCopy;
    if (const char* c = KRK_AB_ENV("KRK_ENGINE_CALLER_RUNS")) E->caller_runs = atoi(c) != 0;
    KRK_HIP(hipMalloc(&E->d_state, 32ull * kStateRows));
    KRK_HIP(hipMalloc(&E->d_digest, 32ull * kStateRows));
    KRK_HIP(hipStreamCreateWithFlags(&E->s_copy, hipStreamNonBlocking));
    KRK_HIP(hipStreamCreateWithFlags(&E->s_gather, hipStreamNonBlocking));
    KRK_HIP(hipStreamCreateWithFlags(&E->sha.s, hipStreamNonBlocking));
    KRK_HIP(hipStreamCreateWithFlags(&E->crc.s, hipStreamNonBlocking));
    E->sha.last_done = E->crc.last_done = Clock::now();
    E->sha.coalesce = true;
    E->sha.th = std::thread(dispatcher, E, &E->sha, true);
    E->sha.th_done = std::thread(completer, E, &E->sha, true);
    E->crc.th = std::thread(dispatcher, E, &E->crc, false);
    E->crc.th_done = std::thread(completer, E, &E->crc, false);
    return KRK_OK;
}

void engine_free_resources(Engine* E) {
    hipSetDevice(E->dev);
    for (hipStream_t s : {E->s_copy, E->s_gather, E->sha.s, E->crc.s})
        if (s) hipStreamSynchronize(s), hipStreamDestroy(s);
    for (Queue* Q : {&E->sha, &E->crc}) {
        for (auto& p : Q->out)
            if (p) hipHostFree(p), p = nullptr;
        for (uint8_t* p : Q->retired) hipHostFree(p);
        Q->retired.clear();
    }
    if (E->d_state) hipFree(E->d_state);
    if (E->d_digest) hipFree(E->d_digest);
    E->pool.destroy();
}

// The engine of device `id`, started on first use.
Engine* engine_of(int id, int* rc) {
    Device* D = device_id(id, rc);
    if (!D) return nullptr;
    std::lock_guard<std::mutex> g(D->engine_mu);
    if (!D->engine) {
        auto* E = new Engine();
        E->D = D;
        E->dev = id;
        *rc = engine_start(E);
        if (*rc) {  // threads start last: none runs when an allocation failed
            engine_free_resources(E);
            delete E;
            return nullptr;
        }
        D->engine = E;
    }
    return D->engine;
}

// r's slot holds r->len bytes copied by the caller: issue its H2D on the copy stream.
int stage(Engine* E, Req* r) {
    if (!r->len) return KRK_OK;
    KRK_HIP(hipSetDevice(E->dev));
    std::lock_guard<std::mutex> g(E->copy_mu);
    KRK_HIP(hipMemcpyAsync(r->slot->dev, r->slot->host, r->len, hipMemcpyHostToDevice, E->s_copy));
    KRK_HIP(hipEventRecord(r->slot->h2d, E->s_copy));
    r->seq = ++E->copy_seq;
    return KRK_OK;
}

// Queue r.  On the SHA queue, the submission that completes the coalescing set (every
// owner with requests on the device has its next one queued; on an idle device, every
// live GPU digester has one) launches the batch on its own thread: with many writer
// threads busy filling slots, the dispatcher thread could wait tens of milliseconds for a
// CPU while the device idled (tools/engine_slow.py: slow rounds' first launch formed ~90
// ms after their requests were all queued).  The dispatcher still forms the batches that
// coalescing times out on.
void submit(Engine* E, Queue& Q, Req* r) {
    r->t_submit = Clock::now();
    Inflight* f = nullptr;
    {
        std::lock_guard<std::mutex> g(Q.mu);
        Q.q.push_back(r);
        if (Q.coalesce) {
            own_update(Q, r->owner, [&](Queue::Own& w) {
                if (w.queued == 0 && w.flying == 0) Q.last_arrival = r->t_submit;
                ++w.queued;
                w.closed = false;
            });
            if (E->caller_runs && !Q.dispatching && !Q.stop && Q.inflight.size() < (size_t)g_inflight &&
                expected_present(Q, E->live_digesters.load(std::memory_order_relaxed)))
                f = take_batch(&Q, true, 'C');
        }
    }
    if (f) {
        const std::string keep = t_err;  // the launch's error text belongs to its requests
        launch_batch(E, &Q, f, true);
        t_err = keep;
        {
            std::lock_guard<std::mutex> g(Q.mu);
            publish(&Q, f, true);
        }
        Q.cv_done.notify_one();
    }
    Q.cv.notify_all();
}

// A request over `len` bytes of `src` (copied into a fresh slot on this thread; its H2D
// issued unless the kernel reads the slot in place).
int make_req(Engine* E, const uint8_t* src, uint64_t len, Req** out, bool h2d = true) {
    *out = nullptr;
    Slot* sl = nullptr;
    if (len) {
        int rc = KRK_OK;
        sl = E->pool.acquire(&rc);
        if (!sl) return rc;
        memcpy(sl->host, src, len);
    }
    auto* r = new Req();
    r->slot = sl;
    r->len = len;
    const int rc = h2d ? stage(E, r) : KRK_OK;
    if (rc) {
        E->pool.release(sl);
        delete r;
        return rc;
    }
    *out = r;
    return KRK_OK;
}

// Wait for r, return its status (the engine's error text moves to this thread).
int wait_req(Req* r) {
    std::unique_lock<std::mutex> lk(r->w->mu);
    r->w->cv.wait(lk, [&] { return r->done; });
    if (r->rc) t_err = r->err;
    return r->rc;
}

void engine_stop(Engine* E) {
    for (Queue* Q : {&E->sha, &E->crc}) {
        {
            std::lock_guard<std::mutex> g(Q->mu);
            Q->stop = true;
        }
        Q->cv.notify_all();
        Q->cv_done.notify_all();
        if (Q->th.joinable()) Q->th.join();
        if (Q->th_done.joinable()) Q->th_done.join();
    }
    engine_free_resources(E);
}

uint32_t row_acquire(Engine* E, int* rc) {
    std::lock_guard<std::mutex> g(E->row_mu);
    if (!E->free_rows.empty()) {
        const uint32_t r = E->free_rows.back();
        E->free_rows.pop_back();
        *rc = KRK_OK;
        return r;
    }
    if (E->next_row < kStateRows) {
        *rc = KRK_OK;
        return E->next_row++;
    }
    set_error(KRK_ENOMEM, "engine: more than %u GPU digesters on one device", kStateRows);
    *rc = KRK_ENOMEM;
    return 0;
}

void row_release(Engine* E, uint32_t row) {
    std::lock_guard<std::mutex> g(E->row_mu);
    E->free_rows.push_back(row);
}

std::unique_ptr<uint8_t[]> pend_acquire(Engine* E) {
    {
        std::lock_guard<std::mutex> g(E->pend_mu);
        if (!E->pend_free.empty()) {
            auto b = std::move(E->pend_free.back());
            E->pend_free.pop_back();
            return b;
        }
    }
    return std::unique_ptr<uint8_t[]>(new uint8_t[E->pool.S]);
}

void pend_release(Engine* E, std::unique_ptr<uint8_t[]> b) {
    if (!b) return;
    std::lock_guard<std::mutex> g(E->pend_mu);
    if (E->pend_free.size() < 4096) E->pend_free.push_back(std::move(b));
}

// ------------------------------------------------------------------ placement
std::atomic<int64_t> g_live_digesters{0};
std::atomic<int64_t> g_host_streams{-1};  // -1: default (host threads x per-stream rate ratio)

unsigned host_threads() {
    // the CPUs this process may use: affinity AND the cgroup's CPU quota (the GPU boxes
    // grant 16 CPUs' worth of quota over an affinity of 256 CPUs; counting the affinity
    // alone kept AUTO digesters on the host up to 10,240 live instead of 640)
    return (unsigned)std::max(1, host_cpu_budget());
}

// Live digesters up to which new ones run on their caller's thread: below the crossover
// where the GPU engine's aggregate (live streams x the planner's per-stream rate, capped by
// the host link) overtakes the host's (the CPU budget x one thread's SHA-NI rate), both
// from the calling thread's device's planner rates (offload.cpp digester_crossover; the
// nominal ones without a device).  KRK_DIGESTER_HOST_STREAMS / krk_set_digester_host_streams
// pin it.
int64_t host_stream_limit() {
    const int64_t v = g_host_streams.load(std::memory_order_relaxed);
    if (v >= 0) return v;
    static const int64_t env = [] {
        const char* e = KRK_OP_ENV("KRK_DIGESTER_HOST_STREAMS");
        return e && *e ? std::max<int64_t>(0, strtoll(e, nullptr, 10)) : int64_t(-1);
    }();
    if (env >= 0) return env;
    int drc = KRK_OK;
    const int64_t x = digester_crossover(planner_rates(device(&drc)), (int)host_threads());
    return x == INT64_MAX ? x : x - 1;
}

}  // namespace

int place_device();  // multidev.cpp: next device of the process's device set

}  // namespace krk

using namespace krk;

// ======================================================================= Digester
struct krk_digester {
    Engine* E = nullptr;  // null: host placement
    // host placement: midstate after every block and the partial block
    uint32_t h[8];
    uint64_t absorbed = 0;
    uint8_t tail[64];
    size_t ntail = 0;
    // GPU placement: the engine state row, bytes not yet submitted (pend[0, fill)),
    // bytes handed to the engine, requests in flight (submission order)
    uint32_t row = 0;
    Slot* cur = nullptr;               // pending bytes filled in place in a staging slot, or
    std::unique_ptr<uint8_t[]> pend;   // in a host buffer when the pool is near its cap
    size_t fill = 0;
    uint64_t submitted = 0;
    std::deque<Req*> inflight;
    uint8_t last_digest[32] = {};
    Waiter w;
    int err = KRK_OK;
    std::string err_msg;
};

namespace {

// Wait until at most `keep` of d's requests are in flight; a failed one poisons d.
int digester_drain(krk_digester* d, size_t keep) {
    while (d->inflight.size() > keep) {
        Req* r = d->inflight.front();
        const int rc = wait_req(r);
        d->inflight.pop_front();
        if (rc == KRK_OK && r->final) memcpy(d->last_digest, r->digest, 32);
        delete r;
        if (rc && !d->err) {
            d->err = rc;
            d->err_msg = t_err;
        }
    }
    if (d->err) t_err = d->err_msg;
    return d->err;
}

// Submit `len` bytes: from the slot `sl` the digester filled in place (handed over to the
// request), else copied from `src` into a fresh slot.
// KRK_ENGINE_TRACE: one stderr line for a submission step that held its caller > 5 ms.
void trace_slow(Engine* E, const char* what, Clock::time_point t0) {
    const double ms = std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
    if (E->trace && ms > 5.0)
        fprintf(stderr, "krk_engine slow %s %.2fms abs=%.3fms\n", what, ms,
                std::chrono::duration<double, std::milli>(t0.time_since_epoch()).count());
}

// Requests a digester may keep in flight: KRK_OWNER_INFLIGHT (8), but no more than its share
// of the slot pool beyond the submissions' reserve, so that many live digesters (the
// crossover sweep: 1,024+) do not fill the hard pinned cap with the few that got there first
// while the others' writers wait at it (then fewer streams make each launch).
size_t owner_inflight(Engine* E) {
    const size_t slots = E->pool.cap() / E->pool.S, reserve = E->pool.reserve();
    const int64_t live = std::max<int64_t>(1, E->live_digesters.load(std::memory_order_relaxed));
    const size_t share = slots > reserve ? (slots - reserve) / (size_t)live : 0;
    return std::max<size_t>(2, std::min(g_owner_inflight, share));
}

int digester_submit(krk_digester* d, const uint8_t* src, uint64_t len, bool final, Slot* sl = nullptr) {
    auto t0 = Clock::now();
    int rc = digester_drain(d, owner_inflight(d->E) - 1);
    trace_slow(d->E, "drain", t0);
    t0 = Clock::now();
    if (rc) {
        d->E->pool.release(sl);
        return rc;
    }
    Req* r = nullptr;
    const bool h2d = stages_on_submit(d->E, true);
    if (sl) {
        r = new Req();
        r->slot = sl;
        r->len = len;
        rc = h2d ? stage(d->E, r) : KRK_OK;
        if (rc) {
            d->E->pool.release(sl);
            delete r;
            return rc;
        }
    } else {
        rc = make_req(d->E, src, len, &r, h2d);
        if (rc) return rc;
    }
    trace_slow(d->E, sl ? "stage" : "make_req", t0);
    r->owner = d;
    r->w = &d->w;
    r->row = d->row;
    r->prefix = d->submitted;
    r->final = final;
    d->inflight.push_back(r);
    submit(d->E, d->E->sha, r);
    if (!final) d->submitted += len;
    return KRK_OK;
}

}  // namespace

extern "C" {

int krk_digester_new_on(int placement, krk_digester** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_CHECK(placement >= KRK_PLACE_AUTO && placement <= KRK_PLACE_GPU, KRK_EINVAL, "unknown placement %d",
              placement);
    *out = nullptr;
    const int64_t live = g_live_digesters.fetch_add(1) + 1;
    bool host = placement == KRK_PLACE_HOST || (placement == KRK_PLACE_AUTO && live <= host_stream_limit());
    if (!host) {
        // GPU placement needs a gfx950 device (KRK_ENODEV without one); AUTO on a host with
        // none is the host placement: the product's own SHA-NI path (host_meta.cpp).
        int drc = KRK_OK;
        if (!device(&drc)) {
            if (placement == KRK_PLACE_GPU) {
                g_live_digesters.fetch_sub(1);
                return drc;
            }
            host = true;
        }
    }
    auto* d = new krk_digester();
    memcpy(d->h, kIV, sizeof d->h);
    if (!host) {
        int rc = KRK_OK;
        d->E = engine_of(place_device(), &rc);
        if (d->E) d->row = row_acquire(d->E, &rc);
        if (d->E && !rc) d->E->live_digesters.fetch_add(1);
        if (rc) {
            delete d;
            g_live_digesters.fetch_sub(1);
            return rc;
        }
    }
    *out = d;
    return KRK_OK;
}

int krk_digester_new(krk_digester** out) { return krk_digester_new_on(KRK_PLACE_AUTO, out); }

int krk_digester_placement(const krk_digester* d, int* placement) {
    KRK_CHECK(d && placement, KRK_EINVAL, "digester_placement: null argument");
    *placement = d->E ? KRK_PLACE_GPU : KRK_PLACE_HOST;
    return KRK_OK;
}

int krk_digester_write(krk_digester* d, const uint8_t* buf, uint64_t n) {
    KRK_CHECK(d, KRK_EINVAL, "digester is NULL");
    KRK_CHECK(n == 0 || buf, KRK_EINVAL, "buffer is NULL");
    if (!d->E) {  // host: whole blocks straight from the caller's buffer
        if (d->ntail) {
            const size_t take = std::min<uint64_t>(n, 64 - d->ntail);
            memcpy(d->tail + d->ntail, buf, take);
            d->ntail += take;
            buf += take;
            n -= take;
            if (d->ntail < 64) return KRK_OK;
            host_sha256_blocks(d->h, d->tail, 1);
            d->absorbed += 64;
            d->ntail = 0;
        }
        const uint64_t nb = n / 64;
        if (nb) host_sha256_blocks(d->h, buf, nb);
        d->absorbed += nb * 64;
        memcpy(d->tail, buf + nb * 64, n - nb * 64);
        d->ntail = n - nb * 64;
        return KRK_OK;
    }
    if (d->err) {
        t_err = d->err_msg;
        return d->err;
    }
    Engine* E = d->E;
    const size_t S = E->pool.S;
    while (n) {
        if (d->fill == 0 && n >= S) {  // a whole slot straight from the caller's buffer
            const int rc = digester_submit(d, buf, S, false);
            if (rc) return rc;
            buf += S;
            n -= S;
            continue;
        }
        if (d->fill == 0 && !d->cur) {
            const auto t0 = Clock::now();
            d->cur = E->pool.try_acquire(E->pool.reserve());
            trace_slow(E, "try_acquire", t0);
        }
        uint8_t* dst;
        if (d->cur) {
            dst = d->cur->host;
        } else {
            if (!d->pend) d->pend = pend_acquire(E);
            dst = d->pend.get();
        }
        const size_t take = std::min<uint64_t>(n, S - d->fill);
        const auto tc = Clock::now();
        memcpy(dst + d->fill, buf, take);
        trace_slow(E, d->cur ? "memcpy_slot" : "memcpy_pend", tc);
        d->fill += take;
        buf += take;
        n -= take;
        if (d->fill == S) {
            Slot* sl = d->cur;
            d->cur = nullptr;
            const int rc = digester_submit(d, dst, S, false, sl);
            if (rc) return rc;
            d->fill = 0;
        }
    }
    return KRK_OK;
}

int krk_digester_sum(krk_digester* d, uint8_t out32[32]) {
    KRK_CHECK(d && out32, KRK_EINVAL, "digester_sum: null argument");
    if (!d->E) {
        host_sha256_final(d->h, d->absorbed, d->tail, d->ntail, out32);
        return KRK_OK;
    }
    if (d->err) {
        t_err = d->err_msg;
        return d->err;
    }
    // the pending bytes stay pending (Digest() does not reset: writing may continue): a
    // slot filled in place goes with the final request and its bytes move to the host
    // buffer
    Slot* sl = d->cur;
    if (sl) {
        if (!d->pend) d->pend = pend_acquire(d->E);
        memcpy(d->pend.get(), sl->host, d->fill);
        d->cur = nullptr;
    }
    int rc = digester_submit(d, d->pend.get(), d->fill, true, sl);
    if (!rc) rc = digester_drain(d, 0);
    if (!rc) memcpy(out32, d->last_digest, 32);
    return rc;
}

void krk_digester_free(krk_digester* d) {
    if (!d) return;
    if (d->E) {
        digester_drain(d, 0);
        d->E->pool.release(d->cur);
        row_release(d->E, d->row);
        pend_release(d->E, std::move(d->pend));
        d->E->live_digesters.fetch_sub(1);
    }
    g_live_digesters.fetch_sub(1);
    delete d;
}

int krk_set_digester_host_streams(int64_t n) {
    g_host_streams.store(n < 0 ? -1 : n);
    return KRK_OK;
}

int krk_digester_host_streams(int64_t* n) {
    KRK_CHECK(n, KRK_EINVAL, "n is NULL");
    *n = host_stream_limit();
    return KRK_OK;
}

}  // extern "C"

// ======================================================================= piece stream
struct krk_piece_stream {
    Engine* E = nullptr;  // null: host placement
    uint64_t P = 0;
    uint64_t submitted = 0;       // stream bytes consumed (host) / handed to the engine (GPU)
    std::vector<uint32_t> sums;   // GPU: folded on the completer thread, in submission order
    // host placement: crc32.Update value of the current piece, bytes of it seen
    uint32_t crc = 0;
    uint64_t in_piece = 0;
    // GPU placement
    std::unique_ptr<uint8_t[]> pend;  // bytes not yet submitted
    size_t fill = 0;
    std::atomic<bool> fold_stop{false};    // completer thread: a request failed or broke the order, stop folding
    std::atomic<bool> fold_broken{false};  // completer thread: a continuation arrived with no start
    std::deque<Req*> inflight;
    Waiter w;
    int err = KRK_OK;
    std::string err_msg;
};

namespace krk {
namespace {

// ------------------------------------------------------- CRC placement
// A piece stream (NewMetaInfo over an io.Reader) and a crc32.Update call (PieceHash) carry
// no state the GPU could keep: every byte crosses the host link once, copied into a pinned
// slot by the caller's thread first.  Measured on MI355X (tests/native/crc_crossover.cpp,
// profiles/r04/crc_crossover.jsonl): the engine's CRC side carries 10 GB/s for one stream
// and ~20 GB/s for 4 to 64 (slot copies and per-slot H2D), where the host placement --
// PCLMUL on the caller's thread, large writes shared with idle host-pool threads -- carries
// 60-80 GB/s for one stream and well over 100 GB/s for several.  So AUTO keeps CRC work on
// the host unless the host's whole CRC capacity (the CPUs this process may use x one thread's
// PCLMUL rate) is below what the host link could carry to the GPU at best (0.85 x the
// measured pinned H2D rate): a box with few or slow cores.
std::atomic<int> g_crc_placement{KRK_PLACE_AUTO};  // krk_set_crc_placement / KRK_CRC_PLACEMENT

int crc_placement_setting() {
    static std::once_flag once;
    std::call_once(once, [] {
        if (const char* e = KRK_OP_ENV("KRK_CRC_PLACEMENT")) {
            const int v = atoi(e);
            if (v >= KRK_PLACE_AUTO && v <= KRK_PLACE_GPU) g_crc_placement.store(v);
        }
    });
    return g_crc_placement.load(std::memory_order_relaxed);
}

// AUTO: true = this stream / call goes to the GPU engine (a device being present).
bool crc_auto_gpu() {
    int drc = KRK_OK;
    Device* D = device(&drc);
    if (!D) return false;
    const Rates R = planner_rates(D);
    return (double)host_threads() * R.host_crc < host_link(R);
}

// The placement a new piece stream / crc32_update call runs on: HOST or GPU.  `placement`
// KRK_PLACE_AUTO follows the process setting, then the crossover; GPU needs a gfx950
// device (KRK_ENODEV), AUTO without one is HOST.
int resolve_placement(int placement, int* rc) {
    *rc = KRK_OK;
    const bool asked_auto = placement == KRK_PLACE_AUTO;
    if (asked_auto) placement = crc_placement_setting();
    const bool forced = placement != KRK_PLACE_AUTO;  // explicit, or the process setting
    if (placement == KRK_PLACE_AUTO) placement = crc_auto_gpu() ? KRK_PLACE_GPU : KRK_PLACE_HOST;
    if (placement == KRK_PLACE_GPU) {
        int drc = KRK_OK;
        if (!device(&drc)) {
            if (forced) {
                *rc = drc;
                return -1;
            }
            return KRK_PLACE_HOST;
        }
    }
    return placement;
}

}  // namespace

// runtime.hpp: the file and host-buffer CRC calls resolve their placement the same way.
int resolve_crc_placement(int placement, int* rc) { return resolve_placement(placement, rc); }

namespace {

// Fold a request's portion CRCs into the stream's piece sums (completer thread, the
// stream's requests in submission order).  Once a request has failed, later ones are
// not folded: a portion that continues a piece begun in the failed request would index
// a sum that was never written.
void stream_fold(Req* r) {
    auto* s = static_cast<krk_piece_stream*>(r->ctx);
    if (s->fold_stop) return;
    if (r->rc) {  // the owner sees r->rc when it drains r
        s->fold_stop = true;
        return;
    }
    const uint64_t a = r->off, b = r->off + r->len, P = r->P;
    uint64_t q = a;
    for (uint32_t c : r->crcs) {
        const uint64_t e = std::min(b, (q / P + 1) * P);
        const uint64_t pi = q / P;
        if (q % P == 0) {
            if (s->sums.size() <= pi) s->sums.resize(pi + 1);
            s->sums[pi] = c;
        } else if (pi < s->sums.size()) {
            s->sums[pi] = gf2_mulmod(s->sums[pi], x8n(e - q, x8().v)) ^ c;
        } else {  // a continuation with no start: never expected in submission order
            s->fold_broken = true;
            s->fold_stop = true;
            return;
        }
        q = e;
    }
}

int stream_drain(krk_piece_stream* s, size_t keep) {
    while (s->inflight.size() > keep) {
        Req* r = s->inflight.front();
        const int rc = wait_req(r);
        s->inflight.pop_front();
        delete r;
        if (rc && !s->err) {
            s->err = rc;
            s->err_msg = t_err;
        }
    }
    if (!s->err && s->fold_broken) {
        set_error(KRK_EHIP, "engine: piece stream portions out of order");
        s->err = KRK_EHIP;
        s->err_msg = t_err;
    }
    if (s->err) t_err = s->err_msg;
    return s->err;
}

int stream_submit(krk_piece_stream* s, const uint8_t* src, uint64_t len) {
    if (!len) return KRK_OK;
    int rc = stream_drain(s, g_owner_inflight - 1);
    if (rc) return rc;
    Req* r = nullptr;
    rc = make_req(s->E, src, len, &r, stages_on_submit(s->E, false));
    if (rc) return rc;
    r->owner = s;
    r->w = &s->w;
    r->off = s->submitted;
    r->P = s->P;
    r->on_done = stream_fold;
    r->ctx = s;
    s->inflight.push_back(r);
    submit(s->E, s->E->crc, r);
    s->submitted += len;
    return KRK_OK;
}

// Host placement: calcPieceSums' loop (core/metainfo.go:157-179) on the caller's thread --
// each piece's crc32.Update value carried across calls, a sum appended when a piece fills.
// A large write is cut into spans (at piece ends, then at most `span` bytes) that idle
// host-pool threads hash beside the caller; the spans' CRCs are combined in order.
void stream_host_update(krk_piece_stream* s, const uint8_t* buf, uint64_t n) {
    const int idle = n >= (2u << 20) && s->P >= (64u << 10) ? host_pool_idle() : 0;
    if (idle <= 0) {  // (small pieces: a span a piece would cost more than it spreads)
        HostCpuToken tok;
        while (n) {
            const uint64_t take = std::min<uint64_t>(n, s->P - s->in_piece);
            s->crc = host_crc32_update(s->crc, buf, take);
            s->in_piece += take;
            s->submitted += take;
            buf += take;
            n -= take;
            if (s->in_piece == s->P) {
                s->sums.push_back(s->crc);
                s->crc = 0;
                s->in_piece = 0;
            }
        }
        return;
    }
    struct Span {
        const uint8_t* p;
        uint64_t n;
        bool ends_piece;
        uint32_t c;
    };
    // A span should outlast a pool thread's wake-up: at least ~40 us of one thread's CRC
    // (256 KiB on the 128-bit PCLMUL loop, ~1.7 MiB on AVX-512 VPCLMULQDQ, where 256 KiB spans
    // took ~6 us each and the caller finished its own before the helpers woke).
    // KRK_STREAM_SPAN_KB overrides it (A/B).
    static const uint64_t min_span = [] {
        const char* v = KRK_AB_ENV("KRK_STREAM_SPAN_KB");
        if (v) return std::max<uint64_t>(64, strtoull(v, nullptr, 10)) << 10;
        const uint64_t b = (uint64_t)(host_crc_rate() * 40e-6);
        return std::max<uint64_t>(256u << 10, (b + 65535) & ~uint64_t(65535));
    }();
    const uint64_t span = std::max<uint64_t>(min_span, ((n / (uint64_t)(idle + 1)) + 63) & ~uint64_t(63));
    std::vector<Span> sp;
    for (uint64_t in = s->in_piece, o = 0; o < n;) {
        const uint64_t take = std::min<uint64_t>(n - o, s->P - in);
        for (uint64_t q = 0; q < take; q += span) {
            const uint64_t m = std::min(span, take - q);
            sp.push_back({buf + o + q, m, q + m == take && in + take == s->P, 0});
        }
        in = (in + take) % s->P;
        o += take;
    }
    host_parallel_for(sp.size(), idle, [&](size_t i) { sp[i].c = host_crc32_update(0, sp[i].p, sp[i].n); });
    for (const Span& x : sp) {
        s->crc = crc32_combine(s->crc, x.c, x.n);
        s->in_piece += x.n;
        s->submitted += x.n;
        if (x.ends_piece) {
            s->sums.push_back(s->crc);
            s->crc = 0;
            s->in_piece = 0;
        }
    }
}

}  // namespace
}  // namespace krk

extern "C" {

int krk_piece_stream_begin_on(int placement, int64_t piece_length, krk_piece_stream** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_CHECK(placement >= KRK_PLACE_AUTO && placement <= KRK_PLACE_GPU, KRK_EINVAL, "unknown placement %d",
              placement);
    KRK_CHECK(piece_length > 0, KRK_EINVAL, "piece length must be positive");
    *out = nullptr;
    int rc = KRK_OK;
    const int where = resolve_placement(placement, &rc);
    if (rc) return rc;
    Engine* E = nullptr;
    if (where == KRK_PLACE_GPU) {
        E = engine_of(place_device(), &rc);
        if (!E) return rc;
    }
    auto* s = new krk_piece_stream();
    s->E = E;
    s->P = (uint64_t)piece_length;
    *out = s;
    return KRK_OK;
}

int krk_piece_stream_begin(int64_t piece_length, krk_piece_stream** out) {
    return krk_piece_stream_begin_on(KRK_PLACE_AUTO, piece_length, out);
}

int krk_piece_stream_placement(const krk_piece_stream* s, int* placement) {
    KRK_CHECK(s && placement, KRK_EINVAL, "piece_stream_placement: null argument");
    *placement = s->E ? KRK_PLACE_GPU : KRK_PLACE_HOST;
    return KRK_OK;
}

int krk_piece_stream_update(krk_piece_stream* s, const uint8_t* buf, uint64_t n) {
    KRK_CHECK(s, KRK_EINVAL, "stream is NULL");
    KRK_CHECK(n == 0 || buf, KRK_EINVAL, "buffer is NULL");
    if (!s->E) {
        stream_host_update(s, buf, n);
        return KRK_OK;
    }
    if (s->err) {
        t_err = s->err_msg;
        return s->err;
    }
    const size_t S = s->E->pool.S;
    while (n) {
        if (s->fill == 0 && n >= S) {
            const int rc = stream_submit(s, buf, S);
            if (rc) return rc;
            buf += S;
            n -= S;
            continue;
        }
        if (!s->pend) s->pend = pend_acquire(s->E);
        const size_t take = std::min<uint64_t>(n, S - s->fill);
        memcpy(s->pend.get() + s->fill, buf, take);
        s->fill += take;
        buf += take;
        n -= take;
        if (s->fill == S) {
            const int rc = stream_submit(s, s->pend.get(), S);
            if (rc) return rc;
            s->fill = 0;
        }
    }
    return KRK_OK;
}

int krk_piece_stream_end(krk_piece_stream* s, uint32_t* sums_out, uint64_t cap, uint64_t* n_sums,
                         uint64_t* length) {
    KRK_CHECK(s, KRK_EINVAL, "stream is NULL");
    if (s->E) {
        if (s->err) {
            t_err = s->err_msg;
            return s->err;
        }
        int rc = stream_submit(s, s->pend.get(), s->fill);
        if (!rc) s->fill = 0;
        if (!rc) rc = stream_drain(s, 0);
        if (rc) return rc;
    }
    const uint64_t np = krk_num_pieces(s->submitted, (int64_t)s->P);
    if (n_sums) *n_sums = np;
    if (length) *length = s->submitted;
    KRK_CHECK(np <= cap || !sums_out, KRK_ERANGE, "sums capacity %llu < %llu pieces", (unsigned long long)cap,
              (unsigned long long)np);
    const uint64_t have = s->sums.size() + (!s->E && s->in_piece ? 1 : 0);
    KRK_CHECK(have >= np, KRK_EHIP, "engine: %llu of %llu piece sums folded", (unsigned long long)have,
              (unsigned long long)np);
    if (sums_out && np) {
        const uint64_t full = std::min<uint64_t>(np, s->sums.size());
        memcpy(sums_out, s->sums.data(), full * 4);
        if (full < np) sums_out[full] = s->crc;  // host: the partial last piece (io.CopyN n > 0)
    }
    return KRK_OK;
}

void krk_piece_stream_free(krk_piece_stream* s) {
    if (!s) return;
    if (s->E) {
        stream_drain(s, 0);
        pend_release(s->E, std::move(s->pend));
    }
    delete s;
}

// crc32.Update(crc, IEEETable, p): on the caller's thread (HOST, and AUTO below the
// crossover or for writes of at most KRK_CRC_HOST_MAX bytes), else through the device's
// CRC queue (slot-sized portions combined in order on this thread).
int krk_crc32_update_on(int placement, uint32_t crc, const uint8_t* data, uint64_t n, uint32_t* out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_CHECK(n == 0 || data, KRK_EINVAL, "data is NULL");
    KRK_CHECK(placement >= KRK_PLACE_AUTO && placement <= KRK_PLACE_GPU, KRK_EINVAL, "unknown placement %d",
              placement);
    static const size_t host_max = env_size(KRK_OP_ENV("KRK_CRC_HOST_MAX"), 64 << 10);
    int rc = KRK_OK;
    const int where = (placement == KRK_PLACE_AUTO && n <= host_max) ? KRK_PLACE_HOST
                                                                      : resolve_placement(placement, &rc);
    if (rc) return rc;
    if (where == KRK_PLACE_HOST) {
        *out = host_crc32_update_par(crc, data, n);
        return KRK_OK;
    }
    Engine* E = engine_of(place_device(), &rc);
    if (!E) return rc;
    Waiter w;
    std::deque<Req*> reqs;
    const size_t S = E->pool.S;
    uint32_t c = crc;
    auto retire = [&](Req* r) {
        const int e = wait_req(r);
        if (e && !rc) rc = e;
        if (!rc) c = gf2_mulmod(c, x8n(r->len, x8().v)) ^ r->crcs[0];
        delete r;
    };
    for (uint64_t off = 0; off < n && !rc; off += S) {
        if (reqs.size() >= g_owner_inflight) {  // bounded: the slots recycle
            retire(reqs.front());
            reqs.pop_front();
            if (rc) break;
        }
        Req* r = nullptr;
        rc = make_req(E, data + off, std::min<uint64_t>(S, n - off), &r, stages_on_submit(E, false));
        if (rc) break;
        r->owner = &w;
        r->w = &w;
        r->off = off;
        r->P = 0;
        reqs.push_back(r);
        submit(E, E->crc, r);
    }
    for (Req* r : reqs) retire(r);
    if (!rc) *out = c;
    return rc;
}

int krk_crc32_update(uint32_t crc, const uint8_t* data, uint64_t n, uint32_t* out) {
    return krk_crc32_update_on(KRK_PLACE_AUTO, crc, data, n, out);
}

int krk_set_crc_placement(int placement) {
    KRK_CHECK(placement >= KRK_PLACE_AUTO && placement <= KRK_PLACE_GPU, KRK_EINVAL, "unknown placement %d",
              placement);
    crc_placement_setting();  // the environment is read first, so this call wins over it
    g_crc_placement.store(placement);
    return KRK_OK;
}

int krk_engine_stats(uint64_t* sha_batches, uint64_t* sha_jobs, uint64_t* crc_batches, uint64_t* crc_requests,
                     uint64_t* pinned_bytes) {
    KRK_DEVICE(D);
    uint64_t v[5] = {0, 0, 0, 0, 0};
    {
        std::lock_guard<std::mutex> g(D->engine_mu);
        if (Engine* E = D->engine) {
            v[0] = E->sha_batches.load();
            v[1] = E->sha_jobs.load();
            v[2] = E->crc_batches.load();
            v[3] = E->crc_reqs.load();
            v[4] = E->pool.pinned_bytes();
        }
    }
    uint64_t* o[5] = {sha_batches, sha_jobs, crc_batches, crc_requests, pinned_bytes};
    for (int i = 0; i < 5; ++i)
        if (o[i]) *o[i] = v[i];
    return KRK_OK;
}

int krk_engine_set_pool_cap(uint64_t bytes, uint64_t* cap_out, uint64_t* waits_out) {
    KRK_DEVICE(D0);
    int rc = KRK_OK;
    Engine* E = engine_of(D0->id, &rc);
    if (!E) return rc;
    if (bytes) E->pool.set_cap(bytes);
    if (cap_out) *cap_out = E->pool.cap();
    if (waits_out) *waits_out = E->pool.waits();
    return KRK_OK;
}

}  // extern "C"

namespace krk {
// krk_shutdown: stop the engine of D (its dispatcher and completer threads drain their queues).
void engine_teardown(Device& D) {
    std::lock_guard<std::mutex> g(D.engine_mu);
    if (D.engine) {
        engine_stop(D.engine);
        delete D.engine;
        D.engine = nullptr;
    }
}
}  // namespace krk
