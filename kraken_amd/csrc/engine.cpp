// engine.cpp -- the per-device submission engine behind the streaming entry points
// (krk_digester_*, krk_piece_stream_*, krk_crc32_update).
//
// The reference calls these from many goroutines at once (SURVEY.md 8(b)
// "Threading": origin/blobserver/uploader.go:75 and lib/store/ca_store.go:119 run a
// Digester per upload / cache fill, lib/torrent/storage/agentstorage/torrent.go:182
// a PieceHash per received piece).  One launch per call would serialise them and
// leave the chip empty, so every device context owns:
//
//  * a pool of fixed-size pinned staging slots, each with a device mirror: a caller
//    copies its bytes into a slot on its own thread and issues the slot's H2D on the
//    engine's copy stream -- no pinning per call, no per-call device allocation;
//  * two queues, each drained by a dispatcher thread that coalesces every pending
//    request into ONE launch: SHA-256 requests (one Merkle-Damgard stream each, so
//    a batch of concurrent digesters is a multi-stream sha256_multi launch) and
//    CRC-32 requests (crc32_pieces over every pending byte range).
//
// Ordering is per request owner, not device-global: a digester's midstate lives on
// the host between its requests and goes into the next job's descriptor, so the SHA
// dispatcher takes at most one request per digester per batch (batches run one
// after the other).  CRC requests carry no state at all: each piece portion is
// hashed as an independent message and the host folds portions together with the
// GF(2) combine crc(A||B) = crc(A) * x^(8|B|) ^ crc(B) (crc_math.hpp), so any
// number of a stream's requests may share a batch and a stream's piece end need not
// be known when its bytes are submitted.
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
#include <unordered_set>

#include "runtime.hpp"

namespace krk {

void host_sha256_blocks(uint32_t h[8], const uint8_t* p, size_t nblocks);
void host_sha256_final(const uint32_t h[8], uint64_t absorbed, const uint8_t* tail, size_t n, uint8_t out[32]);
uint32_t host_crc32_update(uint32_t crc, const uint8_t* p, size_t n);

namespace {

size_t env_size(const char* k, size_t dflt) {
    const char* v = getenv(k);
    if (!v || !*v) return dflt;
    const unsigned long long x = strtoull(v, nullptr, 10);
    return x ? (size_t)x : dflt;
}

// ------------------------------------------------------------------ slots
struct Slot {
    uint8_t* host = nullptr;  // pinned
    uint8_t* dev = nullptr;   // device mirror
    hipEvent_t h2d = nullptr;  // the last H2D of this slot
};

class SlotPool {
  public:
    size_t S = 0;  // bytes per slot (multiple of 64)

    int init(size_t slot_bytes, size_t cap_bytes) {
        S = slot_bytes;
        cap_ = std::max(cap_bytes, S * kPerChunk);
        return KRK_OK;
    }

    // A free slot; grows the pool one chunk at a time up to its cap, then waits for a
    // release.  Call with the owning device current.
    Slot* acquire(int* rc) {
        std::unique_lock<std::mutex> lk(mu_);
        while (free_.empty()) {
            // At the cap, wait for a release; the cap is soft: if nothing comes back within
            // 100 ms (every slot held by an owner that is still filling it) grow anyway
            // rather than deadlock.
            if (allocated_ + S * kPerChunk > cap_ &&
                cv_.wait_for(lk, std::chrono::milliseconds(100)) == std::cv_status::no_timeout)
                continue;
            if (!free_.empty()) break;
            *rc = grow();
            if (*rc) return nullptr;
        }
        Slot* s = free_.back();
        free_.pop_back();
        *rc = KRK_OK;
        return s;
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

    int grow() {  // with mu_ held
        const size_t bytes = S * kPerChunk;
        void *h = nullptr, *d = nullptr;
        KRK_HIP(hipHostMalloc(&h, bytes, hipHostMallocDefault));
        if (hipMalloc(&d, bytes) != hipSuccess) {
            hipHostFree(h);
            set_error(KRK_ENOMEM, "engine: device staging slots (%zu bytes)", bytes);
            return KRK_ENOMEM;
        }
        std::unique_ptr<Slot[]> c(new Slot[kPerChunk]);
        for (int i = 0; i < kPerChunk; ++i) {
            c[i].host = static_cast<uint8_t*>(h) + i * S;
            c[i].dev = static_cast<uint8_t*>(d) + i * S;
            KRK_HIP(hipEventCreateWithFlags(&c[i].h2d, hipEventDisableTiming));
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

enum ReqKind { kReqSha, kReqCrc };

struct Req {
    ReqKind kind = kReqSha;
    Slot* slot = nullptr;
    bool release_slot = true;
    uint64_t len = 0;
    const void* owner = nullptr;  // ordering key (SHA: one request per owner per batch)
    Waiter* w = nullptr;
    // SHA: bytes absorbed before this request; final = pad and write the digest.
    uint64_t prefix = 0;
    bool final = false;
    uint32_t* mid = nullptr;  // the owner's midstate (read at dispatch, written on completion)
    uint8_t digest[32] = {};
    // CRC: stream offset of the slot's first byte and the piece length (0: the request
    // is one portion); crcs[k] = crc32 of portion k as an independent message.
    uint64_t off = 0;
    uint64_t P = 0;
    std::vector<uint32_t> crcs;
    void (*on_done)(Req*) = nullptr;  // runs on the dispatcher thread, in FIFO order
    void* ctx = nullptr;
    int rc = KRK_OK;
    std::string err;
    bool done = false;
};

struct Queue {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Req*> q;
    bool stop = false;
    std::thread th;
    hipStream_t s = nullptr;
    uint8_t* h_out = nullptr;  // pinned result buffer, grown on demand
    size_t h_cap = 0;
};

constexpr size_t kMaxShaBatch = 65536;
constexpr uint64_t kMaxCrcBatchBytes = 4ull << 30;

}  // namespace

struct Engine {
    Device* D = nullptr;
    int dev = 0;
    SlotPool pool;
    hipStream_t s_copy = nullptr;
    Queue sha, crc;
    std::atomic<uint64_t> sha_batches{0}, sha_jobs{0}, crc_batches{0}, crc_reqs{0};
};

namespace {

void finish(Req* r, int rc) {
    r->rc = rc;
    if (rc != KRK_OK) r->err = t_err;
    if (r->on_done) r->on_done(r);
    std::lock_guard<std::mutex> g(r->w->mu);
    r->done = true;
    r->w->cv.notify_all();
}

int grow_out(Queue& Q, size_t n) {
    if (Q.h_cap >= n) return KRK_OK;
    if (Q.h_out) hipHostFree(Q.h_out);
    Q.h_out = nullptr;
    Q.h_cap = 0;
    const size_t cap = std::max<size_t>(n, 1 << 20);
    KRK_HIP(hipHostMalloc(reinterpret_cast<void**>(&Q.h_out), cap, hipHostMallocDefault));
    Q.h_cap = cap;
    return KRK_OK;
}

// One multi-stream SHA-256 launch over the batch: each request is one job whose
// initial state is its owner's midstate; outputs (32-B midstate or digest per job)
// come back in one D2H.
int run_sha_batch(Engine* E, std::vector<Req*>& batch) {
    Device* D = E->D;
    Queue& Q = E->sha;
    const size_t n = batch.size();
    std::vector<ShaJob> jobs(n);
    for (size_t i = 0; i < n; ++i) {
        Req* r = batch[i];
        ShaJob& j = jobs[i];
        j = ShaJob{};
        j.ptr = reinterpret_cast<uint64_t>(r->slot ? r->slot->dev : nullptr);
        j.len = r->len;
        j.prefix = r->prefix;
        j.out = (uint32_t)i;
        j.flags = r->final ? kShaFinal : 0;
        memcpy(j.h, r->mid, 32);
        if (r->slot && r->len) KRK_HIP(hipStreamWaitEvent(Q.s, r->slot->h2d, 0));
    }
    uint8_t* d_out = nullptr;
    KRK_HIP(scratch_alloc(D, &d_out, 64 * n, Q.s));
    int rc = run_jobs(D, jobs, d_out + 32 * n, reinterpret_cast<uint32_t*>(d_out), Q.s);
    if (!rc) rc = grow_out(Q, 64 * n);
    if (!rc && hipMemcpyAsync(Q.h_out, d_out, 64 * n, hipMemcpyDeviceToHost, Q.s) != hipSuccess) {
        set_error(KRK_EHIP, "engine: SHA result copy");
        rc = KRK_EHIP;
    }
    scratch_free(D, d_out, Q.s);
    if (hipStreamSynchronize(Q.s) != hipSuccess && !rc) {
        set_error(KRK_EHIP, "engine: SHA batch failed");
        rc = KRK_EHIP;
    }
    if (rc) return rc;
    for (size_t i = 0; i < n; ++i) {
        Req* r = batch[i];
        if (r->final) memcpy(r->digest, Q.h_out + 32 * n + 32 * i, 32);
        else memcpy(r->mid, Q.h_out + 32 * i, 32);  // the owner waits for this request: no race
    }
    E->sha_batches.fetch_add(1, std::memory_order_relaxed);
    E->sha_jobs.fetch_add(n, std::memory_order_relaxed);
    return KRK_OK;
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

int run_crc_batch(Engine* E, std::vector<Req*>& batch) {
    Device* D = E->D;
    Queue& Q = E->crc;
    ItemBuilder B;
    CrcBatch cb;
    std::vector<uint64_t> base(batch.size());
    uint64_t total = 0;
    for (size_t i = 0; i < batch.size(); ++i) {
        Req* r = batch[i];
        base[i] = total;
        const Portions p = portions(r->off, r->len, r->P);
        total += p.count;
        if (!p.count) continue;
        KRK_HIP(hipStreamWaitEvent(Q.s, r->slot->h2d, 0));
        const uint64_t dev = reinterpret_cast<uint64_t>(r->slot->dev);
        const uint64_t a = r->off, b = r->off + r->len;
        uint64_t idx = base[i];
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
    if (total >= (1ull << 32)) {
        set_error(KRK_EINVAL, "engine: more than 2^32 CRC portions in one batch");
        return KRK_EINVAL;
    }
    uint32_t* d_sums = nullptr;
    if (total) {
        KRK_HIP(scratch_alloc(D, &d_sums, total * 4, Q.s));
        KRK_HIP(hipMemsetAsync(d_sums, 0, total * 4, Q.s));
    }
    int rc = total ? run_items(D, cb, d_sums, Q.s) : KRK_OK;
    if (!rc && total) rc = grow_out(Q, total * 4);
    if (!rc && total && hipMemcpyAsync(Q.h_out, d_sums, total * 4, hipMemcpyDeviceToHost, Q.s) != hipSuccess) {
        set_error(KRK_EHIP, "engine: CRC result copy");
        rc = KRK_EHIP;
    }
    if (d_sums) scratch_free(D, d_sums, Q.s);
    if (hipStreamSynchronize(Q.s) != hipSuccess && !rc) {
        set_error(KRK_EHIP, "engine: CRC batch failed");
        rc = KRK_EHIP;
    }
    if (rc) return rc;
    const uint32_t* res = reinterpret_cast<const uint32_t*>(Q.h_out);
    for (size_t i = 0; i < batch.size(); ++i) {
        const uint64_t c = (i + 1 < batch.size() ? base[i + 1] : total) - base[i];
        batch[i]->crcs.assign(res + base[i], res + base[i] + c);
    }
    E->crc_batches.fetch_add(1, std::memory_order_relaxed);
    E->crc_reqs.fetch_add(batch.size(), std::memory_order_relaxed);
    return KRK_OK;
}

void dispatcher(Engine* E, Queue* Q, bool sha) {
    hipSetDevice(E->dev);
    t_dev = E->dev;
    std::vector<Req*> batch;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(Q->mu);
            Q->cv.wait(lk, [&] { return Q->stop || !Q->q.empty(); });
            if (Q->q.empty()) return;  // stop requested and drained
            if (sha) {
                // FIFO, the oldest request of each owner (its midstate chains through
                // the batches, which run one after the other)
                std::unordered_set<const void*> seen;
                for (auto it = Q->q.begin(); it != Q->q.end() && batch.size() < kMaxShaBatch;) {
                    if (seen.insert((*it)->owner).second) {
                        batch.push_back(*it);
                        it = Q->q.erase(it);
                    } else {
                        ++it;
                    }
                }
            } else {
                uint64_t bytes = 0;
                while (!Q->q.empty() && (batch.empty() || bytes + Q->q.front()->len <= kMaxCrcBatchBytes)) {
                    bytes += Q->q.front()->len;
                    batch.push_back(Q->q.front());
                    Q->q.pop_front();
                }
            }
        }
        const int rc = sha ? run_sha_batch(E, batch) : run_crc_batch(E, batch);
        for (Req* r : batch) {
            if (r->release_slot) E->pool.release(r->slot);
            finish(r, rc);
        }
        batch.clear();
    }
}

int engine_start(Engine* E) {
    E->pool.init(env_size("KRK_SLOT_MB", 2) << 20, env_size("KRK_SLOT_POOL_MB", 4096) << 20);
    KRK_HIP(hipStreamCreateWithFlags(&E->s_copy, hipStreamNonBlocking));
    KRK_HIP(hipStreamCreateWithFlags(&E->sha.s, hipStreamNonBlocking));
    KRK_HIP(hipStreamCreateWithFlags(&E->crc.s, hipStreamNonBlocking));
    E->sha.th = std::thread(dispatcher, E, &E->sha, true);
    E->crc.th = std::thread(dispatcher, E, &E->crc, false);
    return KRK_OK;
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
        if (*rc) {
            delete E;  // threads not started when a stream creation failed
            return nullptr;
        }
        D->engine = E;
    }
    return D->engine;
}

// Copy done by the caller: issue the slot's H2D (bytes [0, n)) on the copy stream.
int stage(Engine* E, Slot* s, size_t n) {
    if (!n) return KRK_OK;
    KRK_HIP(hipSetDevice(E->dev));
    KRK_HIP(hipMemcpyAsync(s->dev, s->host, n, hipMemcpyHostToDevice, E->s_copy));
    KRK_HIP(hipEventRecord(s->h2d, E->s_copy));
    return KRK_OK;
}

void submit(Queue& Q, Req* r) {
    {
        std::lock_guard<std::mutex> g(Q.mu);
        Q.q.push_back(r);
    }
    Q.cv.notify_one();
}

// Wait for r, return its status (the dispatcher's error text moves to this thread).
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
        if (Q->th.joinable()) Q->th.join();
    }
    hipSetDevice(E->dev);
    for (hipStream_t s : {E->s_copy, E->sha.s, E->crc.s})
        if (s) hipStreamSynchronize(s), hipStreamDestroy(s);
    for (Queue* Q : {&E->sha, &E->crc})
        if (Q->h_out) hipHostFree(Q->h_out);
    E->pool.destroy();
}

// ------------------------------------------------------------------ placement
std::atomic<int64_t> g_live_digesters{0};
std::atomic<int64_t> g_host_streams{-1};  // -1: default (host threads x per-stream rate ratio)

unsigned host_threads() {
    // the CPUs this process may use (affinity); the GPU boxes grant a 16-CPU share
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) return std::max(1, CPU_COUNT(&set));
    return std::max(1u, std::thread::hardware_concurrency());
}

// Live digesters up to which new ones run on their caller's thread: where the host's
// aggregate (threads x ~2 GB/s SHA-NI) still beats the GPU's (streams x ~59 MB/s),
// i.e. 40 streams per host thread.  KRK_DIGESTER_HOST_STREAMS / krk_set_digester_host_streams.
int64_t host_stream_limit() {
    int64_t v = g_host_streams.load(std::memory_order_relaxed);
    if (v >= 0) return v;
    const char* e = getenv("KRK_DIGESTER_HOST_STREAMS");
    v = e && *e ? strtoll(e, nullptr, 10) : int64_t(40) * host_threads();
    int64_t expect = -1;
    g_host_streams.compare_exchange_strong(expect, v);
    return g_host_streams.load(std::memory_order_relaxed);
}

}  // namespace

int place_device();  // multidev.cpp: next device of the process's device set

}  // namespace krk

using namespace krk;

// ======================================================================= Digester
struct krk_digester {
    Engine* E = nullptr;  // null: host placement
    uint32_t h[8];        // midstate after every completed request (host: after every block)
    uint64_t absorbed = 0;
    // host placement: the partial block
    uint8_t tail[64];
    size_t ntail = 0;
    // GPU placement
    Slot* cur = nullptr;  // slot being filled
    size_t fill = 0;
    uint64_t submitted = 0;  // bytes handed to the engine
    std::deque<Req*> inflight;
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
        if (rc == KRK_OK) d->absorbed += r->len;
        delete r;
        if (rc && !d->err) {
            d->err = rc;
            d->err_msg = t_err;
        }
    }
    if (d->err) t_err = d->err_msg;
    return d->err;
}

int digester_submit(krk_digester* d, bool final) {
    Engine* E = d->E;
    if (!d->cur) {  // a final job with no pending bytes still needs a slot address
        int rc = KRK_OK;
        d->cur = E->pool.acquire(&rc);
        if (!d->cur) return rc;
        d->fill = 0;
    }
    int rc = stage(E, d->cur, d->fill);
    if (rc) return rc;
    auto* r = new Req();
    r->kind = kReqSha;
    r->slot = d->cur;
    r->len = d->fill;
    r->owner = d;
    r->w = &d->w;
    r->prefix = d->submitted;
    r->final = final;
    r->mid = d->h;
    r->release_slot = !final;  // after Digest() the digester keeps writing into its slot
    d->inflight.push_back(r);
    submit(E->sha, r);
    if (!final) {
        d->submitted += d->fill;
        d->cur = nullptr;
        d->fill = 0;
    }
    return KRK_OK;
}

}  // namespace

extern "C" {

int krk_digester_new_on(int placement, krk_digester** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_CHECK(placement >= KRK_PLACE_AUTO && placement <= KRK_PLACE_GPU, KRK_EINVAL, "unknown placement %d",
              placement);
    *out = nullptr;
    KRK_DEVICE(D0);  // the library serves a gfx950 device; no device is KRK_ENODEV, never a CPU fallback
    (void)D0;
    const int64_t live = g_live_digesters.fetch_add(1) + 1;
    const bool host = placement == KRK_PLACE_HOST || (placement == KRK_PLACE_AUTO && live <= host_stream_limit());
    auto* d = new krk_digester();
    memcpy(d->h, kIV, sizeof d->h);
    if (!host) {
        int rc = KRK_OK;
        d->E = engine_of(place_device(), &rc);
        if (!d->E) {
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
        if (!d->cur) {
            // at most two requests of this digester in flight: the one running and the next
            int rc = digester_drain(d, 1);
            if (rc) return rc;
            d->cur = E->pool.acquire(&rc);
            if (!d->cur) return rc;
            d->fill = 0;
        }
        const size_t take = std::min<uint64_t>(n, S - d->fill);
        memcpy(d->cur->host + d->fill, buf, take);
        d->fill += take;
        buf += take;
        n -= take;
        if (d->fill == S) {
            int rc = digester_submit(d, false);
            if (rc) return rc;
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
    int rc = digester_drain(d, 0);  // the midstate is current once nothing is in flight
    if (rc) return rc;
    rc = digester_submit(d, true);
    if (rc) return rc;
    Req* r = d->inflight.back();
    rc = wait_req(r);
    d->inflight.pop_back();
    if (!rc) memcpy(out32, r->digest, 32);
    delete r;
    return rc;
}

void krk_digester_free(krk_digester* d) {
    if (!d) return;
    if (d->E) {
        digester_drain(d, 0);
        d->E->pool.release(d->cur);
    }
    g_live_digesters.fetch_sub(1);
    delete d;
}

int krk_set_digester_host_streams(int64_t n) {
    g_host_streams.store(n < 0 ? -1 : n);
    return KRK_OK;
}

}  // extern "C"

// ======================================================================= piece stream
struct krk_piece_stream {
    Engine* E = nullptr;
    uint64_t P = 0;
    Slot* cur = nullptr;
    size_t fill = 0;
    uint64_t submitted = 0;       // stream bytes handed to the engine
    std::vector<uint32_t> sums;   // folded on the dispatcher thread, in submission order
    std::deque<Req*> inflight;
    Waiter w;
    int err = KRK_OK;
    std::string err_msg;
};

namespace {

// Fold a request's portion CRCs into the stream's piece sums (dispatcher thread).
void stream_fold(Req* r) {
    if (r->rc) return;
    auto* s = static_cast<krk_piece_stream*>(r->ctx);
    const uint64_t a = r->off, b = r->off + r->len, P = r->P;
    uint64_t q = a;
    for (uint32_t c : r->crcs) {
        const uint64_t e = std::min(b, (q / P + 1) * P);
        const uint64_t pi = q / P;
        if (q % P == 0) {
            if (s->sums.size() <= pi) s->sums.resize(pi + 1);
            s->sums[pi] = c;
        } else {
            s->sums[pi] = gf2_mulmod(s->sums[pi], x8n(e - q, x8().v)) ^ c;
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
    if (s->err) t_err = s->err_msg;
    return s->err;
}

int stream_submit(krk_piece_stream* s) {
    if (!s->fill) return KRK_OK;
    int rc = stage(s->E, s->cur, s->fill);
    if (rc) return rc;
    auto* r = new Req();
    r->kind = kReqCrc;
    r->slot = s->cur;
    r->len = s->fill;
    r->owner = s;
    r->w = &s->w;
    r->off = s->submitted;
    r->P = s->P;
    r->on_done = stream_fold;
    r->ctx = s;
    s->inflight.push_back(r);
    submit(s->E->crc, r);
    s->submitted += s->fill;
    s->cur = nullptr;
    s->fill = 0;
    return KRK_OK;
}

}  // namespace

extern "C" {

int krk_piece_stream_begin(int64_t piece_length, krk_piece_stream** out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_CHECK(piece_length > 0, KRK_EINVAL, "piece length must be positive");
    *out = nullptr;
    KRK_DEVICE(D0);
    (void)D0;
    int rc = KRK_OK;
    Engine* E = engine_of(place_device(), &rc);
    if (!E) return rc;
    auto* s = new krk_piece_stream();
    s->E = E;
    s->P = (uint64_t)piece_length;
    *out = s;
    return KRK_OK;
}

int krk_piece_stream_update(krk_piece_stream* s, const uint8_t* buf, uint64_t n) {
    KRK_CHECK(s, KRK_EINVAL, "stream is NULL");
    KRK_CHECK(n == 0 || buf, KRK_EINVAL, "buffer is NULL");
    if (s->err) {
        t_err = s->err_msg;
        return s->err;
    }
    const size_t S = s->E->pool.S;
    while (n) {
        if (!s->cur) {
            int rc = stream_drain(s, 3);  // a few requests in flight: the slots recycle
            if (rc) return rc;
            s->cur = s->E->pool.acquire(&rc);
            if (!s->cur) return rc;
            s->fill = 0;
        }
        const size_t take = std::min<uint64_t>(n, S - s->fill);
        memcpy(s->cur->host + s->fill, buf, take);
        s->fill += take;
        buf += take;
        n -= take;
        if (s->fill == S) {
            int rc = stream_submit(s);
            if (rc) return rc;
        }
    }
    return KRK_OK;
}

int krk_piece_stream_end(krk_piece_stream* s, uint32_t* sums_out, uint64_t cap, uint64_t* n_sums,
                         uint64_t* length) {
    KRK_CHECK(s, KRK_EINVAL, "stream is NULL");
    if (s->err) {
        t_err = s->err_msg;
        return s->err;
    }
    int rc = stream_submit(s);
    if (!rc) rc = stream_drain(s, 0);
    if (rc) return rc;
    const uint64_t np = krk_num_pieces(s->submitted, (int64_t)s->P);
    if (n_sums) *n_sums = np;
    if (length) *length = s->submitted;
    KRK_CHECK(np <= cap || !sums_out, KRK_ERANGE, "sums capacity %llu < %llu pieces", (unsigned long long)cap,
              (unsigned long long)np);
    if (sums_out && np) memcpy(sums_out, s->sums.data(), np * 4);
    return KRK_OK;
}

void krk_piece_stream_free(krk_piece_stream* s) {
    if (!s) return;
    stream_drain(s, 0);
    s->E->pool.release(s->cur);
    delete s;
}

// crc32.Update(crc, IEEETable, p): small writes on the caller's thread, the rest
// through the CRC queue (slot-sized portions combined in order on this thread).
int krk_crc32_update(uint32_t crc, const uint8_t* data, uint64_t n, uint32_t* out) {
    KRK_CHECK(out, KRK_EINVAL, "out is NULL");
    KRK_CHECK(n == 0 || data, KRK_EINVAL, "data is NULL");
    KRK_DEVICE(D0);
    (void)D0;
    if (n <= env_size("KRK_CRC_HOST_MAX", 64 << 10)) {
        *out = host_crc32_update(crc, data, n);
        return KRK_OK;
    }
    int rc = KRK_OK;
    Engine* E = engine_of(place_device(), &rc);
    if (!E) return rc;
    Waiter w;
    std::vector<Req*> reqs;
    const size_t S = E->pool.S;
    for (uint64_t off = 0; off < n && !rc; off += S) {
        Slot* sl = E->pool.acquire(&rc);
        if (!sl) break;
        const size_t take = std::min<uint64_t>(S, n - off);
        memcpy(sl->host, data + off, take);
        rc = stage(E, sl, take);
        if (rc) {
            E->pool.release(sl);
            break;
        }
        auto* r = new Req();
        r->kind = kReqCrc;
        r->slot = sl;
        r->len = take;
        r->owner = &w;
        r->w = &w;
        r->off = off;
        r->P = 0;
        reqs.push_back(r);
        submit(E->crc, r);
    }
    uint32_t c = crc;
    for (Req* r : reqs) {
        const int e = wait_req(r);
        if (e && !rc) rc = e;
        if (!rc) c = gf2_mulmod(c, x8n(r->len, x8().v)) ^ r->crcs[0];
        delete r;
    }
    if (!rc) *out = c;
    return rc;
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

}  // extern "C"

namespace krk {
// krk_shutdown: stop the engine of D (its dispatcher threads drain their queues).
void engine_teardown(Device& D) {
    std::lock_guard<std::mutex> g(D.engine_mu);
    if (D.engine) {
        engine_stop(D.engine);
        delete D.engine;
        D.engine = nullptr;
    }
}
}  // namespace krk
