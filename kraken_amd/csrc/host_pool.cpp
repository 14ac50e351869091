// host_pool.cpp -- the process's pool of host worker threads for the host placements.
//
// The host side of the crossovers (a piece stream or crc32.Update call on its caller's
// thread; the host share of krk_piece_sums_host / krk_verify_pieces_host)
// runs PCLMUL CRC-32 at ~17 GB/s a core.  A lone large call would leave the process's other
// cores idle, and starting threads per call costs more than a few pieces' CRC,
// so the work is shared with a fixed pool: the caller posts a job, runs its items itself,
// and up to `helpers` pool threads that are idle at that moment join in.  Items are claimed
// one at a time, so a busy pool never delays a caller -- a helper that arrives late finds
// nothing left -- and concurrent callers each keep at least their own thread.  CRC-32 is
// linear over GF(2), so a buffer cut into spans is hashed span by span on any threads and
// recombined in order: crc(A||B) = crc(A) * x^(8|B|) ^ crc(B) (crc_math.hpp).
#include <condition_variable>
#include <deque>
#include <functional>
#include <thread>

#include "runtime.hpp"

namespace krk {

struct HostJob {
    std::function<void(size_t)> f;
    size_t n = 0;
    std::atomic<size_t> next{0};
    std::mutex mu;
    std::condition_variable cv;
    size_t done = 0;  // under mu
    int want = 0;     // helpers still wanted (under the pool's mu)
};

// ------------------------------------------------------------------ CPU tokens
// At most host_cpu_budget() threads run host hash work at once, whoever calls: 64 uploads'
// piece streams on a 16-CPU quota would otherwise all run at once on the machine's many
// cores, stall on each other's memory traffic while burning the quota, and be throttled
// (measured: 64 concurrent streams 92-98 GB/s against 126-158 for 4-16).  The reference's
// goroutines get the same bound from GOMAXPROCS.  Re-entrant per thread.
namespace {
class CpuTokens {
  public:
    explicit CpuTokens(int n) : avail_(n) {}
    void acquire() {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return avail_ > 0; });
        --avail_;
    }
    void release() {
        {
            std::lock_guard<std::mutex> g(mu_);
            ++avail_;
        }
        cv_.notify_one();
    }

  private:
    std::mutex mu_;
    std::condition_variable cv_;
    int avail_;
};
CpuTokens& cpu_tokens() {
    static CpuTokens* t = new CpuTokens(std::max(1, host_cpu_budget()));  // leaked: used by detached workers
    return *t;
}
thread_local int t_token_depth = 0;
}  // namespace

HostCpuToken::HostCpuToken() {
    if (t_token_depth++ == 0) cpu_tokens().acquire();
}
HostCpuToken::~HostCpuToken() {
    if (--t_token_depth == 0) cpu_tokens().release();
}

namespace {

void claim_items(HostJob& j) {
    if (j.next.load(std::memory_order_relaxed) >= j.n) return;  // nothing left: no token
    size_t mine = 0;
    HostCpuToken tok;
    for (size_t i; (i = j.next.fetch_add(1)) < j.n;) {
        j.f(i);
        ++mine;
    }
    if (mine) {
        std::lock_guard<std::mutex> g(j.mu);
        j.done += mine;
        if (j.done == j.n) j.cv.notify_all();
    }
}

class Pool {
  public:
    explicit Pool(int threads) {
        for (int t = 0; t < threads; ++t) std::thread([this] { worker(); }).detach();
    }
    int threads_idle() {
        std::lock_guard<std::mutex> g(mu_);
        return idle_ - wanted_;
    }
    // Offer job j to up to `helpers` idle workers; returns how many were asked.
    int offer(const std::shared_ptr<HostJob>& j, int helpers) {
        std::lock_guard<std::mutex> g(mu_);
        const int k = std::min(helpers, idle_ - wanted_);
        if (k <= 0) return 0;
        j->want = k;
        wanted_ += k;
        q_.push_back(j);
        if (k == 1) cv_.notify_one();
        else cv_.notify_all();
        return k;
    }

  private:
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::shared_ptr<HostJob>> q_;
    int idle_ = 0, wanted_ = 0;

    void worker() {
        std::unique_lock<std::mutex> lk(mu_);
        for (;;) {
            ++idle_;
            cv_.wait(lk, [&] { return !q_.empty(); });
            --idle_;
            std::shared_ptr<HostJob> j = q_.front();
            --wanted_;
            if (--j->want == 0) q_.pop_front();
            lk.unlock();
            claim_items(*j);  // the job stays alive through the shared_ptr
            lk.lock();
        }
    }
};

Pool& pool() {
    // Leaked at exit on purpose: detached workers may still wait on its condition variable.
    static Pool* p = new Pool(std::max(0, host_cpu_budget() - 1));
    return *p;
}

}  // namespace

int host_pool_idle() { return pool().threads_idle(); }

HostBatch::HostBatch(size_t n, int helpers, std::function<void(size_t)> f) {
    if (n == 0) return;
    j_ = std::make_shared<HostJob>();
    j_->f = std::move(f);
    j_->n = n;
    helpers = (int)std::min<size_t>((size_t)std::max(helpers, 0), n);
    if (helpers > 0) pool().offer(j_, helpers);
}

void HostBatch::join() {
    if (!j_) return;
    claim_items(*j_);
    std::unique_lock<std::mutex> lk(j_->mu);
    j_->cv.wait(lk, [&] { return j_->done == j_->n; });
    lk.unlock();
    j_.reset();
}

void host_parallel_for(size_t n, int helpers, std::function<void(size_t)> f) {
    HostBatch b(n, (int)std::min<size_t>((size_t)std::max(helpers, 0), n ? n - 1 : 0), std::move(f));
    b.join();
}

uint32_t crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return len_b ? gf2_mulmod(crc_a, x8n(len_b, x8().v)) ^ crc_b : crc_a;
}

uint32_t host_crc32_update_par(uint32_t crc, const uint8_t* p, size_t n) {
    constexpr size_t kSpan = size_t(1) << 20;
    const int idle = n >= 2 * kSpan ? host_pool_idle() : 0;
    if (idle <= 0) {
        HostCpuToken tok;
        return host_crc32_update(crc, p, n);
    }
    const size_t spans = std::min<size_t>((n + kSpan - 1) / kSpan, (size_t)idle + 1);
    const size_t len = ((n + spans - 1) / spans + 63) & ~size_t(63);
    std::vector<uint32_t> c(spans, 0);
    host_parallel_for(spans, (int)spans - 1, [&](size_t i) {
        const size_t a = std::min(n, i * len), b = std::min(n, a + len);
        c[i] = host_crc32_update(0, p + a, b - a);
    });
    for (size_t i = 0; i < spans; ++i) {
        const size_t a = std::min(n, i * len), b = std::min(n, a + len);
        crc = crc32_combine(crc, c[i], b - a);
    }
    return crc;
}

}  // namespace krk
