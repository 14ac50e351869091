// host_register.hpp -- internal to libkraken_hip: the caller's pageable blobs of one
// host-resident call made page-locked for the GPU's gather (gather.hip, DESIGN.md 4.5,
// VERDICT r04 item 3).
//
// The staged path copies every byte pageable -> pinned window on host threads (a host-DRAM
// read and write) before the DMA reads it again: three host-DRAM touches a byte and most of
// a rank's CPU share in copy threads.  Here the blobs' pages are registered with
// hipHostRegister instead -- no byte is touched on the host -- and each window goes up in
// ONE gather launch that reads the registered pages over PCIe: one host-DRAM read a byte, by
// the GPU.  Used only when KRK_HOST_GATHER=1 asks for it: measured on MI355X it loses to
// the staging copy for ordinary 4 KiB-page memory (C2 end to end 28.4 against 53.9 GB/s,
// profiles/r05/bench_c2.json; registration of fresh pages 20-45 GB/s whatever the thread
// count, profiles/r05/reg_probe.jsonl), so the default stages pageable blobs and gathers
// only page-locked ones.
//
// Registration runs ahead of the window loop on a few helper threads, segment by segment
// (<= kRegSeg bytes of page-aligned, merged blob ranges), in the order the window schedule
// first reads them and at most kRegAhead windows ahead, and a segment is unregistered once
// the window that last reads it has been copied: the call keeps a bounded amount of the
// caller's memory pinned.  A segment that cannot be registered (read-only or foreign
// mappings, a range someone else registered, a device pointer that is not the host address)
// turns the gather off for the rest of the call: the windows stage as before.
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "runtime.hpp"

namespace krk {

// The HIP calls the registry makes, swappable so that the schedule and the page accounting
// run on a CPU with a recording stand-in (tests/native/registry_race.cpp under TSan/ASan).
struct RegBackend {
    hipError_t (*reg)(void* p, size_t n, unsigned flags) = hipHostRegister;
    hipError_t (*unreg)(void* p) = hipHostUnregister;
    hipError_t (*dev_ptr)(void** d, void* p, unsigned flags) = hipHostGetDevicePointer;
};

class HostRegistry {
  public:
    static constexpr uint64_t kPage = 4096;
    static constexpr uint64_t kRegSeg = 16ull << 20;  // bytes a hipHostRegister call
    static constexpr int kRegAhead = 6;               // windows registered ahead of the loop

    // [a, b) ranges of the blobs the windows will read (any alignment, may overlap)
    explicit HostRegistry(std::vector<std::pair<uintptr_t, uintptr_t>> ranges, RegBackend be = RegBackend())
        : be_(be) {
        for (auto& r : ranges) {
            r.first &= ~(kPage - 1);
            r.second = (r.second + kPage - 1) & ~(kPage - 1);
        }
        std::sort(ranges.begin(), ranges.end());
        std::vector<std::pair<uintptr_t, uintptr_t>> merged;
        for (const auto& r : ranges) {
            if (r.first >= r.second) continue;
            if (!merged.empty() && r.first <= merged.back().second)
                merged.back().second = std::max(merged.back().second, r.second);
            else
                merged.push_back(r);
        }
        for (const auto& m : merged)
            for (uintptr_t a = m.first; a < m.second; a += kRegSeg)
                seg_.push_back({a, std::min<uintptr_t>(m.second, a + kRegSeg)});
    }
    ~HostRegistry() { finish(nullptr); }

    bool empty() const { return seg_.empty(); }

    // Window w reads [p, p + n): the segments it touches must be registered by then, and stay
    // so until window w has been copied.  Called for every chunk of the dry-run schedule,
    // windows in order, before start().
    void need(int w, const uint8_t* p, uint64_t n) {
        if (!n) return;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p), b = a + n;
        auto it = std::upper_bound(seg_.begin(), seg_.end(), a, [](uintptr_t x, const Seg& s) { return x < s.b; });
        for (; it != seg_.end() && it->a < b; ++it) {
            if (it->first < 0) it->first = w;
            it->last = std::max(it->last, w);
        }
        windows_ = std::max(windows_, w + 1);
    }

    // Register in first-need order on `threads` helper threads.
    void start(int threads) {
        order_.resize(seg_.size());
        for (size_t i = 0; i < seg_.size(); ++i) order_[i] = (uint32_t)i;
        std::stable_sort(order_.begin(), order_.end(), [&](uint32_t x, uint32_t y) { return seg_[x].first < seg_[y].first; });
        need_count_.assign(windows_ + 1, 0);
        // a segment no window reads (none should exist) sorts first and counts as window 0's,
        // so "the first k segments are registered" always means window w's are
        for (uint32_t i : order_) need_count_[std::max(seg_[i].first, 0) + 1]++;
        for (int w = 0; w < windows_; ++w) need_count_[w + 1] += need_count_[w];
        state_ = std::vector<std::atomic<int>>(seg_.size());
        for (auto& s : state_) s.store(kPending);
        done_.assign(order_.size(), 0);
        const int dev = t_dev;
        for (int t = 0; t < std::max(1, threads); ++t)
            th_.emplace_back([this, dev] {
                hipSetDevice(dev);
                worker();
            });
    }

    // Before window w's gather: true once every segment it reads is registered (and the
    // registered pointers are the host addresses); false: stage this window (and the gather
    // is off for the rest of the call).
    bool ready(int w) {
        std::unique_lock<std::mutex> lk(mu_);
        cur_ = std::max(cur_, w);
        cv_work_.notify_all();
        const size_t want = need_count_[std::min(w + 1, windows_)];
        cv_done_.wait(lk, [&] { return failed_ || prefix_ >= want; });
        return !failed_;
    }

    // Window w has been copied to the device (its gather finished): segments whose last
    // reader is at or before w are unregistered.
    void copied(int w) {
        std::lock_guard<std::mutex> g(mu_);
        for (size_t q = retired_; q < prefix_; ++q) {
            const uint32_t i = order_[q];
            if (state_[i].load() == kRegistered && seg_[i].last <= w) {
                be_.unreg(reinterpret_cast<void*>(seg_[i].a));
                state_[i].store(kReleased);
            }
        }
        while (retired_ < prefix_ && state_[order_[retired_]].load() != kRegistered) ++retired_;
    }

    // End of the call: stop the helpers; once `s` (the stream the gathers ran on) has drained,
    // unregister what is left.
    void finish(hipStream_t s) {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_work_.notify_all();
        for (auto& t : th_) t.join();
        th_.clear();
        if (s) hipStreamSynchronize(s);
        for (size_t i = 0; i < state_.size(); ++i)
            if (state_[i].load() == kRegistered) {
                be_.unreg(reinterpret_cast<void*>(seg_[i].a));
                state_[i].store(kReleased);
            }
    }

    // Segments registered now (0 once finish() has returned): every host-buffer entry point
    // reports this at its copy-out (krk_windows_last_copyout).
    uint64_t live_segments() const {
        uint64_t k = 0;
        for (const auto& s : state_) k += s.load() == kRegistered;
        return k;
    }
    // Whether [p, p + n) touches a page of a segment registered now: a HIP copy whose
    // destination starts in a registered page and runs past it is refused, so no copy-out
    // may target one.
    bool overlaps_live(const void* p, uint64_t n) const {
        if (!n) return false;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p) & ~(kPage - 1), b = reinterpret_cast<uintptr_t>(p) + n;
        for (size_t i = 0; i < seg_.size(); ++i)
            if (state_[i].load() == kRegistered && seg_[i].a < b && a < seg_[i].b) return true;
        return false;
    }

    uint64_t registered_bytes() const { return reg_bytes_.load(); }
    double register_seconds() const { return reg_ns_.load() * 1e-9; }
    bool failed() const { return failed_; }

  private:
    enum { kPending = 0, kRegistered = 1, kFailed = 2, kReleased = 3 };
    struct Seg {
        uintptr_t a, b;
        int first = -1, last = -1;  // windows that first / last read the segment
    };
    RegBackend be_;
    std::vector<Seg> seg_;
    std::vector<uint32_t> order_;       // registration order (first-need window)
    std::vector<size_t> need_count_;    // need_count_[w + 1]: segments windows 0..w need
    std::vector<std::atomic<int>> state_;
    int windows_ = 0;
    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    size_t next_ = 0;     // next segment (in order_) a helper claims
    size_t prefix_ = 0;   // segments order_[0, prefix_) are registered
    size_t retired_ = 0;  // order_[0, retired_) are released
    int cur_ = 0;         // the window the loop is at
    bool stop_ = false, failed_ = false;
    std::vector<char> done_;  // per order position: registered
    std::vector<std::thread> th_;
    std::atomic<uint64_t> reg_bytes_{0}, reg_ns_{0};

    void worker() {
        for (;;) {
            size_t q;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_work_.wait(lk, [&] {
                    return stop_ || failed_ ||
                           (next_ < order_.size() && seg_[order_[next_]].first <= cur_ + kRegAhead);
                });
                if (stop_ || failed_ || next_ >= order_.size()) return;
                q = next_++;
            }
            const Seg& s = seg_[order_[q]];
            const auto t0 = std::chrono::steady_clock::now();
            void* p = reinterpret_cast<void*>(s.a);
            hipError_t e = be_.reg(p, s.b - s.a, hipHostRegisterMapped);
            bool ok = e == hipSuccess;
            if (ok) {
                void* d = nullptr;  // the gather reads the host address itself
                ok = be_.dev_ptr(&d, p, 0) == hipSuccess && d == p;
                if (!ok) be_.unreg(p);
            } else {
                (void)hipGetLastError();  // a refused range: staged instead, not an error of the call
            }
            reg_ns_.fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
                                  std::chrono::steady_clock::now() - t0).count());
            std::lock_guard<std::mutex> g(mu_);
            state_[order_[q]].store(ok ? kRegistered : kFailed);
            if (!ok) failed_ = true;
            else reg_bytes_.fetch_add(s.b - s.a);
            done_[q] = 1;
            while (prefix_ < order_.size() && done_[prefix_]) ++prefix_;
            cv_done_.notify_all();
            cv_work_.notify_all();
        }
    }
};

}  // namespace krk
