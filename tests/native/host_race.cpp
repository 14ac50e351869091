// host_race.cpp -- the device-free host runtime of libkraken_hip under ThreadSanitizer /
// AddressSanitizer (SURVEY.md section 5 maps the reference's
// `go test -race`, /root/reference/Makefile:104, to a sanitizer run of the C++ shim).
//
// Many threads at once drive every entry point that needs no GPU, the way the reference's
// goroutines call the Go API concurrently (HTTP handlers, the blobrefresh workers, the agent's
// dispatcher): piece sums and piece verification over pageable buffers (host pool + CPU
// tokens), host Digesters and piece streams, the InfoHash batch, the window scheduler (also
// with the tail handoff's drops and chunk cap), chains resumed from midstates piece by piece
// (the tail threads' krk_sha256_resume_host), the offload / tail planners under injected
// rates, and the CPU budget.  Every result is checked
// against the oracle (liboracle.so, test infrastructure).  Then the gather's page registry
// (host_register.hpp) runs its helper threads against a recording stand-in for
// hipHostRegister: the copy-out hazard of VERDICT r05 weak #1 is shown to exist while the
// last windows' segments are live, and to be gone -- no registered page anywhere -- once
// release (finish) has run, which every host-buffer entry point now does before copying out.
//
// Built by kraken_amd/csrc/Makefile (targets tsan / asan) against the sanitizer build of the
// library; run by tests/test_sanitizers.py.  Exit 0 = every check passed (the sanitizer
// exits non-zero on a report: halt_on_error / exitcode in the test's options).
#include <sys/mman.h>

#include <atomic>
#include <cstdio>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kraken_hip.h"
#include "../../include/kraken_hip_internal.h"
#include "../../kraken_amd/csrc/host_register.hpp"
#include "../../oracle/oracle.h"

static std::atomic<int> g_fail{0};
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);              \
            fprintf(stderr, "\n");                     \
            g_fail.fetch_add(1);                       \
        }                                              \
    } while (0)

static uint64_t splitmix(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// ------------------------------------------------------------- concurrent entry points
static void worker(int id, int rounds) {
    uint64_t seed = 0x5EED0000ull + id;
    for (int r = 0; r < rounds; ++r) {
        // a batch of pageable blobs: lengths around pieces and words, one 9 MiB blob so the
        // host pool's task split has more than one task
        const int nb = 6;
        std::vector<std::vector<uint8_t>> blob(nb);
        for (int b = 0; b < nb; ++b) {
            const uint64_t L = b == 0 ? (9u << 20) + 13 : splitmix(seed) % 300000;
            blob[b].resize(L);
            orc_synth_fill(id * 1000 + r * 10 + b, 0, blob[b].data(), L, 0);
        }
        const int64_t P = 1 << 16;
        std::vector<krk_blob> kb(nb);
        uint64_t off = 0;
        for (int b = 0; b < nb; ++b) {
            kb[b] = krk_blob{blob[b].data(), blob[b].size(), P, off};
            off += krk_num_pieces(blob[b].size(), P);
        }
        std::vector<uint32_t> sums(off + 1), ref(off + 1);
        CHECK(krk_piece_sums_host(kb.data(), nb, sums.data()) == 0, "piece_sums_host: %s", krk_last_error());
        for (int b = 0; b < nb; ++b) {
            uint64_t ns = 0, len = 0;
            orc_calc_piece_sums(blob[b].data(), blob[b].size(), P, ref.data() + kb[b].sums_offset, &ns, &len);
        }
        CHECK(memcmp(sums.data(), ref.data(), off * 4) == 0, "piece sums differ from the oracle (thread %d)", id);

        // the agent's verify: every piece of every blob, one expected sum corrupted
        std::vector<const uint8_t*> pp;
        std::vector<uint64_t> pl;
        std::vector<uint32_t> exp;
        for (int b = 0; b < nb; ++b)
            for (uint64_t k = 0; k < krk_num_pieces(blob[b].size(), P); ++k) {
                pp.push_back(blob[b].data() + k * P);
                pl.push_back(std::min<uint64_t>(P, blob[b].size() - k * P));
                exp.push_back(ref[kb[b].sums_offset + k]);
            }
        if (!exp.empty()) exp[exp.size() / 2] ^= 1;
        std::vector<uint8_t> ok(exp.size() + 1);
        CHECK(krk_verify_pieces_host(pp.data(), pl.data(), exp.data(), exp.size(), ok.data()) == 0,
              "verify_pieces_host: %s", krk_last_error());
        for (size_t k = 0; k < exp.size(); ++k)
            CHECK(ok[k] == (k == exp.size() / 2 ? 0 : 1), "verify piece %zu", k);

        // host Digesters and piece streams (the reference's Digester / PieceHash per goroutine)
        for (int b = 0; b < nb; ++b) {
            krk_digester* d = nullptr;
            CHECK(krk_digester_new_on(KRK_PLACE_HOST, &d) == 0, "digester_new_on");
            krk_piece_stream* ps = nullptr;
            CHECK(krk_piece_stream_begin_on(KRK_PLACE_HOST, P, &ps) == 0, "piece_stream_begin_on");
            uint64_t pos = 0;
            while (pos < blob[b].size()) {
                const uint64_t take = std::min<uint64_t>(blob[b].size() - pos, 1 + splitmix(seed) % 100000);
                krk_digester_write(d, blob[b].data() + pos, take);
                krk_piece_stream_update(ps, blob[b].data() + pos, take);
                pos += take;
            }
            uint8_t dg[32], rd[32];
            CHECK(krk_digester_sum(d, dg) == 0, "digester_sum");
            orc_sha256(blob[b].data(), blob[b].size(), rd);
            CHECK(memcmp(dg, rd, 32) == 0, "digester differs (thread %d blob %d)", id, b);
            std::vector<uint32_t> s(krk_num_pieces(blob[b].size(), P) + 1);
            uint64_t ns = 0, len = 0;
            CHECK(krk_piece_stream_end(ps, s.data(), s.size(), &ns, &len) == 0, "piece_stream_end");
            CHECK(ns == krk_num_pieces(blob[b].size(), P) && len == blob[b].size(), "piece stream counts");
            CHECK(memcmp(s.data(), ref.data() + kb[b].sums_offset, ns * 4) == 0, "piece stream sums");
            krk_piece_stream_free(ps);
            krk_digester_free(d);
            uint32_t c = 0;
            CHECK(krk_crc32_update_on(KRK_PLACE_HOST, 0, blob[b].data(), blob[b].size(), &c) == 0, "crc32_update_on");
            CHECK(c == orc_crc32_update(0, blob[b].data(), blob[b].size()), "crc32_update_on value");
        }

        // the InfoHash batch (host threads)
        std::vector<int64_t> pls(nb, P), lens(nb);
        std::vector<uint64_t> soff(nb), nsum(nb), noff(nb + 1);
        std::string names;
        for (int b = 0; b < nb; ++b) {
            lens[b] = (int64_t)blob[b].size();
            soff[b] = kb[b].sums_offset;
            nsum[b] = krk_num_pieces(blob[b].size(), P);
            noff[b] = names.size();
            char nm[65];
            snprintf(nm, sizeof nm, "%064llx", (unsigned long long)splitmix(seed));
            names += nm;
        }
        noff[nb] = names.size();
        std::vector<uint8_t> ih(20 * nb);
        CHECK(krk_info_hash_batch(pls.data(), ref.data(), soff.data(), nsum.data(), names.data(), noff.data(),
                                  lens.data(), nb, ih.data()) == 0,
              "info_hash_batch: %s", krk_last_error());
        for (int b = 0; b < nb; ++b) {
            uint8_t want[20];
            orc_info_hash(P, ref.data() + soff[b], nsum[b], names.data() + noff[b], noff[b + 1] - noff[b], lens[b],
                          want);
            CHECK(memcmp(want, ih.data() + 20 * b, 20) == 0, "info hash %d", b);
        }

        // the window scheduler: every byte of every blob exactly once, in order per blob
        std::vector<uint64_t> L(40);
        for (auto& x : L) x = splitmix(seed) % 5000000;
        krk_window_sched* ws = nullptr;
        CHECK(krk_window_sched_new(L.data(), L.size(), 8u << 20, 16, &ws) == 0, "window_sched_new");
        std::vector<uint64_t> done(L.size(), 0);
        std::vector<uint32_t> wb(64);
        std::vector<uint64_t> wo(64), wl(64);
        for (;;) {
            uint64_t k = 0;
            CHECK(krk_window_sched_next(ws, wb.data(), wo.data(), wl.data(), 64, &k) == 0, "window_sched_next");
            if (!k) break;
            for (uint64_t j = 0; j < k; ++j) {
                CHECK(wo[j] == done[wb[j]], "window chunk out of order");
                done[wb[j]] += wl[j];
            }
        }
        krk_window_sched_free(ws);
        for (size_t j = 0; j < L.size(); ++j) CHECK(done[j] == L[j], "window schedule lost bytes of blob %zu", j);

        // the planners (rates set by the main thread; read here concurrently)
        std::vector<uint64_t> pl2(200);
        for (auto& x : pl2) x = (100ull << 20) + splitmix(seed) % (900ull << 20);
        std::vector<uint32_t> hidx(pl2.size());
        std::vector<uint64_t> start(pl2.size());
        uint64_t nh = 0;
        double g = 0, h = 0;
        CHECK(krk_host_offload_plan(pl2.data(), pl2.size(), 8, 256, KRK_OFFLOAD_HOST_WHOLE, hidx.data(), &nh, &g, &h) == 0,
              "host_offload_plan");
        for (uint64_t j = 1; j < nh; ++j) CHECK(pl2[hidx[j - 1]] >= pl2[hidx[j]], "offload plan not longest first");
        double e = 0;
        CHECK(krk_sha_tail_plan(pl2.data(), pl2.size(), 8, hidx.data(), start.data(), &nh, &e, &g) == 0,
              "sha_tail_plan");
        for (uint64_t j = 0; j < nh; ++j) CHECK(start[j] % 64 == 0 && start[j] < pl2[hidx[j]], "tail start");
        // the windowed tail handoff's host side (round 6): chains continued on many threads at
        // once from a midstate, piece by piece (krk_sha256_resume_host: whole blocks, then a final
        // run), with the per-thread stats read beside them
        {
            const std::vector<uint8_t>& B = blob[0];
            uint32_t st[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                              0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};
            uint64_t pos = 0;
            uint8_t dg[32] = {}, rd[32];
            for (;;) {
                const uint64_t left = B.size() - pos;
                const uint64_t take = std::min<uint64_t>(left, 64 * (1 + splitmix(seed) % 40000));
                const int fin = take == left;
                CHECK(krk_sha256_resume_host(st, pos, B.data() + pos, fin ? take : take / 64 * 64, fin, dg) == 0,
                      "sha256_resume_host: %s", krk_last_error());
                if (fin) break;
                pos += take / 64 * 64;
            }
            orc_sha256(B.data(), B.size(), rd);
            CHECK(memcmp(dg, rd, 32) == 0, "resumed chain differs (thread %d)", id);
            double w = 0, hs = 0;
            CHECK(krk_sha256_resume_stats(&w, &hs) == 0 && hs >= 0, "sha256_resume_stats");
        }
        // ... and its schedule: chains dropped from the windows as threads steal them (a dropped
        // blob gets no chunk after the drop, every other blob every byte in order), with the
        // chunk cap the handoff sets
        {
            std::vector<uint64_t> L2(48);
            for (auto& x : L2) x = 64 + splitmix(seed) % 3000000;
            krk_window_sched* ws2 = nullptr;
            CHECK(krk_window_sched_new(L2.data(), L2.size(), 4u << 20, 12, &ws2) == 0, "window_sched_new (drops)");
            CHECK(krk_window_sched_set_chunk_cap(ws2, 1u << 18) == 0, "window_sched_set_chunk_cap");
            std::vector<uint64_t> got(L2.size(), 0);
            std::vector<char> dropped(L2.size(), 0);
            std::vector<uint32_t> b2(64);
            std::vector<uint64_t> o2(64), l2(64);
            for (int w = 0;; ++w) {
                uint64_t k = 0;
                CHECK(krk_window_sched_next(ws2, b2.data(), o2.data(), l2.data(), 64, &k) == 0, "window_sched_next");
                if (!k) break;
                for (uint64_t j = 0; j < k; ++j) {
                    CHECK(!dropped[b2[j]], "a dropped blob got a chunk");
                    CHECK(o2[j] == got[b2[j]] && l2[j] <= (1u << 18), "chunk order / cap");
                    got[b2[j]] += l2[j];
                }
                if (w % 3 == 1) {  // a thread steals one chain (live or still waiting)
                    const uint32_t b = (uint32_t)(splitmix(seed) % L2.size());
                    uint64_t at = 0;
                    if (!dropped[b] && got[b] < L2[b]) {
                        CHECK(krk_window_sched_drop(ws2, b, &at) == 0 && at == got[b], "window_sched_drop");
                        dropped[b] = 1;
                    }
                }
            }
            krk_window_sched_free(ws2);
            for (size_t j = 0; j < L2.size(); ++j)
                CHECK(dropped[j] || got[j] == L2[j], "schedule with drops lost bytes of blob %zu", j);
        }
        int cpus = 0, node = 0;
        char src[64];
        CHECK(krk_host_cpu_budget(&cpus, &node, src, sizeof src) == 0 && cpus >= 1, "host_cpu_budget");
        uint8_t hd[32], rd[32];
        CHECK(krk_host_sha256(blob[0].data(), blob[0].size(), hd) == 0, "host_sha256");
        orc_sha256(blob[0].data(), blob[0].size(), rd);
        CHECK(memcmp(hd, rd, 32) == 0, "host_sha256 value");
    }
}

// ------------------------------------------------------------- the page registry
static std::mutex g_reg_mu;
static std::set<uintptr_t> g_reg_pages;  // pages the stand-in holds "registered"
static std::atomic<int> g_reg_calls{0};

static hipError_t fake_register(void* p, size_t n, unsigned) {
    std::lock_guard<std::mutex> g(g_reg_mu);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    if (a % 4096 || n % 4096) return hipErrorInvalidValue;
    for (uintptr_t q = a; q < a + n; q += 4096)
        if (g_reg_pages.count(q)) return hipErrorHostMemoryAlreadyRegistered;
    for (uintptr_t q = a; q < a + n; q += 4096) g_reg_pages.insert(q);
    g_reg_calls.fetch_add(1);
    return hipSuccess;
}
static std::map<uintptr_t, size_t>* g_reg_len = new std::map<uintptr_t, size_t>();
static hipError_t fake_register_len(void* p, size_t n, unsigned f) {
    hipError_t e = fake_register(p, n, f);
    if (e == hipSuccess) {
        std::lock_guard<std::mutex> g(g_reg_mu);
        (*g_reg_len)[reinterpret_cast<uintptr_t>(p)] = n;
    }
    return e;
}
static hipError_t fake_unregister(void* p) {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg_len->find(reinterpret_cast<uintptr_t>(p));
    if (it == g_reg_len->end()) return hipErrorHostMemoryNotRegistered;
    for (uintptr_t q = it->first; q < it->first + it->second; q += 4096) g_reg_pages.erase(q);
    g_reg_len->erase(it);
    return hipSuccess;
}
static hipError_t fake_dev_ptr(void** d, void* p, unsigned) {
    *d = p;
    return hipSuccess;
}

static bool any_registered(const void* p, size_t n) {
    std::lock_guard<std::mutex> g(g_reg_mu);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p) & ~uintptr_t(4095), b = reinterpret_cast<uintptr_t>(p) + n;
    for (uintptr_t q = a; q < b; q += 4096)
        if (g_reg_pages.count(q)) return true;
    return false;
}

static void registry_case(int rep) {
    // one page-aligned buffer: page 0 holds a tiny blob AND the call's output arrays (the
    // layout of tests/test_gpu_gather.py::test_copyout_shares_page_with_registered_blob); the
    // other blobs follow, a few MiB each, so the schedule has several windows
    const size_t PAGE = 4096, BYTES = 64ull << 20;
    uint8_t* buf = static_cast<uint8_t*>(mmap(nullptr, BYTES, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    CHECK(buf != MAP_FAILED, "mmap");
    uint8_t* tiny = buf + 64;
    const size_t tiny_len = 200;
    uint8_t* out = buf + 1024;  // digests / sums of the call
    const size_t out_len = 2048;
    std::vector<std::pair<uintptr_t, uintptr_t>> ranges;
    std::vector<std::pair<uint8_t*, size_t>> blobs;
    blobs.push_back({tiny, tiny_len});
    for (size_t o = PAGE + 7; o + (3u << 20) < BYTES; o += (3u << 20) + 4099) blobs.push_back({buf + o, 3u << 20});
    for (auto& b : blobs) ranges.push_back({reinterpret_cast<uintptr_t>(b.first), reinterpret_cast<uintptr_t>(b.first) + b.second});
    krk::RegBackend be;
    be.reg = fake_register_len;
    be.unreg = fake_unregister;
    be.dev_ptr = fake_dev_ptr;
    {
        krk::HostRegistry reg(ranges, be);
        // windows of 4 blobs each, the tiny blob read in the LAST window (as a short blob
        // admitted last is): its page stays registered until release
        const int per = 4, nw = (int)((blobs.size() - 1 + per - 1) / per) + 1;
        for (int w = 0; w < nw - 1; ++w)
            for (int k = 0; k < per; ++k) {
                const size_t j = 1 + w * per + k;
                if (j < blobs.size()) reg.need(w, blobs[j].first, blobs[j].second);
            }
        reg.need(nw - 1, tiny, tiny_len);
        reg.start(4);
        const int ring = 3;  // staging windows: window w - ring's copy is known done at w
        for (int w = 0; w < nw; ++w) {
            CHECK(reg.ready(w), "window %d not registered", w);
            if (w >= ring) reg.copied(w - ring);
            // the gather "reads" window w: its blobs must be registered now
            for (int k = 0; k < per && w < nw - 1; ++k) {
                const size_t j = 1 + w * per + k;
                if (j < blobs.size()) CHECK(any_registered(blobs[j].first, 1), "blob %zu read unregistered", j);
            }
        }
        // the hazard: before release, the output arrays share a registered page
        CHECK(reg.live_segments() > 0, "rep %d: nothing live before release", rep);
        CHECK(reg.overlaps_live(out, out_len), "rep %d: output page not registered before release", rep);
        CHECK(any_registered(out, out_len), "stand-in disagrees with overlaps_live");
        // release (windows.cpp release_caller_pages), then the copy-out and any bounce buffer
        reg.finish(nullptr);
        CHECK(reg.live_segments() == 0, "rep %d: %llu segments live after release", rep,
              (unsigned long long)reg.live_segments());
        CHECK(!reg.overlaps_live(out, out_len), "rep %d: output still registered after release", rep);
        CHECK(!any_registered(out, out_len), "rep %d: stand-in still holds the output page", rep);
        std::vector<uint8_t> bounce(out_len);
        CHECK(!any_registered(bounce.data(), bounce.size()), "a heap buffer overlaps a registered page");
        memset(out, 0x5A, out_len);  // the copy-out itself
        reg.finish(nullptr);         // idempotent (the filler's destructor calls it again)
    }
    {
        std::lock_guard<std::mutex> g(g_reg_mu);
        CHECK(g_reg_pages.empty(), "rep %d: %zu pages left registered", rep, g_reg_pages.size());
    }
    munmap(buf, BYTES);
}

int main(int argc, char** argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 8;
    const int rounds = argc > 2 ? atoi(argv[2]) : 2;
    // the planners with injected rates (no device): read concurrently by the workers while
    // the main thread sets them again
    krk_planner_rates R{};
    R.sha_stream_bps[0] = 50e6;
    R.sha_stream_bps[1] = 52e6;
    R.sha_stream_bps[2] = 30e6;
    R.d2h_bps = R.h2d_bps = 55e9;
    R.host_sha_bps = 2.0e9;
    R.host_crc_bps = 15e9;
    R.host_copy_bps = 10e9;
    R.cus = 256;
    CHECK(krk_planner_rates_set(&R) == 0, "planner_rates_set");
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(worker, t, rounds);
    for (int k = 0; k < 20; ++k) {
        R.host_sha_bps = 1.5e9 + 0.05e9 * k;
        krk_planner_rates_set(&R);
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    // the registry's helper threads at the same time as the workers
    std::thread reg_th([] {
        for (int rep = 0; rep < 4; ++rep) registry_case(rep);
    });
    for (auto& t : th) t.join();
    reg_th.join();
    krk_planner_rates_set(nullptr);
    const int f = g_fail.load();
    printf("host_race: %d threads x %d rounds, %d registrations, %s\n", threads, rounds, g_reg_calls.load(),
           f ? "FAILED" : "ok");
    return f ? 1 : 0;
}
