// digesters.cpp -- N concurrent GPU Digesters driven from native threads, the way the
// reference's goroutines drive core.Digester (origin/blobserver/uploader.go:75,
// lib/store/ca_store.go:119): each thread owns one digester, writes its blob in
// random-sized chunks (io.Copy-like), then asks for the digest.  Links the product
// library through its C ABI only (include/kraken_hip.h), as a cgo caller would.
//
//   digesters <n_digesters> <MiB per digester> <rounds> [max write bytes] [gpu|host|auto] [threads]
//
// With fewer threads than digesters (the crossover sweep: thousands of uploads, few OS
// threads, like goroutines on GOMAXPROCS threads), each thread drives its digesters
// round-robin, one write each in turn.  placement: KRK_PLACE_GPU (default), HOST or AUTO.
//
// Prints one JSON line per round: aggregate GB/s (timed from the moment every thread
// holds its digester until the last digest), streams per SHA launch, and whether every
// digest equals krk_host_sha256 of the same bytes (the host SHA-NI path, itself checked
// against hashlib by tests/test_capi_cpu.py).  Exit 1 on any mismatch or error.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <pthread.h>

#include <random>
#include <thread>
#include <vector>

#include "../../include/kraken_hip_internal.h"

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 256;
    const size_t L = (size_t)(argc > 2 ? atoi(argv[2]) : 16) << 20;
    const int rounds = argc > 3 ? atoi(argv[3]) : 2;
    const size_t maxw = argc > 4 ? strtoull(argv[4], nullptr, 10) : (1u << 20);
    const char* pl = argc > 5 ? argv[5] : "gpu";
    const int place = !strcmp(pl, "host") ? KRK_PLACE_HOST : !strcmp(pl, "auto") ? KRK_PLACE_AUTO : KRK_PLACE_GPU;
    const int nt = std::min(n, argc > 6 ? atoi(argv[6]) : n);
    if (n < 1 || L == 0 || maxw == 0 || nt < 1) return 2;
    if (krk_set_device(0) != KRK_OK) {
        fprintf(stderr, "no device: %s\n", krk_last_error());
        return 1;
    }
    // blob i = bytes [i * 4096, i * 4096 + L) of one random buffer
    std::vector<uint8_t> base(L + (size_t)n * 4096);
    std::mt19937_64 g(256);
    for (size_t k = 0; k + 8 <= base.size(); k += 8) {
        const uint64_t v = g();
        memcpy(&base[k], &v, 8);
    }
    std::vector<std::array<uint8_t, 32>> want(n);
    {
        std::vector<std::thread> th;
        std::atomic<int> next{0};
        for (int t = 0; t < 16; ++t)
            th.emplace_back([&] {
                for (int i; (i = next.fetch_add(1)) < n;) krk_host_sha256(base.data() + (size_t)i * 4096, L, want[i].data());
            });
        for (auto& t : th) t.join();
    }
    bool all_ok = true;
    for (int r = 0; r < rounds; ++r) {
        uint64_t b0[5], b1[5];
        krk_engine_stats(&b0[0], &b0[1], &b0[2], &b0[3], &b0[4]);
        // start line: every thread holds its digester, then all are released at once by a
        // barrier (one futex wake for all; a condition variable woke 256 waiters one mutex
        // handoff at a time, ~15 ms).  Not a spin on a flag: the GPU boxes grant a CPU
        // QUOTA (16 CPUs' worth) over many more CPUs, and 256 threads spinning on yield()
        // burnt it, so the whole process was throttled for the rest of the quota period
        // (~90 ms stalls in a third of the rounds: tools/engine_slow.py).
        pthread_barrier_t start;
        pthread_barrier_init(&start, nullptr, (unsigned)nt + 1);
        std::atomic<int> bad{0}, on_gpu{0};
        std::vector<std::thread> th;
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&, t] {
                krk_set_device(0);
                struct Own {
                    int i;
                    krk_digester* d;
                    std::mt19937_64 rg;
                    size_t pos;
                };
                std::vector<Own> own;
                for (int i = t; i < n; i += nt) {
                    krk_digester* d = nullptr;
                    if (krk_digester_new_on(place, &d) != KRK_OK) {
                        bad.fetch_add(1);
                        continue;
                    }
                    int where = 0;
                    krk_digester_placement(d, &where);
                    if (where == KRK_PLACE_GPU) on_gpu.fetch_add(1);
                    own.push_back({i, d, std::mt19937_64((uint64_t)i * 7919 + r), 0});
                }
                pthread_barrier_wait(&start);  // every thread arrives, made or not
                for (size_t live = own.size(); live;) {
                    live = 0;
                    for (Own& o : own) {  // one write per digester in turn
                        if (!o.d || o.pos >= L) continue;
                        const uint8_t* p = base.data() + (size_t)o.i * 4096;
                        const size_t k = std::min<size_t>(L - o.pos, 1 + o.rg() % maxw);
                        if (krk_digester_write(o.d, p + o.pos, k) != KRK_OK) {
                            bad.fetch_add(1);
                            o.pos = L;
                            continue;
                        }
                        o.pos += k;
                        live += o.pos < L;
                    }
                }
                for (Own& o : own) {
                    uint8_t out[32];
                    if (krk_digester_sum(o.d, out) != KRK_OK || memcmp(out, want[o.i].data(), 32) != 0) bad.fetch_add(1);
                    krk_digester_free(o.d);
                }
            });

        // DIGESTERS_CLOCK=1: sample the shader clock every ~20 ms during the round
        // (krk_device_clock_mhz on a stream of its own)
        std::vector<double> clocks;
        std::atomic<bool> done{false};
        std::thread clk;
        if (getenv("DIGESTERS_CLOCK"))
            clk = std::thread([&] {
                krk_set_device(0);
                void* cs = nullptr;
                krk_stream_create(&cs);
                while (!done.load()) {
                    double m = 0;
                    if (krk_device_clock_mhz(cs, &m) == KRK_OK) clocks.push_back(m);
                    std::this_thread::sleep_for(std::chrono::milliseconds(20));
                }
                krk_stream_destroy(cs);
            });
        const auto t0 = std::chrono::steady_clock::now();
        pthread_barrier_wait(&start);  // the last arrival releases every thread
        for (auto& t : th) t.join();
        pthread_barrier_destroy(&start);
        done = true;
        if (clk.joinable()) clk.join();
        std::sort(clocks.begin(), clocks.end());
        const double clk_med = clocks.empty() ? 0.0 : clocks[clocks.size() / 2];
        const double clk_min = clocks.empty() ? 0.0 : clocks.front();
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        krk_engine_stats(&b1[0], &b1[1], &b1[2], &b1[3], &b1[4]);
        const double agg = (double)n * L / el;
        const bool ok = bad.load() == 0;
        all_ok = all_ok && ok;
        printf("{\"round\": %d, \"t_go_ms\": %.3f, \"digesters\": %d, \"threads\": %d, \"placement\": \"%s\", "
               "\"on_gpu\": %d, \"bytes_each\": %zu, \"seconds\": %.4f, \"GBps\": %.3f, "
               "\"MBps_per_stream\": %.2f, \"sha_launches\": %llu, \"streams_per_launch\": %.1f, "
               "\"pinned_bytes\": %llu, \"clock_mhz_median\": %.0f, \"clock_mhz_min\": %.0f, \"digests_match\": %s}\n",
               r, std::chrono::duration<double, std::milli>(t0.time_since_epoch()).count(), n, nt, pl, on_gpu.load(), L, el,
               agg / 1e9, agg / n / 1e6, (unsigned long long)(b1[0] - b0[0]),
               (double)(b1[1] - b0[1]) / (double)std::max<uint64_t>(1, b1[0] - b0[0]),
               (unsigned long long)b1[4], clk_med, clk_min, ok ? "true" : "false");
        fflush(stdout);
    }
    return all_ok ? 0 : 1;
}
