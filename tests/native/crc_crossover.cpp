// crc_crossover.cpp -- the measurements behind the CRC placement crossover:
// NewMetaInfo piece streams (core/metainfo.go:157-179) and PieceHash crc32.Update calls
// (lib/torrent/storage/agentstorage/torrent.go:182-193) driven from native threads, as the
// cgo layer's goroutines drive them, on each placement:
//
//   * one stream over 1 GiB in 4 MiB writes (HOST / GPU / AUTO);
//   * N concurrent streams (N = 4, 16, 64), 128 MiB each in 4 MiB writes;
//   * one thread's crc32_update calls of 64 KiB .. 256 MiB;
//   * 64 threads' crc32_update calls of 4 MiB (an agent verifying received pieces).
//
// Every stream / thread reads bytes of its own (no two share cache lines), and every case
// repeats its work until it has run for at least ~0.4 s, so neither the host's caches nor a
// CPU quota's first-period burst inflates a rate.  Every result is compared with
// krk_host_crc32_update over the same bytes (itself checked against zlib by
// tests/test_capi_cpu.py).  One JSON line per case; exit 1 on a mismatch.
//
//   crc_crossover [scale]   (scale < 1 shrinks every size, for a quick run)
#include <pthread.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kraken_hip_internal.h"

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a) { return std::chrono::duration<double>(Clock::now() - a).count(); }
const char* pname(int p) { return p == KRK_PLACE_HOST ? "host" : p == KRK_PLACE_GPU ? "gpu" : "auto"; }

std::vector<uint8_t> g_buf;
uint64_t g_region = 0;  // bytes of g_buf each thread of the update cases owns
bool g_ok = true;

// One piece stream over [p, p + L) in `w`-byte writes; returns its sums (placement to *where).
std::vector<uint32_t> stream(int placement, const uint8_t* p, uint64_t L, uint64_t P, uint64_t w, int* where) {
    krk_piece_stream* s = nullptr;
    if (krk_piece_stream_begin_on(placement, (int64_t)P, &s) != KRK_OK) {
        fprintf(stderr, "begin: %s\n", krk_last_error());
        g_ok = false;
        return {};
    }
    krk_piece_stream_placement(s, where);
    for (uint64_t a = 0; a < L; a += w)
        if (krk_piece_stream_update(s, p + a, std::min(w, L - a)) != KRK_OK) {
            fprintf(stderr, "update: %s\n", krk_last_error());
            g_ok = false;
            break;
        }
    uint64_t n = 0, len = 0;
    std::vector<uint32_t> sums((L + P - 1) / P);
    if (krk_piece_stream_end(s, sums.data(), sums.size(), &n, &len) != KRK_OK || n != sums.size() || len != L) {
        fprintf(stderr, "end: %s\n", krk_last_error());
        g_ok = false;
    }
    krk_piece_stream_free(s);
    return sums;
}

std::vector<uint32_t> host_sums(const uint8_t* p, uint64_t L, uint64_t P) {
    std::vector<uint32_t> s;
    for (uint64_t a = 0; a < L; a += P) {
        uint32_t c = 0;
        krk_host_crc32_update(0, p + a, std::min(P, L - a), &c);
        s.push_back(c);
    }
    return s;
}

constexpr double kMinSeconds = 0.4;

void run_streams(int placement, int n, uint64_t L, uint64_t P, uint64_t w, int reps) {
    std::vector<std::vector<uint32_t>> want(n);
    for (int i = 0; i < n; ++i) want[i] = host_sums(g_buf.data() + (size_t)i * L, L, P);
    double best = 1e30;
    int where_host = 0, where_gpu = 0;
    bool ok = true;
    int loops = 1;
    for (int r = 0; r < reps; ++r) {
        pthread_barrier_t start;
        pthread_barrier_init(&start, nullptr, (unsigned)n + 1);
        std::vector<std::thread> th;
        std::vector<int> where(n, -1);
        std::vector<char> good(n, 0);
        for (int i = 0; i < n; ++i)
            th.emplace_back([&, i] {
                krk_set_device(0);
                pthread_barrier_wait(&start);
                bool g = true;
                for (int l = 0; l < loops; ++l)
                    g = stream(placement, g_buf.data() + (size_t)i * L, L, P, w, &where[i]) == want[i] && g;
                good[i] = g;
            });
        const auto t0 = Clock::now();
        pthread_barrier_wait(&start);
        for (auto& t : th) t.join();
        const double el = secs(t0);
        best = std::min(best, el / loops);
        if (r == 0 && el < kMinSeconds) {  // the timed reps run long enough
            loops = (int)std::min(1000.0, std::ceil(kMinSeconds / std::max(el, 1e-4)));
            best = 1e30;
        }
        pthread_barrier_destroy(&start);
        where_host = (int)std::count(where.begin(), where.end(), KRK_PLACE_HOST);
        where_gpu = (int)std::count(where.begin(), where.end(), KRK_PLACE_GPU);
        ok = ok && std::all_of(good.begin(), good.end(), [](char c) { return c != 0; });
    }
    g_ok = g_ok && ok;
    printf("{\"case\": \"piece_streams\", \"placement\": \"%s\", \"streams\": %d, \"bytes_each\": %llu, \"write\": %llu, "
           "\"piece_length\": %llu, \"seconds\": %.4f, \"loops\": %d, \"GBps\": %.3f, \"placed_host\": %d, "
           "\"placed_gpu\": %d, \"sums_match\": %s}\n",
           pname(placement), n, (unsigned long long)L, (unsigned long long)w, (unsigned long long)P, best, loops,
           (double)n * L / best / 1e9, where_host, where_gpu, ok ? "true" : "false");
    fflush(stdout);
}

// Thread t's calls walk `span` bytes of its own region (call c at offset (c * size) % span).
void run_updates(int placement, int threads, uint64_t size, uint64_t total_each, int reps) {
    const uint64_t span = std::max<uint64_t>(size, std::min<uint64_t>(g_region, 64ull << 20) / size * size);
    const uint64_t per = std::max<uint64_t>(1, span / size);
    uint64_t calls = std::max<uint64_t>(1, total_each / size);
    std::vector<std::vector<uint32_t>> want(threads, std::vector<uint32_t>(per));
    for (int t = 0; t < threads; ++t)
        for (uint64_t c = 0; c < per; ++c)
            krk_host_crc32_update((uint32_t)t, g_buf.data() + (size_t)t * g_region + c * size, size, &want[t][c]);
    double best = 1e30;
    bool ok = true;
    for (int r = 0; r < reps; ++r) {
        pthread_barrier_t start;
        pthread_barrier_init(&start, nullptr, (unsigned)threads + 1);
        std::atomic<int> bad{0};
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                krk_set_device(0);
                pthread_barrier_wait(&start);
                for (uint64_t c = 0; c < calls; ++c) {
                    uint32_t out = 0;
                    const uint64_t k = c % per;
                    if (krk_crc32_update_on(placement, (uint32_t)t, g_buf.data() + (size_t)t * g_region + k * size, size,
                                            &out) != KRK_OK ||
                        out != want[t][k])
                        bad.fetch_add(1);
                }
            });
        const auto t0 = Clock::now();
        pthread_barrier_wait(&start);
        for (auto& t : th) t.join();
        const double el = secs(t0);
        best = std::min(best, el);
        if (r == 0 && el < kMinSeconds) {  // the timed reps run long enough
            calls = (uint64_t)std::ceil(calls * std::min(1000.0, kMinSeconds / std::max(el, 1e-4)));
            best = 1e30;
            ++reps;
        }
        pthread_barrier_destroy(&start);
        ok = ok && bad.load() == 0;
    }
    g_ok = g_ok && ok;
    printf("{\"case\": \"crc32_update\", \"placement\": \"%s\", \"threads\": %d, \"bytes_per_call\": %llu, "
           "\"calls_per_thread\": %llu, \"seconds\": %.4f, \"GBps\": %.3f, \"us_per_call\": %.2f, \"match\": %s}\n",
           pname(placement), threads, (unsigned long long)size, (unsigned long long)calls, best,
           (double)threads * calls * size / best / 1e9, best / calls * 1e6, ok ? "true" : "false");
    fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
    const double scale = argc > 1 ? atof(argv[1]) : 1.0;
    auto sz = [&](uint64_t b) { return std::max<uint64_t>(1 << 20, (uint64_t)(b * scale)) & ~uint64_t(4095); };
    if (krk_set_device(0) != KRK_OK) {
        fprintf(stderr, "no device: %s\n", krk_last_error());
        return 1;
    }
    const uint64_t L1 = sz(1ull << 30), LN = sz(128ull << 20), P = 4 << 20, W = 4 << 20;
    g_region = std::max<uint64_t>(sz(64ull << 20), 4u << 20);
    g_buf.resize(std::max({L1, 64 * LN, 64 * g_region, sz(256ull << 20)}));
    {  // splitmix64 bytes, filled on 16 threads
        std::vector<std::thread> th;
        const size_t words = g_buf.size() / 8, per = (words + 15) / 16;
        for (int t = 0; t < 16; ++t)
            th.emplace_back([&, t] {
                for (size_t k = t * per; k < std::min(words, (t + 1) * per); ++k) {
                    uint64_t z = (k + 1) * 0x9E3779B97F4A7C15ull;
                    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
                    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
                    z ^= z >> 31;
                    memcpy(&g_buf[8 * k], &z, 8);
                }
            });
        for (auto& t : th) t.join();
    }
    for (int p : {KRK_PLACE_HOST, KRK_PLACE_GPU, KRK_PLACE_AUTO}) run_streams(p, 1, L1, P, W, 3);
    for (int n : {4, 16, 64})
        for (int p : {KRK_PLACE_HOST, KRK_PLACE_GPU, KRK_PLACE_AUTO}) run_streams(p, n, LN, P, W, 2);
    for (uint64_t s : {64ull << 10, 256ull << 10, 1ull << 20, 4ull << 20, 16ull << 20, 64ull << 20, 256ull << 20})
        for (int p : {KRK_PLACE_HOST, KRK_PLACE_GPU}) run_updates(p, 1, std::min<uint64_t>(s, sz(s)), sz(512ull << 20), 2);
    for (int p : {KRK_PLACE_HOST, KRK_PLACE_GPU, KRK_PLACE_AUTO}) run_updates(p, 64, 4 << 20, sz(256ull << 20), 2);
    return g_ok ? 0 : 1;
}
