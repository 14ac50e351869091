// reg_probe.cpp -- hipHostRegister throughput of pageable memory: G GiB
// of touched pageable memory registered in segments of S MiB by T threads at once, with and
// without MADV_HUGEPAGE; register / unregister GB/s and CPU s/GB.
//   reg_probe [GiB=16]          one JSON line per (huge, seg, threads)
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/resource.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static double cpu_s() {
    rusage u{};
    getrusage(RUSAGE_SELF, &u);
    return u.ru_utime.tv_sec + u.ru_stime.tv_sec + 1e-6 * (u.ru_utime.tv_usec + u.ru_stime.tv_usec);
}

int main(int argc, char** argv) {
    const size_t G = (size_t)(argc > 1 ? atoi(argv[1]) : 16) << 30;
    hipSetDevice(0);
    hipFree(nullptr);
    // every row registers FRESH memory (first touch, then register): the driver keeps a
    // registration's pages after hipHostUnregister, so memory registered before registers
    // again almost for free (round-5 first probe: 39 GB/s fresh, > 1 TB/s the second time)
    for (int huge = 0; huge < 2; ++huge)
        for (size_t seg : {size_t(2) << 20, size_t(16) << 20, size_t(100) << 20})
            for (int T : {1, 2, 4, 8}) {
                uint8_t* p = (uint8_t*)mmap(nullptr, G, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
                if (p == MAP_FAILED) return 1;
                if (huge) madvise(p, G, MADV_HUGEPAGE);
                memset(p, 1, G);
                const size_t n = G / seg;
                std::atomic<size_t> next{0};
                std::atomic<int> bad{0};
                double c0 = cpu_s(), t0 = now();
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&] {
                        hipSetDevice(0);
                        for (size_t i; (i = next.fetch_add(1)) < n;)
                            if (hipHostRegister(p + i * seg, seg, hipHostRegisterMapped) != hipSuccess) bad++;
                    });
                for (auto& x : th) x.join();
                double t1 = now(), c1 = cpu_s();
                for (size_t i = 0; i < n; ++i) hipHostUnregister(p + i * seg);
                double t2 = now();
                // the same memory again: the cached case
                for (size_t i = 0; i < n; ++i) hipHostRegister(p + i * seg, seg, hipHostRegisterMapped);
                double t3 = now();
                for (size_t i = 0; i < n; ++i) hipHostUnregister(p + i * seg);
                printf("{\"huge\": %d, \"seg_MiB\": %zu, \"threads\": %d, \"register_GBps\": %.2f, \"cpu_s_per_GB\": %.4f, "
                       "\"us_per_call\": %.1f, \"unregister_GBps\": %.1f, \"again_GBps\": %.1f, \"failed\": %d}\n",
                       huge, seg >> 20, T, n * seg / (t1 - t0) / 1e9, (c1 - c0) / (n * seg / 1e9),
                       (t1 - t0) * 1e6 * T / n, n * seg / (t2 - t1) / 1e9, n * seg / (t3 - t2) / 1e9, bad.load());
                fflush(stdout);
                munmap(p, G);
            }
    return 0;
}
