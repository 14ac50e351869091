// host_mem_probe.cpp -- why host CRC threads read pinned receive buffers at half the rate
// of pageable ones (bench f1verify / c4 end_to_end, round 4), and what to allocate instead.
// For each kind of host buffer (GiB each):
//   hipHostMalloc                 (krk_host_alloc up to round 4)
//   malloc                        (pageable, no madvise)
//   mmap + MADV_HUGEPAGE          (pageable, transparent huge pages)
//   mmap + MADV_HUGEPAGE + hipHostRegister
//   hipHostMalloc NumaUser        (the calling thread's NUMA policy)
// it reports: 16 host threads' CRC-32 over the buffer (krk_host_crc32_update on one span a
// thread), the pinned H2D rate of one hipMemcpyAsync of the whole buffer (pinned kinds), the
// NUMA node of sampled pages and the share of the buffer in huge pages (AnonHugePages delta).
//
//   host_mem_probe [GiB] [threads]      one JSON line per kind
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kraken_hip_internal.h"

namespace {
double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

long anon_huge_kb() {
    std::ifstream f("/proc/self/smaps_rollup");
    std::string k;
    long v = 0;
    while (f >> k) {
        if (k == "AnonHugePages:") {
            f >> v;
            return v;
        }
    }
    return -1;
}

std::string nodes_of(uint8_t* p, size_t n) {
    constexpr int kSamples = 8;
    void* pages[kSamples];
    int status[kSamples];
    for (int i = 0; i < kSamples; ++i) pages[i] = p + (n / kSamples) * i;
    if (syscall(SYS_move_pages, 0, kSamples, pages, nullptr, status, 0) != 0) return "\"?\"";
    std::string s = "[";
    for (int i = 0; i < kSamples; ++i) s += (i ? "," : "") + std::to_string(status[i]);
    return s + "]";
}

double crc_rate(const uint8_t* p, size_t n, int T) {
    double best = 0;
    for (int rep = 0; rep < 3; ++rep) {
        std::vector<std::thread> th;
        const size_t span = n / T;
        const double t0 = now();
        for (int t = 0; t < T; ++t)
            th.emplace_back([=] {
                uint32_t c = 0;
                krk_host_crc32_update(0, p + t * span, span, &c);
                if (c == 0x12345678) fprintf(stderr, ".");
            });
        for (auto& x : th) x.join();
        best = std::max(best, (double)span * T / (now() - t0) / 1e9);
    }
    return best;
}

double h2d_rate(const uint8_t* p, size_t n, void* dev, hipStream_t s) {
    double best = 0;
    for (int rep = 0; rep < 3; ++rep) {
        const double t0 = now();
        if (hipMemcpyAsync(dev, p, n, hipMemcpyHostToDevice, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return -1;
        best = std::max(best, (double)n / (now() - t0) / 1e9);
    }
    return best;
}
// The CPUs of NUMA node nd (empty when sysfs does not list it).
cpu_set_t node_set(int nd) {
    std::ifstream f("/sys/devices/system/node/node" + std::to_string(nd) + "/cpulist");
    std::string list;
    std::getline(f, list);
    cpu_set_t cs;
    CPU_ZERO(&cs);
    for (size_t q = 0; q < list.size();) {
        size_t e = list.find(',', q);
        if (e == std::string::npos) e = list.size();
        const std::string r = list.substr(q, e - q);
        const size_t d = r.find('-');
        const int a = atoi(r.c_str()), b = d == std::string::npos ? a : atoi(r.c_str() + d + 1);
        for (int c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(c, &cs);
        q = e + 1;
    }
    return cs;
}
}  // namespace

int main(int argc, char** argv) {
    const size_t n = (size_t)(argc > 1 ? atof(argv[1]) : 4.0) * (1ull << 30);
    const int T = argc > 2 ? atoi(argv[2]) : 16;
    if (argc > 3 && !strncmp(argv[3], "bind", 4)) {  // "bindN": every thread on node N's CPUs
        std::ifstream f("/sys/devices/system/node/node" + std::string(argv[3] + 4) + "/cpulist");
        std::string list;
        std::getline(f, list);
        cpu_set_t cs;
        CPU_ZERO(&cs);
        for (size_t q = 0; q < list.size();) {
            size_t e = list.find(',', q);
            if (e == std::string::npos) e = list.size();
            const std::string r = list.substr(q, e - q);
            const size_t d = r.find('-');
            const int a = atoi(r.c_str()), b = d == std::string::npos ? a : atoi(r.c_str() + d + 1);
            for (int c = a; c <= b; ++c) CPU_SET(c, &cs);
            q = e + 1;
        }
        sched_setaffinity(0, sizeof cs, &cs);
        printf("{\"bound_to\": \"%s\", \"cpus\": %d}\n", list.c_str(), CPU_COUNT(&cs));
    }
    if (krk_set_device(0) != KRK_OK) {
        fprintf(stderr, "no device: %s\n", krk_last_error());
        return 1;
    }
    void* dev = nullptr;
    hipStream_t s = nullptr;
    if (hipMalloc(&dev, n) != hipSuccess || hipStreamCreate(&s) != hipSuccess) return 1;
    {
        std::ifstream on("/sys/devices/system/node/online"), st("/proc/self/status");
        std::string online, line, mems;
        std::getline(on, online);
        while (std::getline(st, line))
            if (line.rfind("Mems_allowed_list:", 0) == 0) mems = line.substr(18);
        printf("{\"nodes_online\": \"%s\", \"mems_allowed\": \"%s\"}\n", online.c_str(), mems.c_str());
    }
    for (const char* kind : {"hipHostMalloc", "malloc", "malloc_1touch", "mmap_thp", "mmap_thp_registered",
                             "mmap_thp_interleave_registered", "hipHostMalloc_numauser"}) {
        const long huge0 = anon_huge_kb();
        uint8_t* p = nullptr;
        bool pinned = false, mapped = false;
        const double ta = now();
        if (!strcmp(kind, "hipHostMalloc")) {
            if (hipHostMalloc((void**)&p, n, hipHostMallocDefault) != hipSuccess) return 1;
            pinned = true;
        } else if (!strcmp(kind, "hipHostMalloc_numauser")) {
            if (hipHostMalloc((void**)&p, n, hipHostMallocNumaUser) != hipSuccess) return 1;
            pinned = true;
        } else if (!strncmp(kind, "malloc", 6)) {
            p = (uint8_t*)malloc(n);
        } else {
            p = (uint8_t*)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (p == MAP_FAILED) return 1;
            madvise(p, n, MADV_HUGEPAGE);
            mapped = true;
            if (!strcmp(kind, "mmap_thp_interleave_registered")) {
                unsigned long mask[2] = {3, 0};
                const long rc = syscall(SYS_mbind, p, n, 3 /* MPOL_INTERLEAVE */, mask, 65, 0);
                printf("{\"mbind_rc\": %ld, \"errno\": %d}\n", rc, rc ? errno : 0);
            }
        }
        // first touch on T threads (spans), as a filling receive path would (malloc_1touch: on
        // this thread alone, as the bench's numpy buffers are)
        if (!strcmp(kind, "malloc_1touch")) {
            for (size_t i = 0; i < n; i += 8) {
                uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
                memcpy(p + i, &z, 8);
            }
        } else {
            std::vector<std::thread> th;
            const size_t span = n / T;
            for (int t = 0; t < T; ++t)
                th.emplace_back([=] {
                    for (size_t i = t * span; i < (t + 1) * span; i += 8) {
                        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
                        memcpy(p + i, &z, 8);
                    }
                });
            for (auto& x : th) x.join();
        }
        if (!strncmp(kind, "mmap_thp_", 9)) {
            if (hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) return 1;
            pinned = true;
        }
        const double alloc_s = now() - ta;
        const long huge1 = anon_huge_kb();
        const double crc = crc_rate(p, n, T);
        const double h2d = pinned ? h2d_rate(p, n, dev, s) : -1;
        printf("{\"kind\": \"%s\", \"GiB\": %.2f, \"threads\": %d, \"alloc_touch_s\": %.3f, \"crc_GBps\": %.2f, "
               "\"h2d_GBps\": %.2f, \"nodes\": %s, \"huge_frac\": %.3f}\n",
               kind, n / double(1ull << 30), T, alloc_s, crc, h2d, nodes_of(p, n).c_str(),
               huge1 >= 0 ? (huge1 - huge0) * 1024.0 / n : -1.0);
        fflush(stdout);
        if (!strncmp(kind, "mmap_thp_", 9)) hipHostUnregister(p);
        if (!strcmp(kind, "hipHostMalloc") || !strcmp(kind, "hipHostMalloc_numauser")) hipHostFree(p);
        else if (mapped) munmap(p, n);
        else free(p);
    }
    // The library's own host CRC path (krk_piece_sums_host, C4 shape: one blob, 256 KiB
    // pieces) over a hipHostMalloc buffer filled by the CPU, the same filled by D2H DMA, and
    // a pageable buffer.
    {  // the CPUs this process may run on, and their NUMA nodes
        cpu_set_t cs;
        CPU_ZERO(&cs);
        sched_getaffinity(0, sizeof cs, &cs);
        int per_node[8] = {0};
        for (int c = 0; c < CPU_SETSIZE; ++c)
            if (CPU_ISSET(c, &cs))
                for (int nd = 0; nd < 8; ++nd)
                    if (access(("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/node" + std::to_string(nd)).c_str(),
                               F_OK) == 0)
                        ++per_node[nd];
        printf("{\"affinity_cpus\": %d, \"cpus_per_node\": [%d,%d,%d,%d]}\n", CPU_COUNT(&cs), per_node[0], per_node[1],
               per_node[2], per_node[3]);
    }
    for (const char* kind : {"lib_pinned_cpu_filled", "lib_pinned_spread_filled", "lib_pinned_dma_filled", "lib_pageable",
                             "lib_pageable_spread", "lib_thp_interleave_pageable", "lib_thp_local_registered",
                             "lib_thp_local_pageable", "lib_thp_nodespread_registered", "lib_thp_nodespread_pageable"}) {
        uint8_t* p = nullptr;
        const bool pinned = strncmp(kind, "lib_pinned", 10) == 0;
        const bool thp = strncmp(kind, "lib_thp", 7) == 0;
        if (pinned) {
            if (krk_host_alloc(n, (void**)&p) != KRK_OK) return 1;
        } else if (thp) {
            p = (uint8_t*)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            madvise(p, n, MADV_HUGEPAGE);
            if (strstr(kind, "interleave")) {
                unsigned long mask[2] = {3, 0};
                syscall(SYS_mbind, p, n, 3, mask, 65, 0);
            }
        } else {
            p = (uint8_t*)malloc(n);
        }
        if (!strcmp(kind, "lib_pinned_dma_filled")) {
            if (hipMemcpy(p, dev, n, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        } else if (strstr(kind, "nodespread")) {  // T spans first-touched by threads on alternating nodes
            std::vector<std::thread> th;
            const size_t span = n / T;
            for (int t = 0; t < T; ++t)
                th.emplace_back([=] {
                    cpu_set_t cs = node_set(t & 1);
                    if (CPU_COUNT(&cs)) sched_setaffinity(0, sizeof cs, &cs);
                    for (size_t i = t * span; i < (t + 1) * span; i += 8) {
                        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
                        memcpy(p + i, &z, 8);
                    }
                });
            for (auto& x : th) x.join();
        } else if (strstr(kind, "spread")) {  // written by T threads in spans (a receive path's threads)
            std::vector<std::thread> th;
            const size_t span = n / T;
            for (int t = 0; t < T; ++t)
                th.emplace_back([=] {
                    for (size_t i = t * span; i < (t + 1) * span; i += 8) {
                        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
                        memcpy(p + i, &z, 8);
                    }
                });
            for (auto& x : th) x.join();
        } else {
            for (size_t i = 0; i < n; i += 8) {
                uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
                memcpy(p + i, &z, 8);
            }
        }
        const bool reg = thp && strstr(kind, "_registered");
        if (reg && hipHostRegister(p, n, hipHostRegisterDefault) != hipSuccess) return 1;
        const uint64_t P = 256 << 10, np = n / P;
        std::vector<uint32_t> sums(np);
        krk_blob b{p, n, (int64_t)P, 0};
        // the library's NUMA-aware task hand-out with node visits (KRK_CRC_NUMA=2), the
        // hand-out alone (1) and the plain cursor (0, the default), interleaved so all see the same placement
        double best[3] = {0, 0, 0};  // KRK_CRC_NUMA 0 (default) / 1 / 2
        for (int rep = 0; rep < 9; ++rep) {
            setenv("KRK_CRC_NUMA", rep % 3 == 0 ? "2" : rep % 3 == 1 ? "1" : "0", 1);
            const double t0 = now();
            if (krk_piece_sums_host(&b, 1, sums.data()) != KRK_OK) {
                fprintf(stderr, "piece_sums_host: %s\n", krk_last_error());
                return 1;
            }
            double& x = best[rep % 3 == 0 ? 2 : rep % 3 == 1 ? 1 : 0];
            x = std::max(x, n / (now() - t0) / 1e9);
        }
        unsetenv("KRK_CRC_NUMA");
        uint64_t g = 0, h = 0;
        double f = 0;
        krk_crc_host_split(&g, &h, &f);
        printf("{\"kind\": \"%s\", \"GiB\": %.2f, \"lib_GBps_numa_visits\": %.2f, \"lib_GBps_numa_claims\": %.2f, \"lib_GBps\": %.2f, "
               "\"gpu_bytes\": %llu, \"host_bytes\": %llu, \"nodes\": %s}\n",
               kind, n / double(1ull << 30), best[2], best[1], best[0], (unsigned long long)g, (unsigned long long)h,
               nodes_of(p, n).c_str());
        fflush(stdout);
        if (pinned) krk_host_free(p);
        else if (thp) {
            if (reg) hipHostUnregister(p);
            munmap(p, n);
        } else free(p);
    }
    // The agent's verify shape: 2,048 received 4 MiB pieces in one krk_host_alloc block (and
    // in malloc memory), each its own blob, through krk_verify_pieces_host.
    for (const char* kind : {"verify_pinned", "verify_pageable"}) {
        uint8_t* p = nullptr;
        const bool pinned = !strcmp(kind, "verify_pinned");
        if (pinned) {
            if (krk_host_alloc(n, (void**)&p) != KRK_OK) return 1;
        } else {
            p = (uint8_t*)malloc(n);
        }
        for (size_t i = 0; i < n; i += 8) {
            uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
            memcpy(p + i, &z, 8);
        }
        const uint64_t P = 4 << 20, np = n / P;
        std::vector<const uint8_t*> ptr(np);
        std::vector<uint64_t> len(np, P);
        std::vector<uint32_t> exp(np, 0);
        std::vector<uint8_t> ok(np);
        for (uint64_t i = 0; i < np; ++i) ptr[i] = p + i * P;
        double best[3] = {0, 0, 0};  // KRK_CRC_NUMA 0 (default) / 1 / 2
        for (int rep = 0; rep < 9; ++rep) {
            setenv("KRK_CRC_NUMA", rep % 3 == 0 ? "2" : rep % 3 == 1 ? "1" : "0", 1);
            const double t0 = now();
            if (krk_verify_pieces_host(ptr.data(), len.data(), exp.data(), np, ok.data()) != KRK_OK) return 1;
            double& x = best[rep % 3 == 0 ? 2 : rep % 3 == 1 ? 1 : 0];
            x = std::max(x, n / (now() - t0) / 1e9);
        }
        unsetenv("KRK_CRC_NUMA");
        printf("{\"kind\": \"%s\", \"GiB\": %.2f, \"pieces\": %llu, \"lib_GBps_numa_visits\": %.2f, \"lib_GBps_numa_claims\": %.2f, "
               "\"lib_GBps\": %.2f}\n",
               kind, n / double(1ull << 30), (unsigned long long)np, best[2], best[1], best[0]);
        fflush(stdout);
        if (pinned) krk_host_free(p);
        else free(p);
    }
    hipFree(dev);
    return 0;
}
