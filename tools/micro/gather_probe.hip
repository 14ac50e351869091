// gather_probe.hip -- VERDICT r04 item 3: can host-resident batches go to HBM with ONE
// host-DRAM touch per byte (today: pageable -> pinned staging memcpy = read + write, then the
// DMA read)?  Measures, on a pageable source of G GiB laid out as 100 MiB "blobs":
//   register    hipHostRegister of every blob (and hipHostUnregister): GB/s and CPU s/GB
//   dma_blob    hipMemcpyAsync per blob-window chunk from the registered blobs (C2 window:
//               1,000 chunks of 512 KiB)
//   gather      one kernel per window: each workgroup copies chunks from the registered
//               (mapped) host pages into the device window over PCIe; grid sweep, chunk
//               sizes of the C2 (512 KiB) and C3 (~37 KiB) windows
//   staged      the current path: 16 threads memcpy pageable -> pinned window, DMA window
//   pinned_dma  one hipMemcpyAsync of a hipHostMalloc window (the link's rate)
// Every gathered window is checked against the source (sampled words).
//
//   gather_probe [GiB=8] [threads=16]           one JSON line per measurement
#include <hip/hip_runtime.h>
#include <sys/resource.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static double cpu_s() {
    rusage u{};
    getrusage(RUSAGE_SELF, &u);
    return u.ru_utime.tv_sec + u.ru_stime.tv_sec + 1e-6 * (u.ru_utime.tv_usec + u.ru_stime.tv_usec);
}

struct Chunk {
    const uint8_t* src;  // device-visible address of the registered host bytes (16-B aligned here)
    uint64_t dst_off;    // offset in the device window (16-B aligned)
    uint64_t n;          // bytes (multiple of 16 here)
};

// One workgroup walks chunks c = blockIdx.x, blockIdx.x + gridDim.x, ...; its 256 threads
// copy 16 B each per step, UNROLL steps in flight.
template <int UNROLL>
__global__ void __launch_bounds__(256) gather(const Chunk* __restrict__ ch, uint32_t nch, uint8_t* __restrict__ win) {
    for (uint32_t c = blockIdx.x; c < nch; c += gridDim.x) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u* s = reinterpret_cast<const v4u*>(ch[c].src);
        v4u* d = reinterpret_cast<v4u*>(win + ch[c].dst_off);
        const uint64_t words = ch[c].n / 16;
        for (uint64_t base = 0; base < words; base += 256 * UNROLL) {
            v4u v[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const uint64_t i = base + u * 256 + threadIdx.x;
                if (i < words) v[u] = __builtin_nontemporal_load(s + i);
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const uint64_t i = base + u * 256 + threadIdx.x;
                if (i < words) d[i] = v[u];
            }
        }
    }
}

int main(int argc, char** argv) {
    const size_t G = (size_t)(argc > 1 ? atoi(argv[1]) : 8) << 30;
    const int T = argc > 2 ? atoi(argv[2]) : 16;
    const size_t B = size_t(100) << 20;  // blob
    const size_t nb = G / B;
    const size_t W = size_t(512) << 20;  // window
    std::vector<uint8_t*> blob(nb);
    for (size_t i = 0; i < nb; ++i) {
        blob[i] = (uint8_t*)aligned_alloc(4096, B);
        uint64_t* p = (uint64_t*)blob[i];
        for (size_t k = 0; k < B / 8; ++k) p[k] = (i << 40) ^ (k * 0x9E3779B97F4A7C15ull);
    }
    uint8_t* dwin = nullptr;
    CK(hipMalloc(&dwin, W));
    uint8_t* pin = nullptr;
    CK(hipHostMalloc((void**)&pin, W, hipHostMallocDefault));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    Chunk* dch = nullptr;
    CK(hipMalloc(&dch, sizeof(Chunk) * 65536));

    // ---- register / unregister
    double c0 = cpu_s(), t0 = now();
    for (size_t i = 0; i < nb; ++i) CK(hipHostRegister(blob[i], B, hipHostRegisterMapped));
    double t1 = now(), c1 = cpu_s();
    std::vector<const uint8_t*> dptr(nb);
    for (size_t i = 0; i < nb; ++i) {
        void* d = nullptr;
        CK(hipHostGetDevicePointer(&d, blob[i], 0));
        dptr[i] = (const uint8_t*)d;
    }
    printf("{\"what\": \"register\", \"GiB\": %.1f, \"blob_MiB\": 100, \"GBps\": %.2f, \"cpu_s_per_GB\": %.4f, "
           "\"dev_ptr_equals_host\": %s}\n",
           G / 1073741824.0, nb * B / (t1 - t0) / 1e9, (c1 - c0) / (nb * B / 1e9), dptr[0] == blob[0] ? "true" : "false");
    fflush(stdout);

    auto check = [&](const std::vector<Chunk>& hc, const char* what) {
        std::vector<uint8_t> h(W);
        CK(hipMemcpy(h.data(), dwin, W, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t k = 0; k < hc.size(); k += std::max<size_t>(1, hc.size() / 64)) {
            // host address of chunk k: find its blob
            const Chunk& c = hc[k];
            size_t bi = 0;
            while (bi < nb && !(c.src >= dptr[bi] && c.src < dptr[bi] + B)) ++bi;
            const uint8_t* hs = blob[bi] + (c.src - dptr[bi]);
            if (memcmp(h.data() + c.dst_off, hs, c.n) != 0) ++bad;
        }
        if (bad) printf("{\"what\": \"%s\", \"MISMATCH\": %zu}\n", what, bad);
        return bad == 0;
    };

    // window layouts: C2 (every blob live, W / blobs a chunk) and C3 (14,336 live, ~37 KiB)
    auto layout = [&](size_t per, size_t round) {
        std::vector<Chunk> hc;
        size_t off = 0;
        for (size_t k = 0; off + per <= W; ++k) {
            const size_t bi = k % nb, pos = ((k / nb) * per * 7 + round * per) % (B - per);
            hc.push_back({dptr[bi] + (pos & ~size_t(15)), off, per});
            off += per;
        }
        return hc;
    };
    const size_t per_c2 = (W / 1000) & ~size_t(63), per_c3 = (W / 14336) & ~size_t(63);

    // ---- DMA per chunk from the registered pages
    for (size_t per : {per_c2, per_c3}) {
        auto hc = layout(per, 0);
        const int reps = per == per_c2 ? 6 : 2;
        double a = now();
        for (int r = 0; r < reps; ++r)
            for (const Chunk& c : hc) CK(hipMemcpyAsync(dwin + c.dst_off, c.src, c.n, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        const double el = now() - a;
        printf("{\"what\": \"dma_registered_chunks\", \"chunk_KiB\": %zu, \"chunks\": %zu, \"GBps\": %.2f}\n", per >> 10,
               hc.size(), reps * hc.size() * per / el / 1e9);
        check(hc, "dma_registered_chunks");
        fflush(stdout);
    }

    // ---- gather kernel: grid sweep
    for (size_t per : {per_c2, per_c3})
        for (int grid : {256, 1024, 4096}) {
            auto hc = layout(per, 1);
            CK(hipMemcpy(dch, hc.data(), sizeof(Chunk) * hc.size(), hipMemcpyHostToDevice));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            gather<4><<<grid, 256, 0, s>>>(dch, (uint32_t)hc.size(), dwin);  // warm
            CK(hipStreamSynchronize(s));
            const int reps = 8;
            double c2 = cpu_s(), a = now();
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < reps; ++r) gather<4><<<grid, 256, 0, s>>>(dch, (uint32_t)hc.size(), dwin);
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double bytes = (double)reps * hc.size() * per;
            printf("{\"what\": \"gather_kernel\", \"chunk_KiB\": %zu, \"chunks\": %zu, \"grid\": %d, \"GBps\": %.2f, "
                   "\"wall_GBps\": %.2f, \"cpu_s_per_GB\": %.4f}\n",
                   per >> 10, hc.size(), grid, bytes / (ms * 1e-3) / 1e9, bytes / (now() - a) / 1e9,
                   (cpu_s() - c2) / (bytes / 1e9));
            check(hc, "gather_kernel");
            fflush(stdout);
            CK(hipEventDestroy(e0));
            CK(hipEventDestroy(e1));
        }

    // ---- pinned DMA (the link) and the staged path (T threads memcpy + DMA, no overlap)
    {
        const int reps = 8;
        double a = now();
        for (int r = 0; r < reps; ++r) CK(hipMemcpyAsync(dwin, pin, W, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        printf("{\"what\": \"pinned_dma\", \"GBps\": %.2f}\n", reps * (double)W / (now() - a) / 1e9);
        fflush(stdout);
    }
    for (int r = 0; r < nb; ++r) CK(hipHostUnregister(blob[r]));
    {
        auto hc = layout(per_c2, 2);
        // host addresses again (unregistered): dptr == blob on this platform when equal
        std::vector<std::pair<const uint8_t*, size_t>> src;
        for (const Chunk& c : hc) {
            size_t bi = 0;
            while (bi < nb && !(c.src >= dptr[bi] && c.src < dptr[bi] + B)) ++bi;
            src.push_back({blob[bi] + (c.src - dptr[bi]), c.dst_off});
        }
        const int reps = 4;
        double c3 = cpu_s(), a = now();
        for (int r = 0; r < reps; ++r) {
            std::vector<std::thread> th;
            for (int t = 0; t < T; ++t)
                th.emplace_back([&, t] {
                    for (size_t k = t; k < src.size(); k += T) memcpy(pin + src[k].second, src[k].first, per_c2);
                });
            for (auto& x : th) x.join();
        }
        const double tcopy = now() - a, ccopy = cpu_s() - c3;
        printf("{\"what\": \"staged_memcpy\", \"threads\": %d, \"GBps\": %.2f, \"cpu_s_per_GB\": %.4f}\n", T,
               reps * (double)W / tcopy / 1e9, ccopy / (reps * (double)W / 1e9));
        fflush(stdout);
    }
    {
        double c4 = cpu_s(), t4 = now();
        for (size_t i = 0; i < nb; ++i) CK(hipHostRegister(blob[i], B, hipHostRegisterMapped));
        const double reg = now() - t4;
        double t5 = now();
        for (size_t i = 0; i < nb; ++i) CK(hipHostUnregister(blob[i]));
        printf("{\"what\": \"register_again\", \"GBps\": %.2f, \"unregister_GBps\": %.2f, \"cpu_s_per_GB\": %.4f}\n",
               nb * B / reg / 1e9, nb * B / (now() - t5) / 1e9, (cpu_s() - c4) / (nb * B / 1e9));
    }
    return 0;
}
