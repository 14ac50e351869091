// h2d_probe.cpp -- host-side transfer rates that bound the end-to-end path
// (krk_metainfo_digest_host): pageable->pinned memcpy with T threads, hipHostRegister
// of pageable memory, pinned->device DMA in large and in small (per-blob chunk) copies.
// Development tool; build: hipcc -O2 --offload-arch=gfx950 h2d_probe.cpp -o h2d_probe -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

int main() {
    const size_t N = size_t(8) << 30;   // 8 GiB pageable source
    const size_t W = size_t(256) << 20; // one window
    uint8_t* src = (uint8_t*)aligned_alloc(4096, N);
    for (size_t i = 0; i < N; i += 4096) src[i] = (uint8_t)i;  // fault in
    memset(src, 7, N);
    uint8_t *pin = nullptr, *dev = nullptr;
    CK(hipHostMalloc((void**)&pin, W, hipHostMallocDefault));
    CK(hipMalloc((void**)&dev, N));
    hipStream_t s;
    CK(hipStreamCreate(&s));

    for (int T : {1, 4, 8, 16, 32}) {
        double t0 = now();
        for (size_t off = 0; off < N; off += W) {
            std::vector<std::thread> th;
            const size_t span = W / T;
            for (int i = 0; i < T; ++i) th.emplace_back([&, i] { memcpy(pin + i * span, src + off + i * span, span); });
            for (auto& x : th) x.join();
        }
        printf("{\"what\": \"pageable->pinned memcpy\", \"threads\": %d, \"GBps\": %.2f}\n", T, N / (now() - t0) / 1e9);
        fflush(stdout);
    }
    {
        double t0 = now();
        for (size_t off = 0; off < N; off += W) CK(hipMemcpyAsync(dev + off, pin, W, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        printf("{\"what\": \"pinned->device 256MiB copies\", \"GBps\": %.2f}\n", N / (now() - t0) / 1e9);
    }
    for (size_t chunk : {size_t(64) << 10, size_t(256) << 10, size_t(1) << 20, size_t(4) << 20}) {
        double t0 = now();
        for (size_t off = 0; off < N; off += W)
            for (size_t q = 0; q < W; q += chunk) CK(hipMemcpyAsync(dev + off + q, pin + q, chunk, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        printf("{\"what\": \"pinned->device small copies\", \"chunk\": %zu, \"GBps\": %.2f}\n", chunk,
               N / (now() - t0) / 1e9);
        fflush(stdout);
    }
    {
        double t0 = now();
        CK(hipHostRegister(src, N, hipHostRegisterDefault));
        double t1 = now();
        CK(hipMemcpyAsync(dev, src, N, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        double t2 = now();
        CK(hipHostUnregister(src));
        double t3 = now();
        printf("{\"what\": \"hipHostRegister\", \"register_GBps\": %.2f, \"dma_GBps\": %.2f, \"unregister_GBps\": %.2f}\n",
               N / (t1 - t0) / 1e9, N / (t2 - t1) / 1e9, N / (t3 - t2) / 1e9);
    }
    {   // direct DMA from pageable memory (the runtime stages internally)
        double t0 = now();
        CK(hipMemcpyAsync(dev, src, N, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        printf("{\"what\": \"pageable->device hipMemcpy\", \"GBps\": %.2f}\n", N / (now() - t0) / 1e9);
    }
    return 0;
}
