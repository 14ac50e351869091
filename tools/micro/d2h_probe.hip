// d2h_probe.hip -- device -> pinned host transfer rates for the SHA-256 host offload
// (offload.cpp reads the offloaded blobs out of HBM in 8 MiB double-buffered chunks,
// one stream per host thread): one stream vs 16 streams of 8 MiB hipMemcpyAsync, large
// copies, and a copy kernel that stores straight into the mapped pinned buffer.
// Development tool; build: hipcc -O2 --offload-arch=gfx950 d2h_probe.hip -o d2h_probe -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <thread>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__global__ void __launch_bounds__(256) copy_to_host(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                    size_t n16) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

// One wave that spins `ticks` of the 100 MHz s_memrealtime clock: a long kernel
// occupying its stream's hardware queue while the copies run.
__global__ void spin(unsigned long long ticks, unsigned* sink) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned x = 0;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) x += 1;
    if (threadIdx.x == 0 && x == 12345u) sink[0] = x;
}

int main() {
    const size_t N = size_t(8) << 30;  // 8 GiB of device data
    const size_t C = size_t(8) << 20;  // chunk
    const int S = 16;
    uint8_t* dev = nullptr;
    CK(hipMalloc((void**)&dev, N));
    CK(hipMemset(dev, 7, N));
    std::vector<uint8_t*> pin(2 * S);
    for (auto& p : pin) CK(hipHostMalloc((void**)&p, C, hipHostMallocDefault));
    uint8_t* big = nullptr;
    CK(hipHostMalloc((void**)&big, size_t(256) << 20, hipHostMallocDefault));
    std::vector<hipStream_t> st(S);
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());

    unsigned* sink = nullptr;
    CK(hipMalloc((void**)&sink, 4));
    {  // a long kernel on its own stream (the SHA-256 launch of an offloaded batch), then
       // 16 threads' 8 MiB copies: when does each stream finish?
        hipStream_t busy;
        CK(hipStreamCreateWithFlags(&busy, hipStreamNonBlocking));
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, busy, 100000000ull, sink);  // 1 s
        double t0 = now();
        std::vector<double> done(S);
        std::vector<std::thread> th;
        const size_t span = size_t(256) << 20;
        for (int i = 0; i < S; ++i)
            th.emplace_back([&, i] {
                CK(hipSetDevice(0));
                for (size_t o = 0, k = 0; o < span; o += C, ++k) {
                    CK(hipMemcpyAsync(pin[2 * i + (k & 1)], dev + i * span + o, C, hipMemcpyDeviceToHost, st[i]));
                    if (k) CK(hipStreamSynchronize(st[i]));
                }
                CK(hipStreamSynchronize(st[i]));
                done[i] = now() - t0;
            });
        for (auto& x : th) x.join();
        double busy_end;
        CK(hipStreamSynchronize(busy));
        busy_end = now() - t0;
        printf("{\"what\": \"16 threads x 256 MiB D2H beside a long kernel\", \"stream_done_s\": [");
        for (int i = 0; i < S; ++i) printf("%s%.3f", i ? ", " : "", done[i]);
        printf("], \"busy_kernel_done_s\": %.3f}\n", busy_end);
        fflush(stdout);
    }
    {  // the same with the copies done by a copy kernel per chunk (stores into mapped pinned memory)
        hipStream_t busy;
        CK(hipStreamCreateWithFlags(&busy, hipStreamNonBlocking));
        hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, busy, 100000000ull, sink);
        double t0 = now();
        std::vector<double> done(S);
        std::vector<std::thread> th;
        const size_t span = size_t(256) << 20;
        for (int i = 0; i < S; ++i)
            th.emplace_back([&, i] {
                CK(hipSetDevice(0));
                uint4* hd[2];
                CK(hipHostGetDevicePointer((void**)&hd[0], pin[2 * i], 0));
                CK(hipHostGetDevicePointer((void**)&hd[1], pin[2 * i + 1], 0));
                for (size_t o = 0, k = 0; o < span; o += C, ++k) {
                    hipLaunchKernelGGL(copy_to_host, dim3(64), dim3(256), 0, st[i], (const uint4*)(dev + i * span + o),
                                       hd[k & 1], C / 16);
                    if (k) CK(hipStreamSynchronize(st[i]));
                }
                CK(hipStreamSynchronize(st[i]));
                done[i] = now() - t0;
            });
        for (auto& x : th) x.join();
        CK(hipStreamSynchronize(busy));
        const double busy_end = now() - t0;
        printf("{\"what\": \"16 threads x 256 MiB by copy kernels beside a long kernel\", \"stream_done_s\": [");
        for (int i = 0; i < S; ++i) printf("%s%.3f", i ? ", " : "", done[i]);
        printf("], \"busy_kernel_done_s\": %.3f}\n", busy_end);
        fflush(stdout);
    }
    for (int rep = 0; rep < 2; ++rep) {
        {  // one stream, 8 MiB chunks, two buffers
            double t0 = now();
            for (size_t o = 0, k = 0; o < N; o += C, ++k) CK(hipMemcpyAsync(pin[k & 1], dev + o, C, hipMemcpyDeviceToHost, st[0]));
            CK(hipStreamSynchronize(st[0]));
            printf("{\"what\": \"1 stream, 8 MiB D2H copies\", \"GBps\": %.2f}\n", N / (now() - t0) / 1e9);
        }
        {  // one stream, 256 MiB copies
            double t0 = now();
            for (size_t o = 0; o < N; o += size_t(256) << 20)
                CK(hipMemcpyAsync(big, dev + o, size_t(256) << 20, hipMemcpyDeviceToHost, st[0]));
            CK(hipStreamSynchronize(st[0]));
            printf("{\"what\": \"1 stream, 256 MiB D2H copies\", \"GBps\": %.2f}\n", N / (now() - t0) / 1e9);
        }
        for (int ns : {4, 16}) {  // ns streams (host threads), 8 MiB chunks each, sync per chunk
            double t0 = now();
            std::vector<std::thread> th;
            const size_t span = N / ns;
            for (int i = 0; i < ns; ++i)
                th.emplace_back([&, i] {
                    CK(hipSetDevice(0));
                    for (size_t o = 0, k = 0; o < span; o += C, ++k) {
                        CK(hipMemcpyAsync(pin[2 * i + (k & 1)], dev + i * span + o, C, hipMemcpyDeviceToHost, st[i]));
                        if (k) CK(hipStreamSynchronize(st[i]));
                    }
                    CK(hipStreamSynchronize(st[i]));
                });
            for (auto& x : th) x.join();
            printf("{\"what\": \"%d streams/threads, 8 MiB D2H copies\", \"GBps\": %.2f}\n", ns, N / (now() - t0) / 1e9);
        }
        {  // copy kernel storing into the mapped pinned buffer
            uint4* hd = nullptr;
            CK(hipHostGetDevicePointer((void**)&hd, big, 0));
            double t0 = now();
            for (size_t o = 0; o < N; o += size_t(256) << 20)
                hipLaunchKernelGGL(copy_to_host, dim3(1024), dim3(256), 0, st[0], (const uint4*)(dev + o), hd,
                                   (size_t(256) << 20) / 16);
            CK(hipStreamSynchronize(st[0]));
            printf("{\"what\": \"copy kernel into mapped pinned memory, 256 MiB a launch\", \"GBps\": %.2f}\n",
                   N / (now() - t0) / 1e9);
        }
        fflush(stdout);
    }
    return 0;
}
