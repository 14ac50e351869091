// glds_probe.hip -- read-only HBM streaming ceilings for the piece-CRC kernel's loads:
// global_load_dwordx4 into VGPRs (the CRC kernel's path) against global_load_lds_dwordx4
// (LDS-DMA, no VGPR destination), default and nontemporal policy, at several waves per
// CU.  Each wave streams contiguous 4 KiB steps (64 lanes x 4 x 16 B); nothing is
// computed.  Development tool; build: hipcc -O3 --offload-arch=gfx950 glds_probe.hip -o glds_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <chrono>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

// VGPR loads, the CRC kernel's strided lane layout: lane l reads bytes 64 l + 16 k of a step.
template <int WPB>
__global__ void __launch_bounds__(64 * WPB) vgpr_stream(const uint8_t* __restrict__ p, size_t steps, uint32_t* sink) {
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * WPB + threadIdx.x / 64, nw = (size_t)gridDim.x * WPB;
    u4 acc = {0, 0, 0, 0};
    for (size_t s = wave; s < steps; s += nw) {
        const u4* q = reinterpret_cast<const u4*>(p + s * 4096 + 64 * lane);
        u4 a = q[0], b = q[1], c = q[2], d = q[3];
        acc ^= a ^ b ^ c ^ d;
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

// LDS-DMA: each wave-instruction writes 1 KiB of LDS (lane-linear); 4 per 4 KiB step into
// a per-wave ring of RING steps; a counted vmcnt keeps RING - 1 steps in flight.
template <int WPB, int AUX, int RING>
__global__ void __launch_bounds__(64 * WPB) glds_stream(const uint8_t* __restrict__ p, size_t steps, uint32_t* sink) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x / 64;
    const size_t wave = (size_t)blockIdx.x * WPB + w, nw = (size_t)gridDim.x * WPB;
    uint32_t* ring = lds + w * RING * 1024;  // RING steps x 4 KiB
    uint32_t slot = 0;
    for (size_t s = wave; s < steps; s += nw) {
        const uint8_t* g = p + s * 4096 + 16 * lane;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            __builtin_amdgcn_global_load_lds((const void*)(g + 1024 * k),
                                             (__attribute__((address_space(3))) void*)(ring + slot * 1024 + 256 * k),
                                             16, 0, AUX);
        slot = slot + 1 == RING ? 0 : slot + 1;
        if constexpr (RING == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        if constexpr (RING == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        if constexpr (RING == 4) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lds[threadIdx.x] == 0x12345678u) sink[0] = 1;
}

template <class F>
static double time_gbps(F launch, size_t bytes) {
    launch();
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, 0));
    for (int r = 0; r < 3; ++r) launch();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return 3.0 * bytes / (ms / 1e3) / 1e9;
}

int main() {
    const size_t N = size_t(16) << 30, steps = N / 4096;
    uint8_t* p = nullptr;
    uint32_t* sink = nullptr;
    CK(hipMalloc((void**)&p, N));
    CK(hipMalloc((void**)&sink, 4));
    CK(hipMemset(p, 1, N));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int bpc : {1, 2, 4}) {
        printf("{\"what\": \"vgpr loads, 16 waves x %d WG/CU\", \"GBps\": %.1f}\n", bpc,
               time_gbps([&] { hipLaunchKernelGGL(vgpr_stream<16>, dim3(cus * bpc), dim3(1024), 0, 0, p, steps, sink); }, N));
    }
    const size_t l2 = size_t(16) * 2 * 4096, l3 = size_t(8) * 3 * 4096, l4 = size_t(8) * 4 * 4096;
    CK(hipFuncSetAttribute((const void*)glds_stream<16, 0, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l2));
    CK(hipFuncSetAttribute((const void*)glds_stream<16, 2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l2));
    CK(hipFuncSetAttribute((const void*)glds_stream<8, 0, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l3));
    CK(hipFuncSetAttribute((const void*)glds_stream<8, 2, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l3));
    CK(hipFuncSetAttribute((const void*)glds_stream<8, 0, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l4));
    CK(hipFuncSetAttribute((const void*)glds_stream<8, 2, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)l4));
    for (int rep = 0; rep < 2; ++rep) {
        printf("{\"what\": \"glds default, 16 waves/CU, 2 steps in ring\", \"GBps\": %.1f}\n",
               time_gbps([&] { hipLaunchKernelGGL((glds_stream<16, 0, 2>), dim3(cus), dim3(1024), l2, 0, p, steps, sink); }, N));
        printf("{\"what\": \"glds nt, 16 waves/CU, 2 steps in ring\", \"GBps\": %.1f}\n",
               time_gbps([&] { hipLaunchKernelGGL((glds_stream<16, 2, 2>), dim3(cus), dim3(1024), l2, 0, p, steps, sink); }, N));
        printf("{\"what\": \"glds default, 8 waves/CU, 3 steps in ring\", \"GBps\": %.1f}\n",
               time_gbps([&] { hipLaunchKernelGGL((glds_stream<8, 0, 3>), dim3(cus), dim3(512), l3, 0, p, steps, sink); }, N));
        printf("{\"what\": \"glds nt, 8 waves/CU, 3 steps in ring\", \"GBps\": %.1f}\n",
               time_gbps([&] { hipLaunchKernelGGL((glds_stream<8, 2, 3>), dim3(cus), dim3(512), l3, 0, p, steps, sink); }, N));
        printf("{\"what\": \"glds default, 8 waves/CU, 4 steps in ring\", \"GBps\": %.1f}\n",
               time_gbps([&] { hipLaunchKernelGGL((glds_stream<8, 0, 4>), dim3(cus), dim3(512), l4, 0, p, steps, sink); }, N));
        printf("{\"what\": \"glds nt, 8 waves/CU, 4 steps in ring\", \"GBps\": %.1f}\n",
               time_gbps([&] { hipLaunchKernelGGL((glds_stream<8, 2, 4>), dim3(cus), dim3(512), l4, 0, p, steps, sink); }, N));
        fflush(stdout);
    }
    return 0;
}
