// synth_fill.hip -- device generator for the benchmark's synthetic blobs.
// Spec (shared with oracle/oracle.c orc_synth_fill): word j of blob i is
// mix64(seed_i + (j+1)*GAMMA) in little-endian byte order, seed_i =
// mix64((0x4B52414B454E ^ i) + GAMMA); variant 1 maps every byte b to
// "a-zA-Z0-9"[b % 62] (the randutil.Text alphabet, utils/randutil/randutil.go:37).
#include "kernels.hpp"
#include "device_util.hpp"

namespace krk {

constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ULL;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t alnum8(uint64_t w) {
    const char* A = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";
    uint64_t r = 0;
#pragma unroll
    for (int b = 0; b < 8; ++b) r |= (uint64_t)(uint8_t)A[((w >> (8 * b)) & 0xFF) % 62] << (8 * b);
    return r;
}

// Fast path: dst 16-byte aligned and offset 8-byte aligned -> one uint4 (2 words)
// per thread per iteration.
__global__ void synth_fill_words(uint4* dst, uint64_t seed, uint64_t word0, uint64_t npairs,
                                 int variant) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += stride) {
        const uint64_t j = word0 + 2 * i;
        uint64_t a = mix64(seed + (j + 1) * kGamma), b = mix64(seed + (j + 2) * kGamma);
        if (variant) { a = alnum8(a); b = alnum8(b); }
        dst[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    }
}

__global__ void synth_fill_bytes(uint8_t* dst, uint64_t seed, uint64_t offset, uint64_t n, int variant) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t pos = offset + i;
        uint64_t w = mix64(seed + ((pos >> 3) + 1) * kGamma);
        if (variant) w = alnum8(w);
        dst[i] = (uint8_t)(w >> (8 * (pos & 7)));
    }
}

// Many chunks in one launch (window generation for chunked batches): a fixed
// number of workgroups per chunk, each striding over its share of the chunk's
// 16-byte pairs (dst 16-aligned and offset 8-aligned) or bytes otherwise.
constexpr uint32_t kSynthBlocksPerChunk = 16;

__global__ void __launch_bounds__(256) synth_fill_chunks(const SynthChunk* __restrict__ chunks, uint32_t n_chunks,
                                                         int variant) {
    const uint32_t c = blockIdx.x / kSynthBlocksPerChunk, part = blockIdx.x % kSynthBlocksPerChunk;
    if (c >= n_chunks) return;
    const SynthChunk k = chunks[c];
    const uint64_t stride = (uint64_t)kSynthBlocksPerChunk * blockDim.x;
    const uint64_t t0 = (uint64_t)part * blockDim.x + threadIdx.x;
    uint64_t head = 0;
    if ((k.offset & 7) == 0 && (reinterpret_cast<uintptr_t>(k.dst) & 15) == 0) {
        const uint64_t npairs = k.n / 16, word0 = k.offset >> 3;
        uint4* d = reinterpret_cast<uint4*>(k.dst);
        for (uint64_t i = t0; i < npairs; i += stride) {
            const uint64_t j = word0 + 2 * i;
            uint64_t a = mix64(k.seed + (j + 1) * kGamma), b = mix64(k.seed + (j + 2) * kGamma);
            if (variant) { a = alnum8(a); b = alnum8(b); }
            d[i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
        }
        head = npairs * 16;
    }
    for (uint64_t i = head + t0; i < k.n; i += stride) {
        const uint64_t pos = k.offset + i;
        uint64_t w = mix64(k.seed + ((pos >> 3) + 1) * kGamma);
        if (variant) w = alnum8(w);
        k.dst[i] = (uint8_t)(w >> (8 * (pos & 7)));
    }
}

hipError_t launch_synth_fill_chunks(const SynthChunk* chunks, uint32_t n_chunks, int variant, hipStream_t s) {
    if (!n_chunks) return hipSuccess;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(synth_fill_chunks, dim3(n_chunks * kSynthBlocksPerChunk), dim3(256), 0, s, chunks, n_chunks,
                       variant);
    return hipGetLastError();
}

hipError_t launch_synth_fill(uint8_t* dst, uint64_t seed, uint64_t offset, uint64_t n, int variant,
                             hipStream_t s) {
    if (!n) return hipSuccess;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    uint64_t head = 0;
    if ((offset & 7) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        const uint64_t npairs = n / 16;
        if (npairs) {
            const uint64_t blocks = (npairs + 255) / 256;
            hipLaunchKernelGGL(synth_fill_words, dim3((uint32_t)(blocks < 8192 ? blocks : 8192)), dim3(256),
                               0, s, reinterpret_cast<uint4*>(dst), seed, offset >> 3, npairs, variant);
        }
        head = npairs * 16;
    }
    if (head < n) {
        const uint64_t rest = n - head;
        const uint64_t blocks = (rest + 255) / 256;
        hipLaunchKernelGGL(synth_fill_bytes, dim3((uint32_t)(blocks < 8192 ? blocks : 8192)), dim3(256), 0, s,
                           dst + head, seed, offset + head, rest, variant);
    }
    return hipGetLastError();
}

// Shader clock probe (measurement support): one wave spins on a dependent VALU chain
// and stamps s_memtime (shader cycles) and s_memrealtime (constant 100 MHz) around it;
// clock = d(memtime) / d(memrealtime) x 100 MHz (MI355X_MICROARCH.md, DVFS item 6).
// Launched beside a running kernel it reads the clock the chip holds under that load.
__global__ void __launch_bounds__(64) clock_probe_kernel(uint32_t spins, uint32_t seed, uint64_t* out) {
    uint32_t x = seed + threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    for (uint32_t i = 0; i < spins; ++i) x = x * 1664525u + 1013904223u;
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r1 - r0;
        out[2] = x;
    }
}

hipError_t launch_clock_probe(uint32_t spins, uint64_t* out, hipStream_t s) {
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, s, spins, 12345u, out);
    return hipGetLastError();
}

}  // namespace krk
