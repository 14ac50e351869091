// sha256_multi.hip -- multi-buffer SHA-256 for gfx950 (core.Digester,
// core/digester.go:28-72 over crypto/sha256).
//
// SHA-256 is a sequential Merkle-Damgard chain per blob, so parallelism comes only
// from independent blobs: one lane = one stream, 64 streams per wave, one wave per
// workgroup so the waves spread over CUs/SIMDs.  Every lane loads its own next
// 64-byte blocks two blocks ahead (the stream bandwidth is tiny, latency is what
// needs hiding) and runs the 64 rounds fully unrolled in registers with
// v_alignbit rotates; no LDS, no MFMA (integer/bitwise work).
#include <stdlib.h>

#include "kernels.hpp"
#include "device_util.hpp"

namespace krk {

#define KRK_K256                                                                                 \
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,     \
        0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, \
        0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, \
        0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, \
        0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, \
        0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu, \
        0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u, \
        0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u, \
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, \
        0xc67178f2u

__device__ __forceinline__ uint32_t rotr(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// One compression of the 16 big-endian words w[] into state h[].
__device__ __forceinline__ void compress(uint32_t h[8], uint32_t w[16]) {
    constexpr uint32_t K[64] = {KRK_K256};
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        uint32_t wi;
        if (i < 16) {
            wi = w[i];
        } else {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
            w[i & 15] = wi;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t ch = (e & f) ^ (~e & g);  // matched to one v_bitop3 (0xCA)
        const uint32_t t1 = hh + S1 + ch + K[i] + wi;
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);  // majority, symmetric
        const uint32_t t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

__device__ __forceinline__ void load_block(uint64_t p, bool al16, uint32_t w[16], uint64_t lo = 0,
                                           uint64_t hi = ~0ull) {
    if (al16) {
        gptr<u32x4> q = as_global<u32x4>(p);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32x4 v = KRK_GUARD(p + 16 * k, 16, lo, hi, 2) ? q[k] : u32x4{0, 0, 0, 0};
            w[4 * k + 0] = bswap(v.x); w[4 * k + 1] = bswap(v.y);
            w[4 * k + 2] = bswap(v.z); w[4 * k + 3] = bswap(v.w);
        }
    } else {
        load_bytes64(p, 64, w, lo, hi);
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = bswap(w[k]);
    }
}

__global__ void __launch_bounds__(64)
sha256_multi_kernel(const ShaJob* __restrict__ jobs, uint32_t n_jobs, uint8_t* __restrict__ out_digest,
                    uint32_t* __restrict__ out_state) {
    const uint32_t j = blockIdx.x * 64 + threadIdx.x;
    if (j >= n_jobs) return;
    const ShaJob job = jobs[j];
    const uint64_t p = job.ptr;
    const bool al16 = (job.ptr & 15) == 0;
    const uint64_t lo = p & ~uint64_t(3), hi = (p + job.len + 3) & ~uint64_t(3);
    uint32_t h[8];
    if (job.flags & kShaFromState) {
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = out_state[8 * (uint64_t)job.out + k];
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) h[k] = job.h[k];
    }

    const uint64_t nblk = job.len / 64;
    uint32_t w0[16], w1[16], w2[16];
    if (nblk > 0) load_block(p, al16, w0, lo, hi);
    if (nblk > 1) load_block(p + 64, al16, w1, lo, hi);
    uint64_t i = 0;
    // Three register sets rotate so that two blocks are always in flight.
    for (; i + 3 <= nblk; i += 3) {
        load_block(p + (i + 2) * 64, al16, w2, lo, hi);
        compress(h, w0);
        if (i + 3 < nblk) load_block(p + (i + 3) * 64, al16, w0, lo, hi);
        compress(h, w1);
        if (i + 4 < nblk) load_block(p + (i + 4) * 64, al16, w1, lo, hi);
        compress(h, w2);
    }
    if (i < nblk) { compress(h, w0); ++i; }
    if (i < nblk) { compress(h, w1); ++i; }

    if (job.flags & kShaFinal) {
        // Tail (< 64 bytes) + 0x80 + zeros + 64-bit big-endian bit length.
        const uint32_t rem = (uint32_t)(job.len - nblk * 64);
        uint32_t w[16];
        load_bytes64(p + nblk * 64, rem, w, lo, hi);
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            w[k] = bswap(w[k]);
            if (k == (int)(rem >> 2)) w[k] |= 0x80u << (24 - 8 * (rem & 3));
        }
        const uint64_t bits = (job.prefix + job.len) * 8;
        if (rem >= 56) {
            compress(h, w);
#pragma unroll
            for (int k = 0; k < 16; ++k) w[k] = 0;
        }
        w[14] = (uint32_t)(bits >> 32);
        w[15] = (uint32_t)bits;
        compress(h, w);
        uint8_t* o = out_digest + 32 * (uint64_t)job.out;
        if ((reinterpret_cast<uintptr_t>(o) & 15) == 0) {
            reinterpret_cast<uint4*>(o)[0] = make_uint4(bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3]));
            reinterpret_cast<uint4*>(o)[1] = make_uint4(bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7]));
        } else {
            for (int k = 0; k < 32; ++k) o[k] = (uint8_t)(h[k >> 2] >> (24 - 8 * (k & 3)));
        }
    } else {
        uint32_t* o = out_state + 8 * (uint64_t)job.out;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = h[k];
    }
}

// ---------------------------------------------------------------------------
// Wave-specialised variant.  A workgroup = 2 waves over the same 64 streams:
// wave 0 (producer) loads each block, builds the padded tail blocks and expands
// the message schedule into KW[r] = W[r] + K[r] in an LDS ring; wave 1 (consumer)
// only runs the 64 rounds (no VMEM, no schedule: ~14 VALU ops per round).  The
// two waves sit on different SIMDs, so the consumer keeps its full issue rate.
// One s_barrier per block; the producer runs kDepth blocks ahead in a kSlots
// ring (kDepth <= kSlots - 1 keeps every slot's reuse behind its last read).
constexpr int kSlots = 4;
constexpr int kDepth = 3;
constexpr int kSlotWords = 64 * 64;  // 64 rounds x 64 lanes

// LDS image of one slot: [round/4][lane][4] words -> a lane's 4 consecutive KW
// are one conflict-free ds_read_b128 / ds_write_b128 across the wave.
__device__ __forceinline__ uint32_t kw_index(int slot, int quad, uint32_t lane) {
    return (uint32_t)slot * kSlotWords + ((uint32_t)quad * 64 + lane) * 4;
}

__device__ __forceinline__ uint32_t job_blocks(const ShaJob& job) {
    const uint32_t nblk = (uint32_t)(job.len / 64);
    if (!(job.flags & kShaFinal)) return nblk;
    return nblk + (((uint32_t)(job.len & 63) >= 56) ? 2u : 1u);
}

__device__ __forceinline__ void produce(const ShaJob& job, uint32_t b, uint32_t lane, uint32_t* lds) {
    constexpr uint32_t K[64] = {KRK_K256};
    const uint64_t p = job.ptr;
    const uint64_t lo = p & ~uint64_t(3), hi = (p + job.len + 3) & ~uint64_t(3);
    const uint32_t nblk = (uint32_t)(job.len / 64);
    uint32_t w[16];
    if (b < nblk) {
        load_block(p + (uint64_t)b * 64, (p & 15) == 0, w, lo, hi);
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) w[k] = 0;
        if (job.flags & kShaFinal) {
            const uint32_t rem = (uint32_t)(job.len & 63);
            const uint64_t bits = (job.prefix + job.len) * 8;
            if (b == nblk) {
                load_bytes64(p + (uint64_t)nblk * 64, rem, w, lo, hi);
#pragma unroll
                for (int k = 0; k < 16; ++k) {
                    w[k] = bswap(w[k]);
                    if (k == (int)(rem >> 2)) w[k] |= 0x80u << (24 - 8 * (rem & 3));
                }
            }
            if (b == job_blocks(job) - 1) {
                w[14] = (uint32_t)(bits >> 32);
                w[15] = (uint32_t)bits;
            }
        }
    }
    const int slot = (int)(b % kSlots);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        uint32_t kw[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int i = 4 * q + t;
            uint32_t wi;
            if (i < 16) {
                wi = w[i];
            } else {
                const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
                const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
                const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
                wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
                w[i & 15] = wi;
            }
            kw[t] = wi + K[i];
        }
        *reinterpret_cast<u32x4*>(lds + kw_index(slot, q, lane)) = u32x4{kw[0], kw[1], kw[2], kw[3]};
    }
}

__device__ __forceinline__ void rounds(uint32_t h[8], const uint32_t* lds, int slot, uint32_t lane) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const u32x4 kw = *reinterpret_cast<const u32x4*>(lds + kw_index(slot, q, lane));
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
            const uint32_t ch = (e & f) ^ (~e & g);
            const uint32_t t1 = hh + S1 + ch + kw[t];
            const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
            const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + S0 + mj;
        }
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

__global__ void __launch_bounds__(128)
sha256_ws_kernel(const ShaJob* __restrict__ jobs, uint32_t n_jobs, uint8_t* __restrict__ out_digest,
                 uint32_t* __restrict__ out_state) {
    extern __shared__ __attribute__((aligned(16))) uint32_t ring[];
    const uint32_t lane = threadIdx.x & 63;
    const bool producer = threadIdx.x < 64;
    const uint32_t j = blockIdx.x * 64 + lane;
    const bool live = j < n_jobs;
    ShaJob job{};
    if (live) job = jobs[j];
    const uint32_t mine = live ? job_blocks(job) : 0u;
    // wave-uniform block count (both waves see the same 64 jobs)
    uint32_t nb = mine;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nb = max(nb, (uint32_t)__shfl_xor((int)nb, off, 64));
    nb = __builtin_amdgcn_readfirstlane(nb);

    if (producer) {
        const uint32_t pre = nb < (uint32_t)kDepth ? nb : (uint32_t)kDepth;
        for (uint32_t b = 0; b < pre; ++b) produce(job, b, lane, ring);
        for (uint32_t i = 0; i < nb; ++i) {
            __syncthreads();
            if (i + kDepth < nb) produce(job, i + kDepth, lane, ring);
        }
    } else {
        uint32_t h[8];
        if (live && (job.flags & kShaFromState)) {
#pragma unroll
            for (int k = 0; k < 8; ++k) h[k] = out_state[8 * (uint64_t)job.out + k];
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) h[k] = job.h[k];
        }
        for (uint32_t i = 0; i < nb; ++i) {
            __syncthreads();
            uint32_t x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = h[k];
            rounds(x, ring, (int)(i % kSlots), lane);
            if (i < mine) {
#pragma unroll
                for (int k = 0; k < 8; ++k) h[k] = x[k];
            }
        }
        if (live) {
            if (job.flags & kShaFinal) {
                uint8_t* o = out_digest + 32 * (uint64_t)job.out;
                if ((reinterpret_cast<uintptr_t>(o) & 15) == 0) {
                    reinterpret_cast<uint4*>(o)[0] = make_uint4(bswap(h[0]), bswap(h[1]), bswap(h[2]), bswap(h[3]));
                    reinterpret_cast<uint4*>(o)[1] = make_uint4(bswap(h[4]), bswap(h[5]), bswap(h[6]), bswap(h[7]));
                } else {
                    for (int k = 0; k < 32; ++k) o[k] = (uint8_t)(h[k >> 2] >> (24 - 8 * (k & 3)));
                }
            } else {
                uint32_t* o = out_state + 8 * (uint64_t)job.out;
#pragma unroll
                for (int k = 0; k < 8; ++k) o[k] = h[k];
            }
        }
    }
}

static int sha_variant() {
    static int v = [] {
        const char* e = getenv("KRK_SHA_VARIANT");
        return e ? atoi(e) : 1;
    }();
    return v;
}

hipError_t launch_sha256(const ShaJob* jobs, uint32_t n_jobs, uint8_t* out_digest,
                         uint32_t* out_state, hipStream_t s) {
    if (!n_jobs) return hipSuccess;
    const uint32_t grid = (n_jobs + 63) / 64;
    if (sha_variant() == 1) {
        constexpr size_t lds = size_t(kSlots) * kSlotWords * 4;  // 64 KiB
        hipFuncSetAttribute(reinterpret_cast<const void*>(&sha256_ws_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(sha256_ws_kernel, dim3(grid), dim3(128), lds, s, jobs, n_jobs, out_digest, out_state);
    } else {
        hipLaunchKernelGGL(sha256_multi_kernel, dim3(grid), dim3(64), 0, s, jobs, n_jobs, out_digest, out_state);
    }
    return hipGetLastError();
}

}  // namespace krk
