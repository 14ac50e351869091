// device_util.hpp -- device-only helpers shared by the *.hip kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace krk {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Global-address-space views: loads through these compile to global_load_* (counted
// by vmcnt only) rather than flat_load_* (which also count in lgkmcnt, so every LDS
// wait would drain the prefetched loads as well).
template <class T>
using gptr = const __attribute__((address_space(1))) T*;
template <class T>
__device__ __forceinline__ gptr<T> as_global(uint64_t addr) {
    return (gptr<T>)(addr);
}
// a ^ b ^ c in one v_bitop3_b32 (truth table 0x96; symmetric, so input order is moot).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Bytes [a, a+n) (n <= 64, any alignment) as 16 little-endian words, zero padded
// past n.  Only dword-ALIGNED loads are issued, and only for dwords holding at
// least one requested byte, so nothing outside the run's pages is touched and no
// misaligned access is ever formed (the byte-wise form lets the compiler fuse
// odd-address 16-bit loads); the words are re-assembled with v_alignbit.
// KRK_BOUNDS_CHECK (debug builds only): every global access is checked against
// the caller's legitimate byte range [lo, hi); violations are printed and skipped.
#ifdef KRK_BOUNDS_CHECK
__device__ __forceinline__ bool krk_in_range(uint64_t addr, uint32_t size, uint64_t lo, uint64_t hi,
                                             int site) {
    if (addr >= lo && addr + size <= hi) return true;
    printf("KRK_BOUNDS site=%d addr=0x%llx size=%u lo=0x%llx hi=0x%llx block=%u thread=%u\n", site,
           (unsigned long long)addr, size, (unsigned long long)lo, (unsigned long long)hi, blockIdx.x,
           threadIdx.x);
    return false;
}
#define KRK_GUARD(addr, size, lo, hi, site) krk_in_range((addr), (size), (lo), (hi), (site))
#else
#define KRK_GUARD(addr, size, lo, hi, site) true
#endif

__device__ __forceinline__ void load_bytes64(uint64_t a, uint32_t n, uint32_t out[16], uint64_t lo = 0,
                                             uint64_t hi = ~0ull) {
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    const uint32_t nd = n ? (uint32_t)(((a + n - 1) >> 2) - (a >> 2) + 1) : 0;  // <= 17
    gptr<uint32_t> d = as_global<uint32_t>(a & ~uint64_t(3));
    uint32_t raw[17];
#pragma unroll
    for (int k = 0; k < 17; ++k)
        raw[k] = ((uint32_t)k < nd && KRK_GUARD((a & ~uint64_t(3)) + 4 * k, 4, lo, hi, 1)) ? d[k] : 0u;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        uint32_t w = __builtin_amdgcn_alignbit(raw[j + 1], raw[j], sh);
        const int keep = (int)n - 4 * j;  // bytes of word j inside the run
        if (keep <= 0) w = 0;
        else if (keep < 4) w &= (1u << (8 * keep)) - 1;
        out[j] = w;
    }
}

// Bytes [a, a+n) (n <= 16, any alignment) as 4 little-endian words, zero padded;
// the 16-byte form of load_bytes64 (at most 5 aligned dword loads).
__device__ __forceinline__ void load_bytes16(uint64_t a, uint32_t n, uint32_t out[4], uint64_t lo = 0,
                                             uint64_t hi = ~0ull) {
    const uint32_t sh = (uint32_t)(a & 3) * 8;
    const uint32_t nd = n ? (uint32_t)(((a + n - 1) >> 2) - (a >> 2) + 1) : 0;  // <= 5
    gptr<uint32_t> d = as_global<uint32_t>(a & ~uint64_t(3));
    uint32_t raw[5];
#pragma unroll
    for (int k = 0; k < 5; ++k)
        raw[k] = ((uint32_t)k < nd && KRK_GUARD((a & ~uint64_t(3)) + 4 * k, 4, lo, hi, 3)) ? d[k] : 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        uint32_t w = __builtin_amdgcn_alignbit(raw[j + 1], raw[j], sh);
        const int keep = (int)n - 4 * j;
        if (keep <= 0) w = 0;
        else if (keep < 4) w &= (1u << (8 * keep)) - 1;
        out[j] = w;
    }
}

}  // namespace krk
