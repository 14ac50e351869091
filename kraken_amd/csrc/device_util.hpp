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

}  // namespace krk
