// crc_math.hpp -- GF(2) arithmetic for CRC-32/IEEE (reflected 0xEDB88320), shared by
// the host item builder and the device kernels.
//
// Notation: raw(c, M) is the CRC register after feeding M into register c with no
// pre/post conditioning.  It is linear:  raw(c, A||B) = shift(raw(c, A), |B|) ^ raw(0, B),
// where shift(c, n) = c * x^(8n) mod P.  The IEEE CRC that core.PieceHash() returns
// (core/piece_hash.go:22-24) is  crc(M) = raw(0, M) ^ shift(~0, |M|) ^ ~0.
// Polynomials are held bit-reflected: bit 31 is the x^0 coefficient.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define KRK_HD __host__ __device__ __forceinline__
#else
#define KRK_HD inline
#endif

namespace krk {

constexpr uint32_t kCrcPoly = 0xEDB88320u;
constexpr uint32_t kOne = 0x80000000u;  // the polynomial 1

// a * b mod P (branch-free, fixed 32 iterations: uniform cost on the GPU).
KRK_HD uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 31; i >= 0; --i) {
        p ^= b & (0u - ((a >> i) & 1u));
        b = (b >> 1) ^ (kCrcPoly & (0u - (b & 1u)));
    }
    return p;
}

// x^(8 * 2^k) mod P for k = 0..63.
struct X8Pow {
    uint32_t v[64];
};

inline X8Pow make_x8pow() {
    X8Pow t;
    uint32_t p = kOne >> 8;  // x^8
    for (int k = 0; k < 64; ++k) {
        t.v[k] = p;
        p = gf2_mulmod(p, p);
    }
    return t;
}

// x^(8n) mod P using a power table (host or device).
KRK_HD uint32_t x8n(uint64_t n, const uint32_t* x8pow) {
    uint32_t p = kOne;
    for (int k = 0; n; ++k, n >>= 1)
        if (n & 1) p = gf2_mulmod(p, x8pow[k]);
    return p;
}

// Byte table T0 and its slicing extensions: T_k[b] = raw(0, b || k zero bytes).
inline void make_slice_tables(uint32_t* t /* 4*256 */) {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kCrcPoly : (c >> 1);
        t[i] = c;
    }
    for (int k = 1; k < 4; ++k)
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = t[(k - 1) * 256 + i];
            t[k * 256 + i] = (c >> 8) ^ t[c & 0xFF];
        }
}

// Shift tables for a fixed distance: G_k[b] = shift(b << 8k, n), so
// shift(c, n) = G0[c&255] ^ G1[(c>>8)&255] ^ G2[(c>>16)&255] ^ G3[c>>24].
inline void make_shift_tables(uint32_t* g /* 4*256 */, uint32_t xn /* x^(8n) */) {
    for (int k = 0; k < 4; ++k)
        for (uint32_t i = 0; i < 256; ++i) g[k * 256 + i] = gf2_mulmod(i << (8 * k), xn);
}

}  // namespace krk
