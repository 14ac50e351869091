// host_meta.cpp -- host-side pieces of the metainfo path that stay on the CPU by
// design: bencode + SHA-1 InfoHash (O(pieces), core/metainfo.go:37-44,
// core/infohash.go:42-49) and the piece-length range table
// (lib/metainfogen/config.go:71-80).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "knobs.hpp"

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "../../include/kraken_hip_internal.h"

namespace krk {
void set_error(int code, const char* fmt, ...);

namespace {

// ------------------------------------------------------------------- SHA-1
// FIPS 180-4 SHA-1 over whole 64-byte blocks; the x86 SHA extensions when the CPU
// has them (sha1rnds4: four rounds per instruction), the portable compressor
// otherwise.  InfoHash is host work by design (O(pieces)).
static void sha1_blocks_portable(uint32_t h[5], const uint8_t* p, size_t nblocks) {
    auto rol = [](uint32_t x, int k) { return (x << k) | (x >> (32 - k)); };
    for (; nblocks; --nblocks, p += 64) {
        uint32_t w[80];
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 80; ++i) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
        for (int i = 0; i < 80; ++i) {
            uint32_t f, k;
            if (i < 20) { f = d ^ (b & (c ^ d)); k = 0x5A827999; }
            else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1; }
            else if (i < 60) { f = (b & c) | (d & (b | c)); k = 0x8F1BBCDC; }
            else { f = b ^ c ^ d; k = 0xCA62C1D6; }
            const uint32_t t = rol(a, 5) + f + e + k + w[i];
            e = d; d = c; c = rol(b, 30); b = a; a = t;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
    }
}

#if defined(__x86_64__)
// Quad-round q (rounds 4q..4q+3) of the SHA-NI schedule: message words rotate
// through M[0..3]; E alternates between the two E registers.
template <int Q>
__attribute__((target("sha,sse4.1"))) static inline void sha1_quad(__m128i& abcd, __m128i& e0, __m128i& e1,
                                                                    __m128i M[4]) {
    __m128i& ein = (Q & 1) ? e1 : e0;   // E feeding this quad's rounds
    __m128i& eout = (Q & 1) ? e0 : e1;  // receives ABCD for the next quad's E
    if (Q == 0) ein = _mm_add_epi32(ein, M[0]);
    else ein = _mm_sha1nexte_epu32(ein, M[Q & 3]);
    eout = abcd;
    if (Q >= 3 && Q <= 18) M[(Q + 1) & 3] = _mm_sha1msg2_epu32(M[(Q + 1) & 3], M[Q & 3]);
    abcd = _mm_sha1rnds4_epu32(abcd, ein, Q / 5);
    if (Q >= 1 && Q <= 16) M[(Q + 3) & 3] = _mm_sha1msg1_epu32(M[(Q + 3) & 3], M[Q & 3]);
    if (Q >= 2 && Q <= 17) M[(Q + 2) & 3] = _mm_xor_si128(M[(Q + 2) & 3], M[Q & 3]);
}

template <int... Q>
__attribute__((target("sha,sse4.1"))) static inline void sha1_quads(__m128i& abcd, __m128i& e0, __m128i& e1,
                                                                     __m128i M[4], const uint8_t* p,
                                                                     std::integer_sequence<int, Q...>) {
    const __m128i bswap = _mm_set_epi64x(0x0001020304050607ULL, 0x08090a0b0c0d0e0fULL);
    for (int k = 0; k < 4; ++k)
        M[k] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * k)), bswap);
    (sha1_quad<Q>(abcd, e0, e1, M), ...);
}

__attribute__((target("sha,sse4.1"))) static void sha1_blocks_ni(uint32_t h[5], const uint8_t* p,
                                                                  size_t nblocks) {
    __m128i abcd = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h)), 0x1B);
    __m128i e0 = _mm_set_epi32((int)h[4], 0, 0, 0), e1;
    __m128i M[4];
    for (; nblocks; --nblocks, p += 64) {
        const __m128i abcd_save = abcd, e0_save = e0;
        sha1_quads(abcd, e0, e1, M, p, std::make_integer_sequence<int, 20>{});
        e0 = _mm_sha1nexte_epu32(e0, e0_save);
        abcd = _mm_add_epi32(abcd, abcd_save);
    }
    _mm_storeu_si128(reinterpret_cast<__m128i*>(h), _mm_shuffle_epi32(abcd, 0x1B));
    h[4] = (uint32_t)_mm_extract_epi32(e0, 3);
}

static bool have_sha_ni() {
    static const bool ok = __builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1");
    return ok;
}
#endif

// KRK_SHA1_PORTABLE=1 forces the portable compressor (tests compare both).
static void sha1_blocks(uint32_t h[5], const uint8_t* p, size_t nblocks) {
#if defined(__x86_64__)
    static const bool portable = KRK_AB_ENV("KRK_SHA1_PORTABLE") && atoi(KRK_AB_ENV("KRK_SHA1_PORTABLE")) > 0;
    if (!portable && have_sha_ni()) return sha1_blocks_ni(h, p, nblocks);
#endif
    sha1_blocks_portable(h, p, nblocks);
}

// SHA-1 of a whole buffer.
static void sha1(const uint8_t* p, size_t n, uint8_t out[20]) {
    uint32_t h[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
    sha1_blocks(h, p, n / 64);
    uint8_t tail[128] = {};
    const size_t r = n % 64;
    memcpy(tail, p + n - r, r);
    tail[r] = 0x80;
    const size_t tl = r < 56 ? 64 : 128;
    const uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha1_blocks(h, tail, tl / 64);
    for (int i = 0; i < 5; ++i)
        for (int k = 0; k < 4; ++k) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
}

// ----------------------------------------------------------------- SHA-256
// Host SHA-256 (FIPS 180-4) for the Digester's host crossover: one SHA-NI core
// digests ~2 GB/s where one GPU stream (eight lanes) digests ~59 MB/s, so a process
// with few concurrent digesters is served faster on its own threads.
static const uint32_t kK256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static void sha256_blocks_portable(uint32_t h[8], const uint8_t* p, size_t nblocks) {
    auto ror = [](uint32_t x, int k) { return (x >> k) | (x << (32 - k)); };
    for (; nblocks; --nblocks, p += 64) {
        uint32_t w[64];
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
        for (int i = 16; i < 64; ++i) {
            const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
            const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
            w[i] = w[i - 16] + s0 + w[i - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; ++i) {
            const uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + kK256[i] + w[i];
            const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
}

#if defined(__x86_64__)
// Four rounds q (4q..4q+3) with the x86 SHA extensions.  Message words rotate
// through M[0..3]: sha256msg1 at q = 1..12 prepares the words of quad q + 3,
// sha256msg2 at q = 3..14 completes those of quad q + 1.
template <int Q>
__attribute__((target("sha,sse4.1"))) static inline void sha256_quad(__m128i& s0, __m128i& s1, __m128i M[4]) {
    __m128i msg = _mm_add_epi32(M[Q & 3], _mm_loadu_si128(reinterpret_cast<const __m128i*>(kK256 + 4 * Q)));
    s1 = _mm_sha256rnds2_epu32(s1, s0, msg);
    if (Q >= 3 && Q <= 14) {
        const __m128i t = _mm_alignr_epi8(M[Q & 3], M[(Q + 3) & 3], 4);
        M[(Q + 1) & 3] = _mm_sha256msg2_epu32(_mm_add_epi32(M[(Q + 1) & 3], t), M[Q & 3]);
    }
    msg = _mm_shuffle_epi32(msg, 0x0E);
    s0 = _mm_sha256rnds2_epu32(s0, s1, msg);
    if (Q >= 1 && Q <= 12) M[(Q + 3) & 3] = _mm_sha256msg1_epu32(M[(Q + 3) & 3], M[Q & 3]);
}

template <int... Q>
__attribute__((target("sha,sse4.1"))) static inline void sha256_quads(__m128i& s0, __m128i& s1, __m128i M[4],
                                                                       std::integer_sequence<int, Q...>) {
    (sha256_quad<Q>(s0, s1, M), ...);
}

__attribute__((target("sha,sse4.1"))) static void sha256_blocks_ni(uint32_t h[8], const uint8_t* p,
                                                                    size_t nblocks) {
    const __m128i bswap = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    // (a,b,c,d),(e,f,g,h) -> the instruction's (ABEF),(CDGH) operand order
    __m128i t = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h)), 0xB1);
    __m128i s1 = _mm_shuffle_epi32(_mm_loadu_si128(reinterpret_cast<const __m128i*>(h + 4)), 0x1B);
    __m128i s0 = _mm_alignr_epi8(t, s1, 8);
    s1 = _mm_blend_epi16(s1, t, 0xF0);
    __m128i M[4];
    for (; nblocks; --nblocks, p += 64) {
        const __m128i s0_save = s0, s1_save = s1;
        for (int k = 0; k < 4; ++k)
            M[k] = _mm_shuffle_epi8(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p + 16 * k)), bswap);
        sha256_quads(s0, s1, M, std::make_integer_sequence<int, 16>{});
        s0 = _mm_add_epi32(s0, s0_save);
        s1 = _mm_add_epi32(s1, s1_save);
    }
    t = _mm_shuffle_epi32(s0, 0x1B);
    s1 = _mm_shuffle_epi32(s1, 0xB1);
    s0 = _mm_blend_epi16(t, s1, 0xF0);
    s1 = _mm_alignr_epi8(s1, t, 8);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(h), s0);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(h + 4), s1);
}
#endif

// KRK_HOST_PORTABLE=1 forces the portable SHA-256 / CRC-32 routines (tests compare).
static bool host_portable() {
    static const bool p = KRK_AB_ENV("KRK_HOST_PORTABLE") && atoi(KRK_AB_ENV("KRK_HOST_PORTABLE")) > 0;
    return p;
}

// ----------------------------------------------------------------- CRC-32
// Host CRC-32/IEEE (crc32.Update semantics) for the PieceHash crossover (small
// writes never pay a PCIe round trip): slicing-by-8, and carry-less-multiply
// folding (4 x 128 bits per step, Barrett reduction) when the CPU has PCLMULQDQ.
static uint32_t g_crc_tab[8][256];
static void crc_tables_init() {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1)));
        g_crc_tab[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
        for (int t = 1; t < 8; ++t) g_crc_tab[t][i] = (g_crc_tab[t - 1][i] >> 8) ^ g_crc_tab[0][g_crc_tab[t - 1][i] & 0xFF];
}

// Raw register update (no pre/post inversion).
static uint32_t crc_raw_sliced(uint32_t c, const uint8_t* p, size_t n) {
    for (; n >= 8; n -= 8, p += 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = g_crc_tab[7][lo & 0xFF] ^ g_crc_tab[6][(lo >> 8) & 0xFF] ^ g_crc_tab[5][(lo >> 16) & 0xFF] ^
            g_crc_tab[4][lo >> 24] ^ g_crc_tab[3][hi & 0xFF] ^ g_crc_tab[2][(hi >> 8) & 0xFF] ^
            g_crc_tab[1][(hi >> 16) & 0xFF] ^ g_crc_tab[0][hi >> 24];
    }
    for (; n; --n, ++p) c = g_crc_tab[0][(c ^ *p) & 0xFF] ^ (c >> 8);
    return c;
}

#if defined(__x86_64__)
// Folding constants of the reflected polynomial (x^k mod P, bit-reflected):
// 4-way fold (x^(4*128+32), x^(4*128-32)), 1-way fold (x^(128+32), x^(128-32)),
// 64->32 (x^64), and the Barrett pair (P', mu).
__attribute__((target("pclmul,sse4.1"))) static inline __m128i fold(__m128i x, __m128i k, __m128i d) {
    return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), d);
}

__attribute__((target("pclmul,sse4.1"))) static uint32_t crc_clmul_finish(__m128i x1, const __m128i* q, size_t n);

__attribute__((target("pclmul,sse4.1"))) static uint32_t crc_raw_clmul(uint32_t c, const uint8_t* p, size_t n) {
    if (n < 64) return crc_raw_sliced(c, p, n);
    const __m128i k1k2 = _mm_set_epi64x(0x01c6e41596LL, 0x0154442bd4LL);
    const __m128i k3k4 = _mm_set_epi64x(0x00ccaa009eLL, 0x01751997d0LL);
    const __m128i* q = reinterpret_cast<const __m128i*>(p);
    __m128i x1 = _mm_loadu_si128(q + 0), x2 = _mm_loadu_si128(q + 1);
    __m128i x3 = _mm_loadu_si128(q + 2), x4 = _mm_loadu_si128(q + 3);
    x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)c));
    q += 4;
    n -= 64;
    for (; n >= 64; n -= 64, q += 4) {
        x1 = fold(x1, k1k2, _mm_loadu_si128(q + 0));
        x2 = fold(x2, k1k2, _mm_loadu_si128(q + 1));
        x3 = fold(x3, k1k2, _mm_loadu_si128(q + 2));
        x4 = fold(x4, k1k2, _mm_loadu_si128(q + 3));
    }
    x1 = fold(x1, k3k4, x2);
    x1 = fold(x1, k3k4, x3);
    x1 = fold(x1, k3k4, x4);
    return crc_clmul_finish(x1, q, n);
}

// The 128-bit accumulator x1 (all bytes before q folded in) and the n bytes left at q:
// 16-byte folds, 128 -> 64 -> 32 bits (Barrett), the last < 16 bytes by table.
__attribute__((target("pclmul,sse4.1"))) static uint32_t crc_clmul_finish(__m128i x1, const __m128i* q, size_t n) {
    const __m128i k3k4 = _mm_set_epi64x(0x00ccaa009eLL, 0x01751997d0LL);
    const __m128i k5 = _mm_set_epi64x(0, 0x0163cd6124LL);
    const __m128i poly = _mm_set_epi64x(0x01f7011641LL, 0x01db710641LL);
    for (; n >= 16; n -= 16, ++q) x1 = fold(x1, k3k4, _mm_loadu_si128(q));
    // 128 -> 64 bits
    const __m128i mask32 = _mm_setr_epi32(~0, 0, ~0, 0);
    __m128i x2b = _mm_clmulepi64_si128(x1, k3k4, 0x10);
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x2b);
    x2b = _mm_srli_si128(x1, 4);
    x1 = _mm_and_si128(x1, mask32);
    x1 = _mm_xor_si128(_mm_clmulepi64_si128(x1, k5, 0x00), x2b);
    // Barrett reduction 64 -> 32
    x2b = _mm_and_si128(x1, mask32);
    x2b = _mm_clmulepi64_si128(x2b, poly, 0x10);
    x2b = _mm_and_si128(x2b, mask32);
    x2b = _mm_clmulepi64_si128(x2b, poly, 0x00);
    x1 = _mm_xor_si128(x1, x2b);
    const uint32_t c = (uint32_t)_mm_extract_epi32(x1, 1);
    return crc_raw_sliced(c, reinterpret_cast<const uint8_t*>(q), n);
}

// The same folding on AVX-512 VPCLMULQDQ (Zen 4/5, Ice Lake and later): four 512-bit
// accumulators = sixteen 128-bit lanes, 256 bytes an iteration, folded over 2,048 bits
// (x^(2048+32), x^(2048-32) mod P, bit-reflected); then 4 -> 1 register over 512 bits (the
// 4-way constants above) and the register's four lanes into one over 128 bits.  One core
// CRCs about twice as many bytes a second as the 128-bit loop, which is what bounds the
// host CRC threads (~17 GB/s each) below the memory's rate.
__attribute__((target("avx512f,avx512bw,vpclmulqdq,pclmul,sse4.1"))) static inline __m512i fold512(__m512i x,
                                                                                                     __m512i k,
                                                                                                     __m512i d) {
    return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0x00), _mm512_clmulepi64_epi128(x, k, 0x11), d,
                                     0x96);
}

__attribute__((target("avx512f,avx512bw,vpclmulqdq,pclmul,sse4.1"))) static uint32_t crc_raw_vclmul(uint32_t c,
                                                                                                     const uint8_t* p,
                                                                                                     size_t n) {
    if (n < 512) return crc_raw_clmul(c, p, n);
    const __m512i k2048 = _mm512_broadcast_i32x4(_mm_set_epi64x(0x01322d1430LL, 0x011542778aLL));
    const __m512i k512 = _mm512_broadcast_i32x4(_mm_set_epi64x(0x01c6e41596LL, 0x0154442bd4LL));
    __m512i x0 = _mm512_loadu_si512(p), x1 = _mm512_loadu_si512(p + 64);
    __m512i x2 = _mm512_loadu_si512(p + 128), x3 = _mm512_loadu_si512(p + 192);
    x0 = _mm512_xor_si512(x0, _mm512_castsi128_si512(_mm_cvtsi32_si128((int)c)));
    p += 256;
    n -= 256;
    for (; n >= 256; n -= 256, p += 256) {
        x0 = fold512(x0, k2048, _mm512_loadu_si512(p));
        x1 = fold512(x1, k2048, _mm512_loadu_si512(p + 64));
        x2 = fold512(x2, k2048, _mm512_loadu_si512(p + 128));
        x3 = fold512(x3, k2048, _mm512_loadu_si512(p + 192));
    }
    x0 = fold512(x0, k512, x1);
    x0 = fold512(x0, k512, x2);
    x0 = fold512(x0, k512, x3);
    for (; n >= 64; n -= 64, p += 64) x0 = fold512(x0, k512, _mm512_loadu_si512(p));
    const __m128i k3k4 = _mm_set_epi64x(0x00ccaa009eLL, 0x01751997d0LL);
    __m128i a = _mm512_extracti32x4_epi32(x0, 0);
    a = fold(a, k3k4, _mm512_extracti32x4_epi32(x0, 1));
    a = fold(a, k3k4, _mm512_extracti32x4_epi32(x0, 2));
    a = fold(a, k3k4, _mm512_extracti32x4_epi32(x0, 3));
    return crc_clmul_finish(a, reinterpret_cast<const __m128i*>(p), n);
}

static bool have_vclmul() {
    static const bool ok = [] {
        const char* v = KRK_AB_ENV("KRK_HOST_CRC_AVX512");  // 0: the 128-bit loop (A/B)
        if (v && v[0] == '0') return false;
        return __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
               __builtin_cpu_supports("vpclmulqdq") && __builtin_cpu_supports("pclmul");
    }();
    return ok;
}

static bool have_clmul() {
    static const bool ok = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    return ok;
}
#endif

// --------------------------------------------------------------- bencode
// Decimal digits of v at the END of buf[0..20); returns the first digit's index.
static int put_u64(char* buf, uint64_t v) {
    static const char d2[] =
        "0001020304050607080910111213141516171819202122232425262728293031323334353637383940414243444546474849"
        "5051525354555657585960616263646566676869707172737475767778798081828384858687888990919293949596979899";
    int i = 20;
    while (v >= 100) {
        const uint64_t q = v / 100;
        const int r = (int)(v - q * 100);
        buf[--i] = d2[2 * r + 1];
        buf[--i] = d2[2 * r];
        v = q;
    }
    if (v >= 10) {
        buf[--i] = d2[2 * v + 1];
        buf[--i] = d2[2 * v];
    } else {
        buf[--i] = (char)('0' + v);
    }
    return i;
}

static void put_i64(std::string& out, int64_t v) {
    char b[21];
    if (v < 0) {
        out.push_back('-');
        const int i = put_u64(b, (uint64_t)0 - (uint64_t)v);
        out.append(b + i, 20 - i);
    } else {
        const int i = put_u64(b, (uint64_t)v);
        out.append(b + i, 20 - i);
    }
}

// jackpal/bencode-go encoding of core.info (struct -> dict, keys in sorted order:
// Length, Name, PieceLength, PieceSums; []uint32 -> list of ints), as one buffer.
void bencode_info(std::string& out, int64_t piece_length, const uint32_t* sums, uint64_t n_sums,
                  const char* name, uint64_t name_len, int64_t length) {
    out.clear();
    out.reserve(96 + name_len + 12 * n_sums);
    out.append("d6:Lengthi");
    put_i64(out, length);
    out.append("e4:Name");
    put_i64(out, (int64_t)name_len);
    out.push_back(':');
    out.append(name, name_len);
    out.append("11:PieceLengthi");
    put_i64(out, piece_length);
    out.append("e9:PieceSumsl");
    const size_t at = out.size();
    out.resize(at + 12 * n_sums);  // "i" + <= 10 digits + "e"
    char* w = &out[at];
    char b[21];
    for (uint64_t k = 0; k < n_sums; ++k) {
        const int i = put_u64(b, sums[k]);
        *w++ = 'i';
        memcpy(w, b + i, 20 - i);
        w += 20 - i;
        *w++ = 'e';
    }
    out.resize((size_t)(w - out.data()));
    out.append("ee");
}

}  // namespace

void host_sha256_blocks(uint32_t h[8], const uint8_t* p, size_t nblocks) {
#if defined(__x86_64__)
    if (!host_portable() && have_sha_ni()) return sha256_blocks_ni(h, p, nblocks);
#endif
    sha256_blocks_portable(h, p, nblocks);
}

// Digest of (absorbed bytes folded into h) || tail[0..n) without touching h.
void host_sha256_final(const uint32_t h[8], uint64_t absorbed, const uint8_t* tail, size_t n, uint8_t out[32]) {
    uint32_t s[8];
    memcpy(s, h, sizeof s);
    host_sha256_blocks(s, tail, n / 64);
    const size_t r = n % 64;
    uint8_t b[128] = {};
    memcpy(b, tail + n - r, r);
    b[r] = 0x80;
    const size_t tl = r < 56 ? 64 : 128;
    const uint64_t bits = (absorbed + n) * 8;
    for (int i = 0; i < 8; ++i) b[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    host_sha256_blocks(s, b, tl / 64);
    for (int i = 0; i < 8; ++i)
        for (int k = 0; k < 4; ++k) out[4 * i + k] = (uint8_t)(s[i] >> (24 - 8 * k));
}

// crc32.Update(crc, IEEETable, p).
uint32_t host_crc32_update(uint32_t crc, const uint8_t* p, size_t n) {
    static std::once_flag once;
    std::call_once(once, crc_tables_init);
    uint32_t c = ~crc;
#if defined(__x86_64__)
    if (!host_portable() && have_vclmul()) return ~crc_raw_vclmul(c, p, n);
    if (!host_portable() && have_clmul()) return ~crc_raw_clmul(c, p, n);
#endif
    return ~crc_raw_sliced(c, p, n);
}

}  // namespace krk

extern "C" {

int krk_host_sha256(const uint8_t* data, uint64_t n, uint8_t out32[32]) {
    if (!out32 || (n && !data)) {
        krk::set_error(KRK_EINVAL, "host_sha256: null argument");
        return KRK_EINVAL;
    }
    static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                   0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    krk::host_sha256_final(iv, 0, data, n, out32);
    return KRK_OK;
}

int krk_host_crc32_update(uint32_t crc, const uint8_t* data, uint64_t n, uint32_t* out) {
    if (!out || (n && !data)) {
        krk::set_error(KRK_EINVAL, "host_crc32_update: null argument");
        return KRK_EINVAL;
    }
    *out = krk::host_crc32_update(crc, data, n);
    return KRK_OK;
}

int krk_info_hash(int64_t piece_length, const uint32_t* sums, uint64_t n_sums, const char* name,
                  uint64_t name_len, int64_t length, uint8_t out20[20]) {
    if (!out20 || (n_sums && !sums) || (name_len && !name)) {
        krk::set_error(KRK_EINVAL, "info_hash: null argument");
        return KRK_EINVAL;
    }
    std::string b;
    krk::bencode_info(b, piece_length, sums, n_sums, name, name_len, length);
    krk::sha1(reinterpret_cast<const uint8_t*>(b.data()), b.size(), out20);
    return KRK_OK;
}

int krk_info_hash_batch(const int64_t* piece_lengths, const uint32_t* sums, const uint64_t* sums_off,
                        const uint64_t* n_sums, const char* names, const uint64_t* name_off,
                        const int64_t* lengths, uint64_t n, uint8_t* out20) {
    if (!n) return KRK_OK;
    if (!piece_lengths || !sums_off || !n_sums || !name_off || !lengths || !out20 || (name_off[n] && !names)) {
        krk::set_error(KRK_EINVAL, "info_hash_batch: null argument");
        return KRK_EINVAL;
    }
    for (uint64_t i = 0; i < n; ++i)
        if (n_sums[i] && !sums) {
            krk::set_error(KRK_EINVAL, "info_hash_batch: null sums");
            return KRK_EINVAL;
        }
    auto work = [&](uint64_t lo, uint64_t hi) {
        std::string b;
        for (uint64_t i = lo; i < hi; ++i) {
            krk::bencode_info(b, piece_lengths[i], n_sums[i] ? sums + sums_off[i] : nullptr, n_sums[i],
                              names ? names + name_off[i] : "", name_off[i + 1] - name_off[i], lengths[i]);
            krk::sha1(reinterpret_cast<const uint8_t*>(b.data()), b.size(), out20 + 20 * i);
        }
    };
    const unsigned hw = std::thread::hardware_concurrency();
    const uint64_t T = std::min<uint64_t>({n, 16, hw ? hw : 1});
    if (T <= 1 || n < 64) {
        work(0, n);
        return KRK_OK;
    }
    std::vector<std::thread> th;
    const uint64_t span = (n + T - 1) / T;
    for (uint64_t t = 1; t < T; ++t) th.emplace_back(work, t * span, std::min(n, (t + 1) * span));
    work(0, std::min(n, span));
    for (auto& x : th) x.join();
    return KRK_OK;
}

int krk_bencode_info(int64_t piece_length, const uint32_t* sums, uint64_t n_sums, const char* name,
                     uint64_t name_len, int64_t length, uint8_t* out, uint64_t cap, uint64_t* written) {
    std::string b;
    krk::bencode_info(b, piece_length, sums, n_sums, name, name_len, length);
    const uint64_t pos = b.size();
    if (out && pos <= cap) memcpy(out, b.data(), pos);
    if (written) *written = pos;
    if (out && pos > cap) {
        krk::set_error(KRK_ERANGE, "bencode: need %llu bytes, have %llu", (unsigned long long)pos,
                       (unsigned long long)cap);
        return KRK_ERANGE;
    }
    return KRK_OK;
}

int64_t krk_piece_length_for_size(const int64_t* thresholds, const int64_t* lengths, uint32_t n,
                                  int64_t size) {
    if (!n) return 0;
    int64_t pl = lengths[0];
    for (uint32_t i = 0; i < n; ++i) {
        if (size < thresholds[i]) break;
        pl = lengths[i];
    }
    return pl;
}

}  // extern "C"
