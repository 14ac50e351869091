// host_meta.cpp -- host-side pieces of the metainfo path that stay on the CPU by
// design: bencode + SHA-1 InfoHash (O(pieces), core/metainfo.go:37-44,
// core/infohash.go:42-49) and the piece-length range table
// (lib/metainfogen/config.go:71-80).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "../../include/kraken_hip.h"

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
    static const bool portable = getenv("KRK_SHA1_PORTABLE") && atoi(getenv("KRK_SHA1_PORTABLE")) > 0;
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
}  // namespace krk

extern "C" {

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
