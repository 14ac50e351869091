/*
 * oracle.c -- CPU restatement of the reference's blob-metainfo hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Each function cites the reference
 * file:line whose behaviour it restates.  The reference is Go; no Go toolchain
 * exists in this image, so this is a restatement, pinned by the reference's
 * own known-answer tests (tests/test_oracle_golden.py).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <fcntl.h>
#include <pthread.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>
#include <cpuid.h>

/* ======================================================================
 * CRC-32/IEEE -- core/piece_hash.go:22-24 returns crc32.NewIEEE(); Go's
 * hash/crc32 IEEE is the reflected polynomial 0xEDB88320 with
 * init = xorout = 0xFFFFFFFF (crc32.Update(crc, tab, p) = ^update(^crc, p)).
 * ====================================================================== */
static uint32_t crc_tab[256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;

static void crc_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
        crc_tab[i] = c;
    }
}

uint32_t orc_crc32_update(uint32_t crc, const uint8_t* p, uint64_t n) {
    pthread_once(&crc_once, crc_init);
    uint32_t c = ~crc;
    for (uint64_t i = 0; i < n; i++) c = crc_tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

int orc_have_clmul(void) {
    unsigned a, b, c, d;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & bit_PCLMUL) && (c & bit_SSE4_1);
}

/* Bit-reflected 4x128 folding with Barrett reduction: the same algorithm Go's
 * amd64 ieeeCLMUL uses for >=64-byte runs (folding constants for 0xEDB88320). */
__attribute__((target("pclmul,sse4.1")))
static uint32_t crc32_clmul_raw(uint32_t crc, const uint8_t* buf, uint64_t len) {
    __m128i x1 = _mm_loadu_si128((const __m128i*)(buf + 0));
    __m128i x2 = _mm_loadu_si128((const __m128i*)(buf + 16));
    __m128i x3 = _mm_loadu_si128((const __m128i*)(buf + 32));
    __m128i x4 = _mm_loadu_si128((const __m128i*)(buf + 48));
    x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)crc));
    buf += 64;
    len -= 64;
    __m128i k = _mm_set_epi64x(0x1c6e41596LL, 0x154442bd4LL);
    while (len >= 64) {
        __m128i t1 = _mm_clmulepi64_si128(x1, k, 0x00), t2 = _mm_clmulepi64_si128(x2, k, 0x00);
        __m128i t3 = _mm_clmulepi64_si128(x3, k, 0x00), t4 = _mm_clmulepi64_si128(x4, k, 0x00);
        x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, k, 0x11), t1),
                           _mm_loadu_si128((const __m128i*)(buf + 0)));
        x2 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x2, k, 0x11), t2),
                           _mm_loadu_si128((const __m128i*)(buf + 16)));
        x3 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x3, k, 0x11), t3),
                           _mm_loadu_si128((const __m128i*)(buf + 32)));
        x4 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x4, k, 0x11), t4),
                           _mm_loadu_si128((const __m128i*)(buf + 48)));
        buf += 64;
        len -= 64;
    }
    k = _mm_set_epi64x(0x0ccaa009eLL, 0x1751997d0LL);
    __m128i t = _mm_clmulepi64_si128(x1, k, 0x00);
    x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, k, 0x11), t), x2);
    t = _mm_clmulepi64_si128(x1, k, 0x00);
    x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, k, 0x11), t), x3);
    t = _mm_clmulepi64_si128(x1, k, 0x00);
    x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, k, 0x11), t), x4);
    while (len >= 16) {
        t = _mm_clmulepi64_si128(x1, k, 0x00);
        x1 = _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x1, k, 0x11), t),
                           _mm_loadu_si128((const __m128i*)buf));
        buf += 16;
        len -= 16;
    }
    /* 128 -> 64: fold the low qword by R4 */
    t = _mm_clmulepi64_si128(x1, k, 0x10);
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), t);
    /* 64 -> 32 */
    const __m128i mask32 = _mm_set_epi32(0, 0, 0, -1);
    k = _mm_set_epi64x(0, 0x163cd6124LL);
    x2 = _mm_srli_si128(x1, 4);
    x1 = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k, 0x00), x2);
    /* Barrett */
    k = _mm_set_epi64x(0x1F7011641LL, 0x1DB710641LL);
    x2 = x1;
    x1 = _mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k, 0x10);
    x1 = _mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k, 0x00);
    x1 = _mm_xor_si128(x1, x2);
    return (uint32_t)_mm_extract_epi32(x1, 1);
}

uint32_t orc_crc32_update_clmul(uint32_t crc, const uint8_t* p, uint64_t n) {
    pthread_once(&crc_once, crc_init);
    uint32_t c = ~crc;
    if (n >= 64 && orc_have_clmul()) {
        uint64_t run = n & ~(uint64_t)15;
        c = crc32_clmul_raw(c, p, run);
        p += run;
        n -= run;
    }
    for (uint64_t i = 0; i < n; i++) c = crc_tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

/* core.calcPieceSums -- core/metainfo.go:158-179.  Loop: fresh PieceHash per
 * piece, io.CopyN(h, blob, pieceLength); append Sum32 iff n > 0; stop when
 * n < pieceLength.  So L = 0 gives no sums and L % P == 0 gives no empty
 * trailing piece. */
int orc_calc_piece_sums(const uint8_t* blob, uint64_t len, int64_t piece_len,
                        uint32_t* sums, uint64_t* n_sums, uint64_t* length) {
    if (piece_len <= 0) return -1; /* "piece length must be positive" :159-161 */
    uint64_t P = (uint64_t)piece_len, off = 0, k = 0;
    for (;;) {
        uint64_t n = len - off < P ? len - off : P;
        if (n == 0) break;
        if (sums) sums[k] = orc_crc32_update(0, blob + off, n);
        k++;
        off += n;
        if (n < P) break;
    }
    if (n_sums) *n_sums = k;
    if (length) *length = off;
    return 0;
}

/* MetaInfo.GetPieceLength -- core/metainfo.go:109-118 */
int64_t orc_get_piece_length(int64_t length, int64_t piece_len, uint64_t n_pieces, int64_t i) {
    if (i < 0 || (uint64_t)i >= n_pieces) return 0;
    if ((uint64_t)i == n_pieces - 1) return length - piece_len * i;
    return piece_len;
}

/* ======================================================================
 * SHA-256 -- core/digester.go:34-72 wraps crypto.SHA256.New(); FIPS 180-4.
 * ====================================================================== */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
static const uint32_t H256[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};

#define ROR32(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t h[8], const uint8_t* p) {
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROR32(w[i - 15], 7) ^ ROR32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR32(w[i - 2], 17) ^ ROR32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
        uint32_t S1 = ROR32(e, 6) ^ ROR32(e, 11) ^ ROR32(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = hh + S1 + ch + K256[i] + w[i];
        uint32_t S0 = ROR32(a, 2) ^ ROR32(a, 13) ^ ROR32(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void orc_sha256_init(orc_sha256_ctx* c) {
    memcpy(c->h, H256, sizeof H256);
    c->nbytes = 0;
    c->nbuf = 0;
}

void orc_sha256_update(orc_sha256_ctx* c, const uint8_t* p, uint64_t n) {
    c->nbytes += n;
    if (c->nbuf) {
        uint32_t take = 64 - c->nbuf;
        if (take > n) take = (uint32_t)n;
        memcpy(c->buf + c->nbuf, p, take);
        c->nbuf += take;
        p += take;
        n -= take;
        if (c->nbuf == 64) { sha256_block(c->h, c->buf); c->nbuf = 0; }
    }
    while (n >= 64) { sha256_block(c->h, p); p += 64; n -= 64; }
    if (n) { memcpy(c->buf, p, n); c->nbuf = (uint32_t)n; }
}

void orc_sha256_sum(const orc_sha256_ctx* c0, uint8_t out[32]) {
    orc_sha256_ctx c = *c0; /* Sum does not reset (hash.Hash contract) */
    uint64_t bits = c.nbytes * 8;
    uint8_t pad[72] = {0x80};
    uint64_t padlen = (c.nbuf < 56) ? 56 - c.nbuf : 120 - c.nbuf;
    uint8_t lenb[8];
    for (int i = 0; i < 8; i++) lenb[i] = (uint8_t)(bits >> (56 - 8 * i));
    uint64_t saved = c.nbytes;
    orc_sha256_update(&c, pad, padlen);
    orc_sha256_update(&c, lenb, 8);
    (void)saved;
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(c.h[i] >> 24); out[4 * i + 1] = (uint8_t)(c.h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c.h[i] >> 8); out[4 * i + 3] = (uint8_t)c.h[i];
    }
}

void orc_sha256(const uint8_t* p, uint64_t n, uint8_t out[32]) {
    orc_sha256_ctx c;
    orc_sha256_init(&c);
    orc_sha256_update(&c, p, n);
    orc_sha256_sum(&c, out);
}

int orc_have_shani(void) {
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return 0;
    if (!(b & (1u << 29))) return 0; /* SHA */
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & bit_SSE4_1) != 0;
}

__attribute__((target("sha,sse4.1")))
static void sha256_blocks_shani(uint32_t state[8], const uint8_t* data, uint64_t nblocks) {
    const __m128i MASK = _mm_set_epi64x(0x0c0d0e0f08090a0bLL, 0x0405060700010203LL);
    __m128i tmp = _mm_loadu_si128((const __m128i*)&state[0]);
    __m128i s1 = _mm_loadu_si128((const __m128i*)&state[4]);
    tmp = _mm_shuffle_epi32(tmp, 0xB1);
    s1 = _mm_shuffle_epi32(s1, 0x1B);
    __m128i s0 = _mm_alignr_epi8(tmp, s1, 8);
    s1 = _mm_blend_epi16(s1, tmp, 0xF0);
    while (nblocks--) {
        __m128i abef = s0, cdgh = s1, m[4], msg;
#pragma GCC unroll 16
        for (int g = 0; g < 16; g++) {
            if (g < 4) m[g] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(data + 16 * g)), MASK);
            msg = _mm_add_epi32(m[g & 3], _mm_loadu_si128((const __m128i*)&K256[4 * g]));
            s1 = _mm_sha256rnds2_epu32(s1, s0, msg);
            if (g >= 3 && g < 15) {
                __m128i t = _mm_alignr_epi8(m[g & 3], m[(g + 3) & 3], 4);
                m[(g + 1) & 3] = _mm_add_epi32(m[(g + 1) & 3], t);
                m[(g + 1) & 3] = _mm_sha256msg2_epu32(m[(g + 1) & 3], m[g & 3]);
            }
            msg = _mm_shuffle_epi32(msg, 0x0E);
            s0 = _mm_sha256rnds2_epu32(s0, s1, msg);
            if (g >= 1 && g < 13) m[(g + 3) & 3] = _mm_sha256msg1_epu32(m[(g + 3) & 3], m[g & 3]);
        }
        s0 = _mm_add_epi32(s0, abef);
        s1 = _mm_add_epi32(s1, cdgh);
        data += 64;
    }
    tmp = _mm_shuffle_epi32(s0, 0x1B);
    s1 = _mm_shuffle_epi32(s1, 0xB1);
    s0 = _mm_blend_epi16(tmp, s1, 0xF0);
    s1 = _mm_alignr_epi8(s1, tmp, 8);
    _mm_storeu_si128((__m128i*)&state[0], s0);
    _mm_storeu_si128((__m128i*)&state[4], s1);
}

void orc_sha256_shani(const uint8_t* p, uint64_t n, uint8_t out[32]) {
    if (!orc_have_shani()) { orc_sha256(p, n, out); return; }
    orc_sha256_ctx c;
    orc_sha256_init(&c);
    uint64_t nb = n / 64;
    sha256_blocks_shani(c.h, p, nb);
    c.nbytes = nb * 64;
    orc_sha256_update(&c, p + nb * 64, n - nb * 64);
    orc_sha256_sum(&c, out);
}

/* ======================================================================
 * SHA-1 (crypto/sha1) for InfoHash -- core/infohash.go:42-49
 * ====================================================================== */
#define ROL32(x, n) (((x) << (n)) | ((x) >> (32 - (n))))
static void sha1_block(uint32_t h[5], const uint8_t* p) {
    uint32_t w[80];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 80; i++) w[i] = ROL32(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int i = 0; i < 80; i++) {
        uint32_t f, k;
        if (i < 20) { f = (b & c) | (~b & d); k = 0x5A827999; }
        else if (i < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1; }
        else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDC; }
        else { f = b ^ c ^ d; k = 0xCA62C1D6; }
        uint32_t t = ROL32(a, 5) + f + e + k + w[i];
        e = d; d = c; c = ROL32(b, 30); b = a; a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

void orc_sha1(const uint8_t* p, uint64_t n, uint8_t out[20]) {
    uint32_t h[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
    uint64_t full = n / 64;
    for (uint64_t i = 0; i < full; i++) sha1_block(h, p + 64 * i);
    uint8_t tail[128] = {0};
    uint64_t r = n - full * 64;
    memcpy(tail, p + full * 64, r);
    tail[r] = 0x80;
    uint64_t tl = (r < 56) ? 64 : 128;
    uint64_t bits = n * 8;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    sha1_block(h, tail);
    if (tl == 128) sha1_block(h, tail + 64);
    for (int i = 0; i < 5; i++) {
        out[4 * i] = (uint8_t)(h[i] >> 24); out[4 * i + 1] = (uint8_t)(h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(h[i] >> 8); out[4 * i + 3] = (uint8_t)h[i];
    }
}

/* bencode of the info struct -- core/metainfo.go:29-35,37-44 via
 * jackpal/bencode-go @227668e8 (glide.lock:172-173): struct -> dict with keys
 * sorted (Length, Name, PieceLength, PieceSums), ints as i<d>e, strings as
 * <len>:<s>, []uint32 as l...e (nil -> "le": unpinned edge, L == 0). */
static uint64_t put(uint8_t* out, uint64_t cap, uint64_t pos, const char* s, uint64_t n) {
    if (out && pos + n <= cap) memcpy(out + pos, s, n);
    return pos + n;
}
static uint64_t put_int(uint8_t* out, uint64_t cap, uint64_t pos, long long v) {
    char b[32];
    int n = snprintf(b, sizeof b, "i%llde", v);
    return put(out, cap, pos, b, (uint64_t)n);
}

uint64_t orc_bencode_info(int64_t piece_len, const uint32_t* sums, uint64_t n_sums,
                          const char* name, uint64_t name_len, int64_t length,
                          uint8_t* out, uint64_t cap) {
    uint64_t pos = 0;
    char b[32];
    pos = put(out, cap, pos, "d6:Length", 9);
    pos = put_int(out, cap, pos, (long long)length);
    pos = put(out, cap, pos, "4:Name", 6);
    int n = snprintf(b, sizeof b, "%llu:", (unsigned long long)name_len);
    pos = put(out, cap, pos, b, (uint64_t)n);
    pos = put(out, cap, pos, name, name_len);
    pos = put(out, cap, pos, "11:PieceLength", 14);
    pos = put_int(out, cap, pos, (long long)piece_len);
    pos = put(out, cap, pos, "9:PieceSumsl", 12);
    for (uint64_t i = 0; i < n_sums; i++) pos = put_int(out, cap, pos, (long long)sums[i]);
    pos = put(out, cap, pos, "ee", 2);
    return pos;
}

void orc_info_hash(int64_t piece_len, const uint32_t* sums, uint64_t n_sums,
                   const char* name, uint64_t name_len, int64_t length, uint8_t out[20]) {
    uint64_t need = orc_bencode_info(piece_len, sums, n_sums, name, name_len, length, NULL, 0);
    uint8_t* buf = (uint8_t*)malloc(need ? need : 1);
    orc_bencode_info(piece_len, sums, n_sums, name, name_len, length, buf, need);
    orc_sha1(buf, need, out);
    free(buf);
}

/* ======================================================================
 * murmur3 -- spaolacci/murmur3 @9f5d223c (glide.lock:231-232), New64():
 * MurmurHash3_x64_128 with h1 = h2 = seed; Sum64 / Sum return h1
 * (Sum is big-endian 8 bytes).  Used at lib/hrw/rendezvous.go:39.
 * ====================================================================== */
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
}
static inline uint64_t le64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

uint64_t orc_murmur3_h1(const uint8_t* p, uint64_t n, uint64_t seed) {
    const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    uint64_t h1 = seed, h2 = seed;
    uint64_t nb = n / 16;
    for (uint64_t i = 0; i < nb; i++) {
        uint64_t k1 = le64(p + 16 * i), k2 = le64(p + 16 * i + 8);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t* t = p + 16 * nb;
    uint64_t k1 = 0, k2 = 0;
    switch (n & 15) {
    case 15: k2 ^= (uint64_t)t[14] << 48; /* fallthrough */
    case 14: k2 ^= (uint64_t)t[13] << 40; /* fallthrough */
    case 13: k2 ^= (uint64_t)t[12] << 32; /* fallthrough */
    case 12: k2 ^= (uint64_t)t[11] << 24; /* fallthrough */
    case 11: k2 ^= (uint64_t)t[10] << 16; /* fallthrough */
    case 10: k2 ^= (uint64_t)t[9] << 8;   /* fallthrough */
    case 9:  k2 ^= (uint64_t)t[8];
             k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; /* fallthrough */
    case 8:  k1 ^= (uint64_t)t[7] << 56;  /* fallthrough */
    case 7:  k1 ^= (uint64_t)t[6] << 48;  /* fallthrough */
    case 6:  k1 ^= (uint64_t)t[5] << 40;  /* fallthrough */
    case 5:  k1 ^= (uint64_t)t[4] << 32;  /* fallthrough */
    case 4:  k1 ^= (uint64_t)t[3] << 24;  /* fallthrough */
    case 3:  k1 ^= (uint64_t)t[2] << 16;  /* fallthrough */
    case 2:  k1 ^= (uint64_t)t[1] << 8;   /* fallthrough */
    case 1:  k1 ^= (uint64_t)t[0];
             k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= n; h2 ^= n;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2;
    return h1;
}

/* ======================================================================
 * Go math.Log -- src/math/log.go (FreeBSD e_log.c).  Restated operation by
 * operation; compiled with -ffp-contract=off so no FMA is formed (Go's amd64
 * backend does not fuse).  Frexp restated from src/math/frexp.go.
 * ====================================================================== */
static double go_frexp(double f, int* e) {
    if (f == 0 || isinf(f) || isnan(f)) { *e = 0; return f; }
    int exp = 0;
    if (fabs(f) < 2.2250738585072014e-308) { f *= (double)(1ULL << 52); exp = -52; }
    uint64_t x;
    memcpy(&x, &f, 8);
    exp += (int)((x >> 52) & 0x7FF) - 1023 + 1;
    x &= ~(0x7FFULL << 52);
    x |= (uint64_t)(-1 + 1023) << 52;
    memcpy(&f, &x, 8);
    *e = exp;
    return f;
}

double orc_go_log(double x) {
    const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10,
                 L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01,
                 L3 = 2.857142874366239149e-01, L4 = 2.222219843214978396e-01,
                 L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
                 L7 = 1.479819860511658591e-01;
    if (isnan(x) || (isinf(x) && x > 0)) return x;
    if (x < 0) return NAN;
    if (x == 0) return -INFINITY;
    int ki;
    double f1 = go_frexp(x, &ki);
    if (f1 < 1.41421356237309504880168872420969808 / 2) { f1 *= 2; ki--; }
    double f = f1 - 1;
    double k = (double)ki;
    double s = f / (2 + f);
    double s2 = s * s;
    double s4 = s2 * s2;
    double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
    double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
    double R = t1 + t2;
    double hfsq = 0.5 * f * f;
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}

/* hrw.UInt64ToFloat64 -- lib/hrw/rendezvous.go:99-118 with the 8-byte
 * murmur3 Sum: val = BE64(sum) & (2^53-1); when val == 0 and a hasher is
 * given, rehash the 8 bytes once (Reset + Write(bytesUInt)). */
double orc_uint64_to_float64(uint64_t h1, int rehash) {
    const uint64_t m53 = (1ULL << 53) - 1;
    uint64_t val = h1 & m53;
    if (val == 0 && rehash) {
        uint8_t be[8];
        for (int i = 0; i < 8; i++) be[i] = (uint8_t)(h1 >> (56 - 8 * i));
        val = orc_murmur3_h1(be, 8, 0) & m53;
    }
    return (double)val / (double)(1ULL << 53);
}

static int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

/* hex.DecodeString: error on odd length or non-hex (rendezvous.go:154-157 -> NaN) */
static int hex_decode(const char* s, uint64_t n, uint8_t* out) {
    if (n & 1) return -1;
    for (uint64_t i = 0; i < n / 2; i++) {
        int a = hexval(s[2 * i]), b = hexval(s[2 * i + 1]);
        if (a < 0 || b < 0) return -1;
        out[i] = (uint8_t)(a << 4 | b);
    }
    return 0;
}

static double score_bytes(const uint8_t* key, uint64_t klen, const char* label, uint64_t llen,
                          int64_t weight, uint8_t* scratch) {
    memcpy(scratch, key, klen);
    memcpy(scratch + klen, label, llen);
    uint64_t h1 = orc_murmur3_h1(scratch, klen + llen, 0);
    double s = orc_uint64_to_float64(h1, 1);
    return -(double)weight / orc_go_log(s);
}

/* RendezvousHashNode.Score -- lib/hrw/rendezvous.go:151-172 */
double orc_hrw_score(const char* key_hex, uint64_t key_len, const char* label,
                     uint64_t label_len, int64_t weight) {
    uint8_t* kb = (uint8_t*)malloc(key_len / 2 + label_len + 1);
    double r;
    if (hex_decode(key_hex, key_len, kb) != 0) r = NAN;
    else r = score_bytes(kb, key_len / 2, label, label_len, weight, kb);
    free(kb);
    return r;
}

typedef struct { double s; int32_t i; } sc_t;
static int sc_cmp(const void* a, const void* b) {
    const sc_t *x = (const sc_t*)a, *y = (const sc_t*)b;
    /* descending score; NaN compares equal to everything; ties -> ascending index */
    if (x->s > y->s) return -1;
    if (x->s < y->s) return 1;
    return (x->i > y->i) - (x->i < y->i);
}

/* RendezvousHash.GetOrderedNodes -- lib/hrw/rendezvous.go:207-217 */
int orc_hrw_ordered(const char* key_hex, uint64_t key_len, const char* labels,
                    const uint64_t* label_off, const int64_t* weights, uint32_t n_nodes,
                    uint32_t n_out, int32_t* order_out, double* scores_out) {
    uint64_t maxl = 0;
    for (uint32_t j = 0; j < n_nodes; j++) {
        uint64_t l = label_off[j + 1] - label_off[j];
        if (l > maxl) maxl = l;
    }
    uint8_t* kb = (uint8_t*)malloc(key_len / 2 + 1);
    uint8_t* scratch = (uint8_t*)malloc(key_len / 2 + maxl + 1);
    sc_t* v = (sc_t*)malloc(sizeof(sc_t) * (n_nodes ? n_nodes : 1));
    int bad = hex_decode(key_hex, key_len, kb) != 0;
    for (uint32_t j = 0; j < n_nodes; j++) {
        v[j].i = (int32_t)j;
        v[j].s = bad ? NAN : score_bytes(kb, key_len / 2, labels + label_off[j],
                                         label_off[j + 1] - label_off[j], weights[j], scratch);
        if (scores_out) scores_out[j] = v[j].s;
    }
    qsort(v, n_nodes, sizeof(sc_t), sc_cmp);
    uint32_t m = n_out < n_nodes ? n_out : n_nodes;
    for (uint32_t r = 0; r < m; r++) order_out[r] = v[r].i;
    free(kb); free(scratch); free(v);
    return (int)m;
}

/* ring.Locations -- lib/hashring/ring.go:96-118 over a full HRW order. */
uint32_t orc_ring_locations(const int32_t* order, uint32_t n_nodes, const uint8_t* healthy,
                            int32_t max_replica, int32_t* out) {
    int any = 0;
    for (uint32_t j = 0; j < n_nodes; j++) any |= healthy[j] != 0;
    if (!any) { out[0] = order[0]; return 1; }
    uint32_t k = 0;
    for (uint32_t i = 0; i < n_nodes && (k == 0 || (int64_t)i < max_replica); i++)
        if (healthy[order[i]]) out[k++] = order[i];
    return k;
}

/* Every ShardID's ring.Locations (lib/hashring/ring.go:96-118 over rendezvous.go:207-217):
 * key = 4 lowercase hex digits "%04x" of shard (core/digest.go ShardID = hex[:4]); the full
 * HRW order, then the replica filter -- 65,536 rows of row_out (>= 1) owners, -1 padded,
 * counts[shard] owners each.  A plain loop over orc_hrw_ordered + orc_ring_locations: the
 * exhaustive checker of the device owner table (tests/test_gpu_hrw.py). */
void orc_ring_owner_table(const char* labels, const uint64_t* label_off, const int64_t* weights,
                          uint32_t n_nodes, const uint8_t* healthy, int32_t max_replica, uint32_t row_out,
                          int32_t* locs, uint8_t* counts) {
    int32_t* order = (int32_t*)malloc(sizeof(int32_t) * (n_nodes ? n_nodes : 1));
    int32_t* out = (int32_t*)malloc(sizeof(int32_t) * (n_nodes ? n_nodes : 1));
    static const char hx[] = "0123456789abcdef";
    for (uint32_t shard = 0; shard < 65536; shard++) {
        char key[4] = {hx[(shard >> 12) & 15], hx[(shard >> 8) & 15], hx[(shard >> 4) & 15], hx[shard & 15]};
        orc_hrw_ordered(key, 4, labels, label_off, weights, n_nodes, n_nodes, order, NULL);
        uint32_t k = orc_ring_locations(order, n_nodes, healthy, max_replica, out);
        counts[shard] = (uint8_t)k;
        for (uint32_t r = 0; r < row_out; r++) locs[(uint64_t)shard * row_out + r] = r < k ? out[r] : -1;
    }
    free(order);
    free(out);
}

/* pieceLengthConfig.get -- lib/metainfogen/config.go:71-80 (ranges sorted asc). */
int64_t orc_piece_length_for_size(const int64_t* thresholds, const int64_t* lengths,
                                  uint32_t n, int64_t size) {
    int64_t pl = lengths[0];
    for (uint32_t i = 0; i < n; i++) {
        if (size < thresholds[i]) break;
        pl = lengths[i];
    }
    return pl;
}

/* ======================================================================
 * Synthetic content -- splitmix64 counter stream (BASELINE.md / SURVEY §8d).
 * word j of blob i = mix(seed_i + (j+1)*GAMMA), little-endian bytes;
 * seed_i = mix((0x4B52414B454E ^ i) + GAMMA).  The device fill kernel
 * implements the same spec.
 * ====================================================================== */
#define GAMMA 0x9E3779B97F4A7C15ULL
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
uint64_t orc_blob_seed(uint64_t blob_idx) { return mix64((0x4B52414B454EULL ^ blob_idx) + GAMMA); }

static const char ALNUM[] = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789";

void orc_synth_fill(uint64_t blob_idx, uint64_t off, uint8_t* out, uint64_t n, int variant) {
    uint64_t seed = orc_blob_seed(blob_idx);
    uint64_t i = 0;
    while (i < n) {
        uint64_t pos = off + i, j = pos >> 3;
        uint64_t w = mix64(seed + (j + 1) * GAMMA);
        unsigned b = (unsigned)(pos & 7);
        for (; b < 8 && i < n; b++, i++) {
            uint8_t v = (uint8_t)(w >> (8 * b));
            out[i] = variant ? (uint8_t)ALNUM[v % 62] : v;
        }
    }
}

/* ======================================================================
 * CPU baseline: the reference's structure, one blob per worker.
 * ====================================================================== */
typedef struct {
    uint8_t** bufs;
    const uint64_t* lengths;
    uint64_t n;
    int64_t piece_len;
    int fast;
    int passes; /* bit 0: SHA-256 pass, bit 1: CRC piece pass */
    uint8_t* digests;
    uint32_t* sums;
    const uint64_t* sums_off;
    uint64_t n_jobs;  /* n * repeats: job q processes blob q % n */
    volatile uint64_t next;
    pthread_barrier_t bar;
    double t0, t1;
} bl_job;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void bl_blob(bl_job* J, uint64_t b) {
    const uint8_t* p = J->bufs[b];
    uint64_t L = J->lengths[b];
    const uint64_t CH = 32768; /* io.Copy's 32 KiB buffer */
    uint8_t dg[32];
    /* pass 1: SHA-256 (uploader.verify / CAStore.WriteCacheFile) */
    if (!(J->passes & 1)) {
        memset(dg, 0, sizeof dg);
    } else if (J->fast && orc_have_shani()) {
        /* SHA-NI block function over whole 32 KiB chunks (chunks are multiples of 64 B) */
        orc_sha256_ctx c;
        orc_sha256_init(&c);
        uint64_t off = 0;
        while (off + CH <= L) { sha256_blocks_shani(c.h, p + off, CH / 64); off += CH; }
        c.nbytes = off;
        orc_sha256_update(&c, p + off, L - off);
        orc_sha256_sum(&c, dg);
    } else {
        orc_sha256_ctx c;
        orc_sha256_init(&c);
        for (uint64_t off = 0; off < L; off += CH) orc_sha256_update(&c, p + off, L - off < CH ? L - off : CH);
        orc_sha256_sum(&c, dg);
    }
    if (J->digests) memcpy(J->digests + 32 * b, dg, 32);
    /* pass 2: CRC piece sums (Generate -> NewMetaInfo -> calcPieceSums) */
    if (!(J->passes & 2)) return;
    uint64_t P = (uint64_t)J->piece_len, k = 0, off = 0;
    for (;;) {
        uint64_t n = L - off < P ? L - off : P;
        if (n == 0) break;
        uint32_t crc = 0;
        for (uint64_t q = 0; q < n; q += CH) {
            uint64_t m = n - q < CH ? n - q : CH;
            crc = J->fast ? orc_crc32_update_clmul(crc, p + off + q, m) : orc_crc32_update(crc, p + off + q, m);
        }
        if (J->sums) J->sums[J->sums_off[b] + k] = crc;
        k++;
        off += n;
        if (n < P) break;
    }
}

static void* bl_worker(void* arg) {
    bl_job* J = (bl_job*)arg;
    pthread_barrier_wait(&J->bar);
    for (;;) {
        uint64_t q = __atomic_fetch_add(&J->next, 1, __ATOMIC_RELAXED);
        if (q >= J->n_jobs) break;
        bl_blob(J, q % J->n);
    }
    pthread_barrier_wait(&J->bar);
    return NULL;
}

typedef struct { uint8_t* buf; uint64_t idx, len; } fill_arg;
static void* fill_worker(void* a) {
    fill_arg* f = (fill_arg*)a;
    orc_synth_fill(f->idx, 0, f->buf, f->len, 0);
    return NULL;
}

double orc_baseline_run(const uint64_t* blob_idx, const uint64_t* lengths, uint64_t n_blobs,
                        int64_t piece_len, int n_threads, int fast, int passes, uint64_t repeats,
                        uint8_t* digests_out, uint32_t* sums_out, const uint64_t* sums_off) {
    if (n_threads < 1) n_threads = 1;
    if (repeats < 1) repeats = 1;
    bl_job J;
    memset(&J, 0, sizeof J);
    J.bufs = (uint8_t**)calloc(n_blobs, sizeof(uint8_t*));
    /* untimed: materialise the synthetic blobs, n_threads at a time */
    for (uint64_t b0 = 0; b0 < n_blobs; b0 += (uint64_t)n_threads) {
        uint64_t m = n_blobs - b0 < (uint64_t)n_threads ? n_blobs - b0 : (uint64_t)n_threads;
        pthread_t th[m];
        fill_arg fa[m];
        for (uint64_t i = 0; i < m; i++) {
            J.bufs[b0 + i] = (uint8_t*)malloc(lengths[b0 + i] ? lengths[b0 + i] : 1);
            fa[i].buf = J.bufs[b0 + i]; fa[i].idx = blob_idx[b0 + i]; fa[i].len = lengths[b0 + i];
            pthread_create(&th[i], NULL, fill_worker, &fa[i]);
        }
        for (uint64_t i = 0; i < m; i++) pthread_join(th[i], NULL);
    }
    J.lengths = lengths; J.n = n_blobs; J.piece_len = piece_len; J.fast = fast;
    J.passes = passes ? passes : 3;
    J.digests = digests_out; J.sums = sums_out; J.sums_off = sums_off; J.next = 0;
    J.n_jobs = n_blobs * repeats;
    pthread_barrier_init(&J.bar, NULL, (unsigned)n_threads + 1);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, bl_worker, &J);
    double t0 = now_s();
    pthread_barrier_wait(&J.bar);
    pthread_barrier_wait(&J.bar);
    double t1 = now_s();
    for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
    pthread_barrier_destroy(&J.bar);
    for (uint64_t b = 0; b < n_blobs; b++) free(J.bufs[b]);
    free(J.bufs);
    free(th);
    return t1 - t0;
}

/* The reference's per-piece check over buffers that already sit in memory (the agent's
 * received pieces, agentstorage/torrent.go:174-199 writePiece: crc32 over the piece, compared
 * with GetPieceSum) -- the bench's A/B leg that runs over the SAME host bytes the library
 * verified, interleaved with it, so both see one memory placement and one box state.
 * n_threads workers take the next piece in turn; 32 KiB PCLMUL chunks as baseline_run.
 * Returns wall seconds. */
typedef struct { const uint8_t* const* p; const uint64_t* len; uint64_t n, next; uint32_t* out; pthread_barrier_t bar; } bufs_job;
static void* bufs_worker(void* a) {
    bufs_job* J = (bufs_job*)a;
    pthread_barrier_wait(&J->bar);
    for (;;) {
        uint64_t q = __atomic_fetch_add(&J->next, 1, __ATOMIC_RELAXED);
        if (q >= J->n) break;
        const uint64_t CH = 32768; /* io.Copy's 32 KiB buffer */
        uint32_t crc = 0;
        for (uint64_t o = 0; o < J->len[q]; o += CH) {
            uint64_t m = J->len[q] - o < CH ? J->len[q] - o : CH;
            crc = orc_crc32_update_clmul(crc, J->p[q] + o, m);
        }
        J->out[q] = crc;
    }
    pthread_barrier_wait(&J->bar);
    return NULL;
}

double orc_crc_bufs(const uint8_t* const* ptrs, const uint64_t* lens, uint64_t n, int n_threads, uint32_t* out) {
    if (n_threads < 1) n_threads = 1;
    bufs_job J;
    memset(&J, 0, sizeof J);
    J.p = ptrs; J.len = lens; J.n = n; J.out = out;
    pthread_barrier_init(&J.bar, NULL, (unsigned)n_threads + 1);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, bufs_worker, &J);
    double t0 = now_s();
    pthread_barrier_wait(&J.bar);
    pthread_barrier_wait(&J.bar);
    double t1 = now_s();
    for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
    pthread_barrier_destroy(&J.bar);
    free(th);
    return t1 - t0;
}

/* Bounded-memory form for samples too large to hold at once (C3's blobs are 100 MiB -
 * 1 GiB): each worker thread owns one buffer, takes the next blob, materialises it
 * (untimed) and times only its two passes.  Returns the summed busy seconds of all
 * threads; bytes / (busy / threads) is the rate the cores sustain while every one of
 * them has a blob to hash -- the reference's steady state of many concurrent uploads,
 * without the end-of-sample tail of a one-shot batch. */
typedef struct { bl_job* J; const uint64_t* idx; uint64_t maxlen; double busy; } lazy_arg;
static void* lazy_worker(void* a) {
    lazy_arg* A = (lazy_arg*)a;
    bl_job* J = A->J;
    uint8_t* buf = (uint8_t*)malloc(A->maxlen ? A->maxlen : 1);
    for (;;) {
        uint64_t b = __atomic_fetch_add(&J->next, 1, __ATOMIC_RELAXED);
        if (b >= J->n) break;
        orc_synth_fill(A->idx[b], 0, buf, J->lengths[b], 0);
        J->bufs[b] = buf;
        double t0 = now_s();
        bl_blob(J, b);
        A->busy += now_s() - t0;
        J->bufs[b] = NULL;
    }
    free(buf);
    return NULL;
}

double orc_baseline_run_lazy(const uint64_t* blob_idx, const uint64_t* lengths, uint64_t n_blobs,
                             int64_t piece_len, int n_threads, int passes, uint8_t* digests_out,
                             uint32_t* sums_out, const uint64_t* sums_off) {
    if (n_threads < 1) n_threads = 1;
    bl_job J;
    memset(&J, 0, sizeof J);
    J.bufs = (uint8_t**)calloc(n_blobs ? n_blobs : 1, sizeof(uint8_t*));
    J.lengths = lengths; J.n = n_blobs; J.piece_len = piece_len; J.fast = 1;
    J.passes = passes ? passes : 3;
    J.digests = digests_out; J.sums = sums_out; J.sums_off = sums_off; J.next = 0;
    uint64_t maxlen = 0;
    for (uint64_t b = 0; b < n_blobs; b++) maxlen = lengths[b] > maxlen ? lengths[b] : maxlen;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    lazy_arg* la = (lazy_arg*)calloc((size_t)n_threads, sizeof(lazy_arg));
    for (int i = 0; i < n_threads; i++) {
        la[i].J = &J; la[i].idx = blob_idx; la[i].maxlen = maxlen;
        pthread_create(&th[i], NULL, lazy_worker, &la[i]);
    }
    double busy = 0;
    for (int i = 0; i < n_threads; i++) { pthread_join(th[i], NULL); busy += la[i].busy; }
    free(la); free(th); free(J.bufs);
    return busy;
}

/* The reference's passes over CAS FILES, n_threads workers taking whole files in turn (the
 * origin verifies and regenerates many blobs at once).  passes & 2 -- Generate over the
 * cache file (lib/metainfogen/generator.go:41-58 -> core.NewMetaInfo(d, blob, P) ->
 * calcPieceSums, core/metainfo.go:157-179): per piece, io.CopyN(crc32 hasher, file, P), i.e.
 * io.Copy through a LimitReader with its 32 KiB buffer -- read(2) calls of at most 32 KiB,
 * each folded into the piece's CRC (PCLMUL).  passes & 1 -- the upload verify before it
 * (files_sha).  Returns wall seconds; -1 on an open/read failure (a short file: the
 * reference's "unexpected EOF"). */
typedef struct {
    const char* const* paths; const uint64_t* lengths; uint64_t n; int64_t piece_len;
    uint32_t* sums; const uint64_t* sums_off; uint8_t* digests; int passes; uint64_t next; int failed;
} files_job;

/* Pass 1 (passes & 1): the upload verify -- Digester.FromReader over the upload file
 * (origin/blobserver/uploader.go:74-94 -> core/digester.go: io.Copy into sha256), 32 KiB
 * reads, whole reads through the SHA-NI block function. */
static int files_sha(int fd, uint64_t L, uint8_t* buf, uint64_t CH, uint8_t out[32]) {
    orc_sha256_ctx c;
    orc_sha256_init(&c);
    uint64_t got = 0;
    const int ni = orc_have_shani();
    while (got < L) {
        uint64_t want = L - got < CH ? L - got : CH;
        ssize_t r = read(fd, buf, want);
        if (r <= 0) return -1;
        if (ni && c.nbuf == 0 && r % 64 == 0) {
            sha256_blocks_shani(c.h, buf, (uint64_t)r / 64);
            c.nbytes += (uint64_t)r;
        } else {
            orc_sha256_update(&c, buf, (uint64_t)r);
        }
        got += (uint64_t)r;
    }
    orc_sha256_sum(&c, out);
    return 0;
}

static void* files_worker(void* a) {
    files_job* F = (files_job*)a;
    const uint64_t CH = 32768; /* io.Copy's 32 KiB buffer */
    uint8_t* buf = (uint8_t*)malloc(CH);
    for (;;) {
        uint64_t b = __atomic_fetch_add(&F->next, 1, __ATOMIC_RELAXED);
        if (b >= F->n) break;
        if (F->passes & 1) {
            int fd = open(F->paths[b], O_RDONLY);
            uint8_t dg[32];
            if (fd < 0 || files_sha(fd, F->lengths[b], buf, CH, dg) != 0) F->failed = 1;
            else if (F->digests) memcpy(F->digests + 32 * b, dg, 32);
            if (fd >= 0) close(fd);
        }
        if (!(F->passes & 2)) continue;
        /* pass 2: Generate re-reads the committed cache file for the piece sums */
        int fd = open(F->paths[b], O_RDONLY);
        if (fd < 0) { F->failed = 1; continue; }
        uint64_t L = F->lengths[b], P = (uint64_t)F->piece_len, off = 0, k = 0;
        while (off < L) {
            uint64_t n = L - off < P ? L - off : P, got = 0;
            uint32_t crc = 0;
            while (got < n) {
                uint64_t want = n - got < CH ? n - got : CH;
                ssize_t r = read(fd, buf, want);
                if (r <= 0) { F->failed = 1; break; }
                crc = orc_crc32_update_clmul(crc, buf, (uint64_t)r);
                got += (uint64_t)r;
            }
            if (got < n) break;
            if (F->sums) F->sums[F->sums_off[b] + k] = crc;
            k++;
            off += n;
        }
        close(fd);
    }
    free(buf);
    return NULL;
}

double orc_baseline_files(const char* const* paths, const uint64_t* lengths, uint64_t n, int64_t piece_len,
                          int n_threads, int passes, uint32_t* sums_out, const uint64_t* sums_off,
                          uint8_t* digests_out) {
    if (n_threads < 1) n_threads = 1;
    files_job F;
    memset(&F, 0, sizeof F);
    F.paths = paths; F.lengths = lengths; F.n = n; F.piece_len = piece_len;
    F.sums = sums_out; F.sums_off = sums_off; F.digests = digests_out; F.passes = passes ? passes : 2;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    double t0 = now_s();
    for (int i = 0; i < n_threads; i++) pthread_create(&th[i], NULL, files_worker, &F);
    for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
    double t1 = now_s();
    free(th);
    return F.failed ? -1.0 : t1 - t0;
}

typedef struct {
    const uint8_t* digests; uint64_t n; const char* labels; const uint64_t* label_off;
    uint32_t n_nodes; const uint8_t* healthy; int32_t max_replica;
    int32_t* locs; uint8_t* counts; int tid, nt;
} hrw_arg;

static void* hrw_worker(void* a) {
    hrw_arg* H = (hrw_arg*)a;
    uint32_t N = H->n_nodes;
    int64_t* w = (int64_t*)malloc(sizeof(int64_t) * N);
    int32_t* order = (int32_t*)malloc(sizeof(int32_t) * N);
    int32_t loc[256];
    uint32_t mo = H->max_replica > 1 ? (uint32_t)H->max_replica : 1;
    for (uint32_t j = 0; j < N; j++) w[j] = 100; /* ring.go:28,152 */
    static const char hx[] = "0123456789abcdef";
    for (uint64_t i = (uint64_t)H->tid; i < H->n; i += (uint64_t)H->nt) {
        const uint8_t* d = H->digests + 32 * i;
        char key[4] = {hx[d[0] >> 4], hx[d[0] & 15], hx[d[1] >> 4], hx[d[1] & 15]}; /* ShardID */
        orc_hrw_ordered(key, 4, H->labels, H->label_off, w, N, N, order, NULL);
        uint32_t k = orc_ring_locations(order, N, H->healthy, H->max_replica, loc);
        if (H->locs) for (uint32_t r = 0; r < mo; r++) H->locs[i * mo + r] = r < k ? loc[r] : -1;
        if (H->counts) H->counts[i] = (uint8_t)k;
    }
    free(w); free(order);
    return NULL;
}

double orc_baseline_hrw(const uint8_t* digests, uint64_t n, const char* labels,
                        const uint64_t* label_off, uint32_t n_nodes, const uint8_t* healthy,
                        int32_t max_replica, int n_threads, int32_t* locs_out, uint8_t* counts_out) {
    if (n_threads < 1) n_threads = 1;
    pthread_t th[n_threads];
    hrw_arg a[n_threads];
    double t0 = now_s();
    for (int t = 0; t < n_threads; t++) {
        a[t] = (hrw_arg){digests, n, labels, label_off, n_nodes, healthy, max_replica,
                         locs_out, counts_out, t, n_threads};
        pthread_create(&th[t], NULL, hrw_worker, &a[t]);
    }
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
    return now_s() - t0;
}
