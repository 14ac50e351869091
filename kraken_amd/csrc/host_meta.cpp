// host_meta.cpp -- host-side pieces of the metainfo path that stay on the CPU by
// design: bencode + SHA-1 InfoHash (O(pieces), core/metainfo.go:37-44,
// core/infohash.go:42-49) and the piece-length range table
// (lib/metainfogen/config.go:71-80).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/kraken_hip.h"

namespace krk {
void set_error(int code, const char* fmt, ...);

namespace {

struct Sha1 {
    uint32_t h[5] = {0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0};
    uint8_t buf[64];
    uint64_t n = 0;
    uint32_t nb = 0;

    static uint32_t rol(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
    void block(const uint8_t* p) {
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
    void write(const void* data, size_t len) {
        const uint8_t* p = static_cast<const uint8_t*>(data);
        n += len;
        while (len) {
            const uint32_t take = (uint32_t)(len < 64 - nb ? len : 64 - nb);
            memcpy(buf + nb, p, take);
            nb += take; p += take; len -= take;
            if (nb == 64) { block(buf); nb = 0; }
        }
    }
    void sum(uint8_t out[20]) {
        const uint64_t bits = n * 8;
        const uint8_t pad = 0x80, zero = 0;
        write(&pad, 1);
        while (nb != 56) write(&zero, 1);
        uint8_t lb[8];
        for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
        write(lb, 8);
        for (int i = 0; i < 5; ++i)
            for (int k = 0; k < 4; ++k) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
    }
};

// jackpal/bencode-go encoding of core.info (struct -> dict, keys in sorted order:
// Length, Name, PieceLength, PieceSums; []uint32 -> list of ints).
template <class Sink>
void bencode_info(Sink& out, int64_t piece_length, const uint32_t* sums, uint64_t n_sums,
                  const char* name, uint64_t name_len, int64_t length) {
    char b[48];
    int k;
    out("d6:Lengthi", 10);
    k = snprintf(b, sizeof b, "%lld", (long long)length); out(b, k);
    out("e4:Name", 7);
    k = snprintf(b, sizeof b, "%llu:", (unsigned long long)name_len); out(b, k);
    out(name, name_len);
    out("11:PieceLengthi", 15);
    k = snprintf(b, sizeof b, "%lld", (long long)piece_length); out(b, k);
    out("e9:PieceSumsl", 13);
    for (uint64_t i = 0; i < n_sums; ++i) {
        k = snprintf(b, sizeof b, "i%ue", sums[i]);
        out(b, k);
    }
    out("ee", 2);
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
    krk::Sha1 h;
    auto sink = [&](const char* p, uint64_t n) { h.write(p, n); };
    krk::bencode_info(sink, piece_length, sums, n_sums, name, name_len, length);
    h.sum(out20);
    return KRK_OK;
}

int krk_bencode_info(int64_t piece_length, const uint32_t* sums, uint64_t n_sums, const char* name,
                     uint64_t name_len, int64_t length, uint8_t* out, uint64_t cap, uint64_t* written) {
    uint64_t pos = 0;
    auto sink = [&](const char* p, uint64_t n) {
        if (out && pos + n <= cap) memcpy(out + pos, p, n);
        pos += n;
    };
    krk::bencode_info(sink, piece_length, sums, n_sums, name, name_len, length);
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
