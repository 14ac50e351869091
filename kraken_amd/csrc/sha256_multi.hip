// sha256_multi.hip -- multi-buffer SHA-256 for gfx950 (core.Digester,
// core/digester.go:28-72 over crypto/sha256).
//
// SHA-256 is a sequential Merkle-Damgard chain per blob, so parallelism comes only
// from independent blobs.  Production kernel: sha256_ws_kernel, a wave-specialised
// workgroup of producer/consumer wave pairs:
//  * the producer wave loads each stream's 64-byte blocks two steps ahead, builds
//    the padded tail blocks, expands the message schedule and writes
//    KW[r] = W[r] + K[r] into an LDS ring;
//  * the consumer wave runs only the rounds, reading KW from the ring with
//    ds_read_b128, one s_barrier per producer step.
// Streams per consumer wave: 8 with eight lanes per stream (sha256_w8_kernel: an E quad
// and an A quad, Sigma rotated across the quad, an 8-instruction round, blocks
// pipelined; up to 16 x CUs streams), 32 with two lanes (the A lane carries the a..d
// history, the E lane e..h, a 9-instruction round) or 64 with one lane (a
// 14-instruction round) as the batch fills the chip.  Jobs start from
// the IV or a midstate (streaming Digester, windowed host paths) and either write
// the digest (final, padding done here) or the midstate back.  No MFMA: the work is
// 32-bit integer rotate/xor/add.
#include <stdlib.h>

#include <atomic>
#include <mutex>

#include "../../include/kraken_hip_internal.h"
#include "kernels.hpp"
#include "knobs.hpp"
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

#ifdef KRK_DIAG  // one lane does loads + schedule + rounds: the round-1 baseline kernel
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

#endif  // KRK_DIAG

// ---------------------------------------------------------------------------
// Wave-specialised variant.  A workgroup = 2 waves over the same 64 streams:
// wave 0 (producer) loads each block, builds the padded tail blocks and expands
// the message schedule into KW[r] = W[r] + K[r] in an LDS ring; wave 1 (consumer)
// only runs the 64 rounds (no VMEM, no schedule: ~14 VALU ops per round).  The
// two waves sit on different SIMDs, so the consumer keeps its full issue rate.
// One s_barrier per block; the producer fills a ring of kSlots slots (one lane,
// 4 slots) or kSlots2 slots (two lanes per stream, where each producer step
// builds two blocks), see produce_step.
constexpr int kSlots = 4;
#define KRK_RING2 3  // two-lane ring slots (a ring one slot deeper measured 0.4 % slower, profiles/r03/c3_ring4_ab.txt)
constexpr int kSlots2 = 2 * KRK_RING2;  // two lanes: block positions in the ring ...
constexpr int kRing2 = kSlots2 / 2;     // ... in 3 slots, two blocks per slot (A / E columns)
constexpr int kSlotWords = 64 * 64;  // 64 rounds x 64 lanes
// eight lanes: 1 KiB of 1s past the all-1 slot (the A lanes' column walks one block ahead)
constexpr uint32_t kOnesPad8 = 256;

// LDS image of one slot: [round/4][lane][4] words -> a lane's 4 consecutive KW
// are one conflict-free ds_read_b128 / ds_write_b128 across the wave.
__device__ __forceinline__ uint32_t kw_index(int slot, int quad, uint32_t lane) {
    return (uint32_t)slot * kSlotWords + ((uint32_t)quad * 64 + lane) * 4;
}
// Word offset of quad 0 of one column of a slot; quad q is 256 words further.
__device__ __forceinline__ uint32_t kw_base(uint32_t slot, uint32_t col) { return slot * kSlotWords + col * 4; }

// Two lanes per stream: block b lives in slot (b / 2) % kRing2, the even block in
// the A lanes' columns and the odd block in the E lanes' (each producer lane writes
// its own column).  Every consumer lane reads column lane ^ 15 for even blocks
// (the E lanes their partner's, the A lanes the all-1 slot's) and its own column
// for odd blocks: a bijection within each 16-lane row, so the ds_read_b128 stays
// conflict-free.  3 slots + the all-1 slot = 64 KiB: two workgroups fit a CU.
__device__ __forceinline__ uint32_t kw2_base(uint32_t b, bool is_e, uint32_t lane) {
    return kw_base(is_e ? (b >> 1) % kRing2 : kRing2, (b & 1) ? lane : (lane ^ 15u));
}

__device__ __forceinline__ uint32_t job_blocks(const ShaJob& job) {
    const uint32_t nblk = (uint32_t)(job.len / 64);
    if (!(job.flags & kShaFinal)) return nblk;
    return nblk + (((uint32_t)(job.len & 63) >= 56) ? 2u : 1u);
}

// Bytes of block b that lie inside the run (64 for full blocks, the tail for
// b == len/64, 0 past the data).
__device__ __forceinline__ uint32_t block_bytes(const ShaJob& job, uint32_t b) {
    const uint64_t off = (uint64_t)b * 64;
    return off < job.len ? (uint32_t)min<uint64_t>(64, job.len - off) : 0u;
}

// Issue the loads of block b into raw[]: the five 16-byte-aligned chunks from
// (block start & ~15), as five dwordx4 that every lane always issues (no branch,
// so the compiler's vmcnt accounting stays exact and the loads stay in flight
// across the schedule work of the blocks in between).  An aligned chunk that
// holds a byte of the run lies in a page holding that byte, so it is always
// mapped; chunks past the last one holding a byte of the block re-read that
// chunk, and lanes with no bytes read the always-valid `safe` chunk.
constexpr int kRaw = 5;  // chunks

__device__ __forceinline__ void fetch(const ShaJob& job, uint32_t b, u32x4 raw[kRaw], uint64_t safe) {
    const uint64_t a = job.ptr + (uint64_t)b * 64;
    const uint32_t n = block_bytes(job, b);
    const uint64_t base = n ? (a & ~uint64_t(15)) : safe;
    const uint32_t cmax = n ? (uint32_t)(((a + n - 1) >> 4) - (a >> 4)) : 0u;  // <= 4
    const uint64_t lo = job.ptr & ~uint64_t(15), hi = (job.ptr + job.len + 15) & ~uint64_t(15);
    (void)lo;
    (void)hi;
    gptr<u32x4> q = as_global<u32x4>(base);
#pragma unroll
    for (int c = 0; c < 5; ++c) {
        const uint32_t cc = min((uint32_t)c, cmax);
        raw[c] = (!n || KRK_GUARD(base + 16 * cc, 16, lo, hi, 1)) ? q[cc] : u32x4{0, 0, 0, 0};
    }
}

// Block b's 16 big-endian message words from raw[] (+ the 0x80 terminator and the
// bit length on the final blocks), expanded to KW[r] = W[r] + K[r] in ring slot b % kNs,
// LDS column `lane`.
template <int kNs>
__device__ __forceinline__ void build(const ShaJob& job, uint32_t b, const u32x4 rawc[kRaw], uint32_t base,
                                      uint32_t* lds) {
    constexpr uint32_t K[64] = {KRK_K256};
    const uint32_t n = block_bytes(job, b);
    uint32_t raw[4 * kRaw];
#pragma unroll
    for (int c = 0; c < kRaw; ++c) {
        raw[4 * c + 0] = rawc[c].x; raw[4 * c + 1] = rawc[c].y; raw[4 * c + 2] = rawc[c].z; raw[4 * c + 3] = rawc[c].w;
    }
    uint32_t w[16];
    // Wave-uniform split: every live lane on a 16-byte aligned run inside a full block.
    if (__all((n == 64 && (job.ptr & 15) == 0) || b >= job_blocks(job))) {
#pragma unroll
        for (int j = 0; j < 16; ++j) w[j] = bswap(raw[j]);
    } else {
        // Dword q of the first chunk starts the block; bytes shift by sh within it.
        const uint32_t qd = (uint32_t)(job.ptr >> 2) & 3, sh = (uint32_t)(job.ptr & 3) * 8;
        // Value muxes (v_bfi), not selects of addresses: a selected index would
        // leave these arrays in scratch.
        const uint32_t m1 = 0u - (qd & 1), m2 = 0u - ((qd >> 1) & 1);
        uint32_t t[19], u[17];
#pragma unroll
        for (int j = 0; j < 19; ++j) t[j] = (raw[j + 1] & m1) | (raw[j] & ~m1);
#pragma unroll
        for (int j = 0; j < 17; ++j) u[j] = (t[j + 2] & m2) | (t[j] & ~m2);
        const bool fin = (job.flags & kShaFinal) != 0;
        const uint32_t nblk = (uint32_t)(job.len / 64);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            uint32_t x = __builtin_amdgcn_alignbit(u[j + 1], u[j], sh);
            const int keep = (int)n - 4 * j;
            if (keep <= 0) x = 0;
            else if (keep < 4) x &= (1u << (8 * keep)) - 1;
            w[j] = bswap(x);
            if (fin && b == nblk && j == (int)(n >> 2)) w[j] |= 0x80u << (24 - 8 * (n & 3));
        }
        if (fin && b == job_blocks(job) - 1) {
            const uint64_t bits = (job.prefix + job.len) * 8;
            w[14] = (uint32_t)(bits >> 32);
            w[15] = (uint32_t)bits;
        }
    }
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
        *reinterpret_cast<u32x4*>(lds + base + 256 * q) = u32x4{kw[0], kw[1], kw[2], kw[3]};
    }
}

// One producer step over blocks b .. b + kStep - 1 (b wave-uniform); this lane
// builds block ob (one lane per stream: ob = b; two lanes: the A lane b, the E
// lane b + 1, both into the E lane's column `col`).  The consumer passes one
// barrier per step (kStep blocks), the producer one per step too, so a step has
// a whole consumer step of time (two blocks with two lanes: a producer step takes
// 1.4 us, a consumer block 1.26).  Slot reuse: step m lands on the slots of step
// m - kNs/kStep, free once the consumer has started step m - kNs/kStep + 1, i.e.
// passed barrier m - kNs/kStep + 1; the producer reaches barrier j only after
// building step j + kNs/kStep - 1, and the consumer needs steps j and j + 1 (its
// prefetch of the next block's first quads) after barrier j.  The loads of this
// lane's block two steps ahead are issued here (always, so no branch sits between
// a load and its use), then block ob is built from registers.
template <int kNs, int kStep, bool kNoLoad = false>
__device__ __forceinline__ void produce_step(const ShaJob& job, uint32_t b, uint32_t ob, uint32_t nb,
                                             uint32_t col, uint32_t* lds, const u32x4 use[kRaw],
                                             u32x4 next[kRaw], uint64_t safe, uint32_t& passed) {
    const bool act = b < nb;
    if (act) {
        while (passed + kNs / kStep < b / kStep + 2) {
            __syncthreads();
            ++passed;
        }
    }
    if (kNoLoad) {
#pragma unroll
        for (int c = 0; c < kRaw; ++c) next[c] = u32x4{b, col, (uint32_t)c, b ^ col};
    } else {
        fetch(job, ob + 2 * kStep, next, safe);
    }
    // one slot a step: block ob in slot (ob / kStep) % (kNs / kStep) (ob - b < kStep)
    const uint32_t base = kw_base((ob / kStep) % (kNs / kStep), col);
    if (act) build<kNs>(job, ob, use, base, lds);
}

// Four SHA-256 rounds as one fixed 56-instruction sequence.  The compiler's
// scheduler does not model the gfx950 dependent-issue latency and places most
// results right before their consumer; here every result is consumed at least
// one instruction after it is produced, so a lone wave keeps issuing one VALU op
// per slot (and the hazard recognizer pads once per four rounds, not per round).
// hk = h + KW[r] enters precomputed; each round forms the next one's
// (g + KW[r+1]) in its own shadow.  Round operands: state A..G, HK, next KW,
// outputs NE (new e), NA (new a), NH (next hk); S1 lands in r6, S0 in q2.
#define KRK_SHA_ROUND(A, B, C, D, E, F, G, HK, KWN, NE, NA, NH)                  \
    "v_alignbit_b32 %[r6], %[" #E "], %[" #E "], 6\n\t"                        \
    "v_alignbit_b32 %[r11], %[" #E "], %[" #E "], 11\n\t"                      \
    "v_alignbit_b32 %[r25], %[" #E "], %[" #E "], 25\n\t"                      \
    "v_bitop3_b32 %[ch], %[" #E "], %[" #F "], %[" #G "] bitop3:0xca\n\t"     \
    "v_bitop3_b32 %[r6], %[r6], %[r11], %[r25] bitop3:0x96\n\t"                \
    "v_alignbit_b32 %[q2], %[" #A "], %[" #A "], 2\n\t"                        \
    "v_add3_u32 %[t1], %[" #HK "], %[r6], %[ch]\n\t"                           \
    "v_alignbit_b32 %[q13], %[" #A "], %[" #A "], 13\n\t"                      \
    "v_add_u32_e32 %[" #NE "], %[" #D "], %[t1]\n\t"                           \
    "v_alignbit_b32 %[q22], %[" #A "], %[" #A "], 22\n\t"                      \
    "v_bitop3_b32 %[mj], %[" #A "], %[" #B "], %[" #C "] bitop3:0xe8\n\t"     \
    "v_bitop3_b32 %[q2], %[q2], %[q13], %[q22] bitop3:0x96\n\t"                \
    "v_add_u32_e32 %[" #NH "], %[" #G "], %[" #KWN "]\n\t"                     \
    "v_add3_u32 %[" #NA "], %[t1], %[q2], %[mj]\n\t"

// Rounds r..r+3: (a..g, hk) in, KW[r+1..r+4] in (0 past the block), state after
// round r+3 out.  The h entering round r+3 is e1 (returned for the final add).
__device__ __forceinline__ void sha_quad(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                                         uint32_t& f, uint32_t& g, uint32_t& hk, uint32_t k1, uint32_t k2,
                                         uint32_t k3, uint32_t k4, uint32_t& h_last) {
    uint32_t r6, r11, r25, ch, q2, t1, q13, q22, mj;
    uint32_t e1, e2, e3, e4, a1, a2, a3, a4, h1, h2, h3, h4;
    asm volatile(KRK_SHA_ROUND(a, b, c, d, e, f, g, hk, k1, e1, a1, h1)
                 KRK_SHA_ROUND(a1, a, b, c, e1, e, f, h1, k2, e2, a2, h2)
                 KRK_SHA_ROUND(a2, a1, a, b, e2, e1, e, h2, k3, e3, a3, h3)
                 KRK_SHA_ROUND(a3, a2, a1, a, e3, e2, e1, h3, k4, e4, a4, h4)
                 : [r6] "=&v"(r6), [r11] "=&v"(r11), [r25] "=&v"(r25), [ch] "=&v"(ch), [q2] "=&v"(q2),
                   [t1] "=&v"(t1), [q13] "=&v"(q13), [q22] "=&v"(q22), [mj] "=&v"(mj), [e1] "=&v"(e1),
                   [e2] "=&v"(e2), [e3] "=&v"(e3), [e4] "=&v"(e4), [a1] "=&v"(a1), [a2] "=&v"(a2),
                   [a3] "=&v"(a3), [a4] "=&v"(a4), [h1] "=&v"(h1), [h2] "=&v"(h2), [h3] "=&v"(h3),
                   [h4] "=&v"(h4)
                 : [a] "v"(a), [b] "v"(b), [c] "v"(c), [d] "v"(d), [e] "v"(e), [f] "v"(f), [g] "v"(g),
                   [hk] "v"(hk), [k1] "v"(k1), [k2] "v"(k2), [k3] "v"(k3), [k4] "v"(k4));
    h_last = e1;
    a = a4; b = a3; c = a2; d = a1;
    e = e4; f = e3; g = e2;
    hk = h4;
}
#undef KRK_SHA_ROUND

// The 64 rounds of one block; quads 0 and 1 of its KW arrive already loaded
// (read before the barrier that opens the block), the rest are read two quads ahead.
__device__ __forceinline__ void rounds(uint32_t h[8], const uint32_t* lds, int slot, uint32_t lane,
                                       const u32x4& k0, const u32x4& k1) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6];
    uint32_t hk = h[7] + k0[0], hl = 0;
    u32x4 kw = k0, nkw = k1, nnkw = k1;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        // quad q+2 is read while quads q and q+1 are consumed (one quad of slack)
        if (q + 2 < 16) nnkw = *reinterpret_cast<const u32x4*>(lds + kw_index(slot, q + 2, lane));
        sha_quad(a, b, c, d, e, f, g, hk, kw[1], kw[2], kw[3], q + 1 < 16 ? nkw[0] : 0u, hl);
        kw = nkw;
        nkw = nnkw;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hl;
}

__device__ __forceinline__ u32x4 kw_quad(const uint32_t* lds, int slot, int q, uint32_t lane) {
    return *reinterpret_cast<const u32x4*>(lds + kw_index(slot, q, lane));
}

// ---------------------------------------------------------------------------
// Two lanes per stream.  One lane runs the rounds of a stream at one VALU op per
// ~4.4 cycles (a lone wave cannot issue faster), so when a batch has fewer
// streams than the chip has SIMDs the per-stream chain is the bound, and spending
// two lanes on one stream buys a shorter chain.  The A lane keeps the a-history
// (a, b, c, d) and the E lane the e-history (e, f, g, h) of the same stream; both
// run ONE instruction stream with per-lane operands, the A lane two rounds behind
// the E lane (in instruction-round n the E lane runs round n, the A lane n-2):
//   S = rotr(x0, r1) ^ rotr(x0, r2) ^ rotr(x0, r3)   A: Sigma0(a)        E: Sigma1(e)
//   k = x0 ^ (x1 & mA) ^ ~mA                         A: a ^ b            E: ~e
//   F = k ? x2 : x1                                  A: Maj(a, b, c)     E: Ch(e, f, g)
//   z = (x3 ^ mA) + W                                A: -d  (W = 1)      E: h + KW[n]
//   P = partner's x1 + z                             A: e[n-1] - d       E: a[n-3] + h + KW[n]
//   x0' = S + F + P                                  A: a[n-1]           E: e[n+1]
// With the two-round skew the A lane's T1 (= e[n-1] - d) and the E lane's d
// (= a[n-3]) both sit in the partner's x1, so ONE unmasked DPP add (row_mirror)
// serves both lanes, and it reads a register written two rounds earlier: the
// recurrence is three VALU ops deep (rotate, xor3, add3) and a round is nine ops
// (7 VOP3, 1 DPP, 1 xad).  tools/micro/sha2lane.hip prices the variants.
//
// Lane layout: in each DPP row of 16 lanes, stream s's A lane is lane s and its E
// lane lane 15 - s (row_mirror pairs them); 8 streams a row, 32 a wave.  W comes
// from the LDS ring like KW: the E lanes' columns hold KW, the A lanes' columns
// are filled with 1 once at kernel start and never written again.
__device__ __forceinline__ bool two_lane_is_e(uint32_t lane) { return (lane >> 3) & 1; }
__device__ __forceinline__ uint32_t two_lane_stream(uint32_t lane) {
    return (lane >> 4) * 8 + (two_lane_is_e(lane) ? 7 - (lane & 7) : (lane & 7));
}

// One instruction-round; the new x0 overwrites x3 (dead once P is formed) or NX.
// z for the NEXT round is formed here (its x3 is this round's x2) so that no DPP
// reads a result of the instruction right before it (that costs ~8 cycles; see
// tools/micro/sha2lane.hip: 38 cycles a round this way, 47 with z formed in-round).
#define KRK_SHA2_ROUND(X0, X1, X2, NX, WN)                                              \
    "v_add_u32_dpp %[p], %[" #X1 "], %[z] row_mirror row_mask:0xf bank_mask:0xf\n\t"    \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                          \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                          \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                          \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_xad_u32 %[z], %[" #X2 "], %[ma], %[" #WN "]\n\t"                                \
    "v_add3_u32 %[" #NX "], %[t1], %[k], %[p]\n\t"

struct TwoLaneConst {
    uint32_t r1, r2, r3, ma, one_a;
};

#define KRK_SHA2_OPERANDS                                                                             \
    : [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [k] "=&v"(kk), [p] "=&v"(p), [z] "+v"(z),       \
      [R0] "+v"(R0), [R1] "+v"(R1), [R2] "+v"(R2), [R3] "+v"(R3)
#define KRK_SHA2_CONSTS [r1] "v"(c.r1), [r2] "v"(c.r2), [r3] "v"(c.r3), [ma] "v"(c.ma)

// ---------------------------------------------------------------------------
// Eight lanes per stream.  Four of the two-lane round's nine instructions compute
// Sigma (three v_alignbit rotations + an xor3).  Here a stream has an E quad and an
// A quad of lanes: the three active lanes of a quad carry the same history and each
// rotates by ONE of the three Sigma amounts (r1 per lane), and two quad_perm DPP
// xors combine the three rotations so every active lane ends with the full Sigma:
// eight instructions a round (one v_alignbit + two DPP xors in place of three
// v_alignbit + the xor3), all 8-byte encodings, whose fetch sets the pace of a lone
// wave (tools/micro/sha8lane.hip: 2,684 vs 2,920 cycles a block, bit-exact).  The
// rest is the two-lane round: k / F (Maj or Ch), z for the next round, one cross
// add P = partner's x1 + z, x0' = S + F + P, the A quad two rounds behind the E quad.
// Lane layout: in each DPP row of 16 lanes quads 0 / 1 are the E quads of streams
// 2r / 2r + 1 and quads 2 / 3 their A quads, so row_ror:8 pairs E with A; lane 3 of
// each quad rotates once and its state is never read.  8 streams a wave.  The first
// DPP xor reads t1 three instructions after it is written (two wait states needed),
// the cross add reads a register written a round earlier.
#define KRK_SHA8_ROUND(X0, X1, X2, NX, WN)                                                   \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                               \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                      \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                       \
    "v_xor_b32_dpp %[t2], %[t1], %[t1] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t"  \
    "v_xor_b32_dpp %[t2], %[t1], %[t2] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t"  \
    "v_add_u32_dpp %[p], %[" #X1 "], %[z] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"          \
    "v_xad_u32 %[z], %[" #X2 "], %[ma], %[" #WN "]\n\t"                                     \
    "v_add3_u32 %[" #NX "], %[t2], %[k], %[p]\n\t"
#define KRK_SHA8_OPERANDS                                                                    \
    : [t1] "=&v"(t1), [t2] "=&v"(t2), [k] "=&v"(kk), [p] "=&v"(p), [z] "+v"(z), [R0] "+v"(R0), \
      [R1] "+v"(R1), [R2] "+v"(R2), [R3] "+v"(R3)
#define KRK_SHA8_CONSTS [r1] "v"(c.r1), [ma] "v"(c.ma)

// Instruction-rounds 4q..4q+3; W of rounds 4q+1..4q+4 (for the z's).  History
// registers rotate: in instruction-round n, x0 = R[n%4], x3 = R[(n+1)%4].
__device__ __forceinline__ void sha2_quad(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                          const TwoLaneConst& c, uint32_t w1, uint32_t w2, uint32_t w3,
                                          uint32_t w4) {
    uint32_t t1, t2, t3, kk, p;
    asm volatile(KRK_SHA2_ROUND(R0, R3, R2, R1, w1)
                 KRK_SHA2_ROUND(R1, R0, R3, R2, w2)
                 KRK_SHA2_ROUND(R2, R1, R0, R3, w3)
                 KRK_SHA2_ROUND(R3, R2, R1, R0, w4)
                 KRK_SHA2_OPERANDS
                 : KRK_SHA2_CONSTS, [w1] "v"(w1), [w2] "v"(w2), [w3] "v"(w3), [w4] "v"(w4));
    (void)t3;
}

// The W read-ahead: a consumer reads KW quads kAhead quads before their use (quad q+1's
// first W feeds quad q's last z, so its read must have landed when quad q starts: issued
// one quad before its use it stalled ~230 cycles a block in round 1's one-block-a-step
// two-lane consumer), and the next block's first kAhead quads during the last ones.
#define KRK_SHA_AHEAD 3
constexpr int kAhead = KRK_SHA_AHEAD;
#define KRK_SHA8_UNROLL 4  // eight-lane consumer: blocks per loop iteration
static_assert(kAhead >= 2 && kAhead <= 8, "read-ahead distance");

// Rounds n = 4j + 2 .. 4j + 5 of an eight-lane block (block8p), the register roles of
// instruction-rounds 2 .. 5: W operands are W[n + 1] for the z of the next round.
__device__ __forceinline__ void sha8_quad2(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                           const TwoLaneConst& c, uint32_t w1, uint32_t w2, uint32_t w3,
                                           uint32_t w4) {
    uint32_t t1, t2, kk, p;
    asm volatile(KRK_SHA8_ROUND(R2, R1, R0, R3, w1) KRK_SHA8_ROUND(R3, R2, R1, R0, w2)
                 KRK_SHA8_ROUND(R0, R3, R2, R1, w3) KRK_SHA8_ROUND(R1, R0, R3, R2, w4)
                 KRK_SHA8_OPERANDS
                 : KRK_SHA8_CONSTS, [w1] "v"(w1), [w2] "v"(w2), [w3] "v"(w3), [w4] "v"(w4));
}

// W read groups of the eight-lane consumer: three quads read between 12-round asm blocks, four quads ahead (a group's last block
// needs quad j + 3, read one group earlier), so ONE s_waitcnt precedes every 12 rounds;
// 1 = one read and one wait per 4 rounds (round 2's first form).  C2-shaped A/B on one
// box (profiles/r02/sha8_read_groups.jsonl): 56.2 MB/s a stream with one read a group,
// 57.2 with pairs, 58.7 with threes, 58.3 with fives (two asm statements a group); the
// threes' reads issued mid-way through the previous group (two six-round statements)
// instead of right before its wait: 59.1 vs 59.2 (profiles/r02/sha8_read_split.jsonl).
constexpr int kAhead8 = 4;
// Twelve eight-lane rounds, n = 4j + 2 .. 4j + 13: W quads a = j, b = j + 1, d = j + 2,
// e = j + 3 (each block of four takes its first quad's last word and the next quad's
// first three).
__device__ __forceinline__ void sha8_dodec2(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                            const TwoLaneConst& c, const u32x4& a, const u32x4& b, const u32x4& d,
                                            const u32x4& e) {
    uint32_t t1, t2, kk, p;
    asm volatile(KRK_SHA8_ROUND(R2, R1, R0, R3, w1) KRK_SHA8_ROUND(R3, R2, R1, R0, w2)
                 KRK_SHA8_ROUND(R0, R3, R2, R1, w3) KRK_SHA8_ROUND(R1, R0, R3, R2, w4)
                 KRK_SHA8_ROUND(R2, R1, R0, R3, w5) KRK_SHA8_ROUND(R3, R2, R1, R0, w6)
                 KRK_SHA8_ROUND(R0, R3, R2, R1, w7) KRK_SHA8_ROUND(R1, R0, R3, R2, w8)
                 KRK_SHA8_ROUND(R2, R1, R0, R3, w9) KRK_SHA8_ROUND(R3, R2, R1, R0, w10)
                 KRK_SHA8_ROUND(R0, R3, R2, R1, w11) KRK_SHA8_ROUND(R1, R0, R3, R2, w12)
                 KRK_SHA8_OPERANDS
                 : KRK_SHA8_CONSTS, [w1] "v"(a[3]), [w2] "v"(b[0]), [w3] "v"(b[1]), [w4] "v"(b[2]),
                   [w5] "v"(b[3]), [w6] "v"(d[0]), [w7] "v"(d[1]), [w8] "v"(d[2]), [w9] "v"(d[3]),
                   [w10] "v"(e[0]), [w11] "v"(e[1]), [w12] "v"(e[2]));
}

// Eight lanes a stream, blocks pipelined: the A quad runs rounds 62, 63 of block i
// while the E quad already runs rounds 0, 1 of block i + 1, so a block costs 64
// instruction-rounds instead of 66.  State crosses blocks in registers: R0..R3 (the
// history, same register roles as rounds2), z, and each half's chaining value hE
// (E quads: H4..H7, 0 on A lanes) / hA (A quads: H2, H3, H0, H1, 0 on E lanes) --
// masked to its own quad so that one unmasked add feeds one half forward and adds 0
// to the other.  Per block (instruction-rounds n = 2 .. 65 of block i):
//   n = 2 .. 63: both halves (E round n, A round n - 2);
//   F1 (E finished block i): R += hE (E's feed-forward); E's round 0 of block i + 1
//      reads d through the cross add as A's raw a61, so its z also takes the A
//      half's H3 (partner's hA[1], via DPP) and the feed-forward of h (hE[3]); A's
//      rounds 62, 63 read e63, e64 through the cross add from registers E has just
//      fed forward, so A's z gives back H5 now and H4 after n = 64;
//      hE <- R where i < this stream's block count;
//   n = 64: E round 0 of block i + 1 (W = its KW0 .. KW1), A round 62;
//   F2: E's round 1 reads raw a62 as d: z += partner's hA[0] (H2); A: z -= H4
//      (both in one register cc formed in F1);
//   n = 65: E round 1, A round 63;
//   F3 (A finished block i): A's round 0 of block i + 1 takes -d from z formed on raw
//      a61: z -= hA[1]; R += hA; hA <- R where i < the block count.
// A finished stream's lanes keep computing on garbage; their hE / hA stay frozen.
__device__ __forceinline__ void block8p(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                        uint32_t hE[4], uint32_t hA[4], uint32_t mineE, uint32_t mineA,
                                        uint32_t i, const uint32_t* lds, uint32_t cbase, uint32_t nbase,
                                        const TwoLaneConst& c, u32x4 k[kAhead8]) {
    constexpr int kRS = kAhead8 + 1;
    u32x4 wq[kRS];
#pragma unroll
    for (int j = 0; j < kAhead8; ++j) wq[j] = k[j];
    // Rounds n = 2 .. 61: 5 asm blocks of twelve rounds,
    // the next three W quads read before each (four quads ahead), so one s_waitcnt per
    // twelve rounds.  Otherwise 15 asm blocks of four, n = 4j + 2 .. 4j + 5 (W: quad j's
    // last word, quad j + 1's first three), each W read between two blocks -- two rounds
    // into a W quad (issued right before a W quad's rounds a read cost ~16 cycles of the
    // wave's stream, two rounds in ~8, tools/micro/sha8lds.hip); the read + its wait
    // between two asm blocks are the two wait states the hazard recognizer would pad.
    constexpr int RS = kAhead8 + 3;
    u32x4 wr[RS];
#pragma unroll
    for (int j = 0; j < kAhead8; ++j) wr[j] = wq[j];
    auto rd = [&](int q) {  // W quad q of this block (q < 16) or q - 16 of the next block
        if (q < 16) wr[q % RS] = *reinterpret_cast<const u32x4*>(lds + cbase + 256 * q);
        else k[q - 16] = *reinterpret_cast<const u32x4*>(lds + nbase + 256 * (q - 16));
    };
#pragma unroll
    for (int j = 0; j < 15; j += 3) {
        rd(j + kAhead8);
        rd(j + kAhead8 + 1);
        rd(j + kAhead8 + 2);
        sha8_dodec2(R0, R1, R2, R3, z, c, wr[j % RS], wr[(j + 1) % RS], wr[(j + 2) % RS], wr[(j + 3) % RS]);
    }
    wq[15 % kRS] = wr[15 % RS];
    k[kAhead8 - 1] = *reinterpret_cast<const u32x4*>(lds + nbase + 256 * (kAhead8 - 1));
    {
        uint32_t t1, t2, kk, p;  // n = 62, 63
        asm volatile(KRK_SHA8_ROUND(R2, R1, R0, R3, w3)
                     KRK_SHA8_ROUND(R3, R2, R1, R0, w4)
                     KRK_SHA8_OPERANDS
                     : KRK_SHA8_CONSTS, [w3] "v"(wq[15 % kRS][3]), [w4] "v"(k[0][0]));
    }
    {
        // F1, n = 64, F2, n = 65, F3.  The cross terms go through one DPP each: every
        // lane forms hA - hE of its own (E lanes: -hE, A lanes: hA) and reads its
        // partner's, so E picks up the A half's H2 / H3 and A gives back E's H4 / H5.
        // (v_subrev_u32_dpp swizzles its second operand on gfx950, tools/micro/dppsem.hip,
        // so it is not used.)  Every VGPR a DPP instruction reads is written at least two
        // instructions earlier.
        uint32_t t1, t2, kk, p, cc, dd, c2;
        asm volatile("v_sub_u32_e32 %[cc], %[a0], %[e0]\n\t"   // own hA0 - hE0
                     "v_sub_u32_e32 %[dd], %[a1], %[e1]\n\t"   // own hA1 - hE1
                     "v_add_u32_e32 %[R0], %[e0], %[R0]\n\t"
                     "v_add_u32_e32 %[R3], %[e1], %[R3]\n\t"
                     "v_mov_b32_dpp %[c2], %[cc] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"  // E: H2 of A, A: -H4
                     "v_add_u32_dpp %[z], %[dd], %[z] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"  // E: +H3 of A, A: -H5
                     "v_add_u32_e32 %[R2], %[e2], %[R2]\n\t"
                     "v_add_u32_e32 %[R1], %[e3], %[R1]\n\t"
                     "v_add_u32_e32 %[z], %[e3], %[z]\n\t"
                     "v_cmp_lt_u32_e32 vcc, %[i], %[mineE]\n\t"
                     "v_cndmask_b32_e32 %[e0], %[e0], %[R0], vcc\n\t"
                     "v_cndmask_b32_e32 %[e1], %[e1], %[R3], vcc\n\t"
                     "v_cndmask_b32_e32 %[e2], %[e2], %[R2], vcc\n\t"
                     "v_cndmask_b32_e32 %[e3], %[e3], %[R1], vcc\n\t"
                     KRK_SHA8_ROUND(R0, R3, R2, R1, w1)
                     "v_add_u32_e32 %[z], %[c2], %[z]\n\t"
                     KRK_SHA8_ROUND(R1, R0, R3, R2, w2)
                     "v_sub_u32_e32 %[z], %[z], %[a1]\n\t"
                     "v_add_u32_e32 %[R0], %[a0], %[R0]\n\t"
                     "v_add_u32_e32 %[R3], %[a1], %[R3]\n\t"
                     "v_add_u32_e32 %[R2], %[a2], %[R2]\n\t"
                     "v_add_u32_e32 %[R1], %[a3], %[R1]\n\t"
                     "v_cmp_lt_u32_e32 vcc, %[i], %[mineA]\n\t"
                     "v_cndmask_b32_e32 %[a0], %[a0], %[R0], vcc\n\t"
                     "v_cndmask_b32_e32 %[a1], %[a1], %[R3], vcc\n\t"
                     "v_cndmask_b32_e32 %[a2], %[a2], %[R2], vcc\n\t"
                     "v_cndmask_b32_e32 %[a3], %[a3], %[R1], vcc\n\t"
                     : [t1] "=&v"(t1), [t2] "=&v"(t2), [k] "=&v"(kk), [p] "=&v"(p), [cc] "=&v"(cc), [dd] "=&v"(dd),
                       [c2] "=&v"(c2), [z] "+v"(z),
                       [R0] "+v"(R0), [R1] "+v"(R1), [R2] "+v"(R2), [R3] "+v"(R3), [e0] "+v"(hE[0]),
                       [e1] "+v"(hE[1]), [e2] "+v"(hE[2]), [e3] "+v"(hE[3]), [a0] "+v"(hA[0]), [a1] "+v"(hA[1]),
                       [a2] "+v"(hA[2]), [a3] "+v"(hA[3])
                     : KRK_SHA8_CONSTS, [w1] "v"(k[0][1]), [w2] "v"(k[0][2]), [i] "s"(i), [mineE] "v"(mineE),
                       [mineA] "v"(mineA)
                     : "vcc");
    }
}

// Instruction-rounds 0, 1 of a stream's first block (E rounds 0, 1; A idles and its
// two results are replaced by H1, H0: rounds2's start).
__device__ __forceinline__ void prologue8p(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                           const uint32_t h[4], bool is_e, const TwoLaneConst& c,
                                           const u32x4& k0) {
    {
        uint32_t t1, t2, kk, p;
        asm volatile("v_xad_u32 %[z], %[R1], %[ma], %[w0]\n\t"
                     KRK_SHA8_ROUND(R0, R3, R2, R1, w1)
                     KRK_SHA8_OPERANDS
                     : KRK_SHA8_CONSTS, [w0] "v"(k0[0]), [w1] "v"(k0[1]));
    }
    R1 = is_e ? R1 : h[3];
    {
        uint32_t t1, t2, kk, p;
        asm volatile(KRK_SHA8_ROUND(R1, R0, R3, R2, w2)
                     KRK_SHA8_OPERANDS
                     : KRK_SHA8_CONSTS, [w2] "v"(k0[2]));
    }
    R2 = is_e ? R2 : h[2];
}
// Two-lane counterparts (block2p, sha2_quad2, prologue2p): the same pipelined block on
// the two-lane round (KRK_SHA2_ROUND, partner lane by row_mirror), 64 instruction-rounds
// a block instead of rounds2's 66.  The two-lane round opens with its DPP add, so the
// F2 compensation of z is folded into round 64's W operand (w1 + c2) instead of being
// added between rounds 64 and 65.
// Rounds n = 4j + 2 .. 4j + 5 of a two-lane block (block2p), the register roles of
// instruction-rounds 2 .. 5: W operands are W[n + 1] for the z of the next round.
__device__ __forceinline__ void sha2_quad2(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                           const TwoLaneConst& c, uint32_t w1, uint32_t w2, uint32_t w3,
                                           uint32_t w4) {
    uint32_t t1, t2, t3, kk, p;
    asm volatile(KRK_SHA2_ROUND(R2, R1, R0, R3, w1) KRK_SHA2_ROUND(R3, R2, R1, R0, w2)
                 KRK_SHA2_ROUND(R0, R3, R2, R1, w3) KRK_SHA2_ROUND(R1, R0, R3, R2, w4)
                 KRK_SHA2_OPERANDS
                 : KRK_SHA2_CONSTS, [w1] "v"(w1), [w2] "v"(w2), [w3] "v"(w3), [w4] "v"(w4));
}

// The two-lane consumer's W read groups: as the eight-lane consumer's (three quads read
// four ahead, twelve rounds a wait) instead of one read and one wait per four rounds.  Same-box A/B (profiles/r02/sha2_read_groups.jsonl): 16,384
// streams 49.7 -> 51.6 MB/s a stream, 8,192 streams 50.4 -> 51.9 (pairs were 0.5 % slower
// than one read a quad).
constexpr int kAhead2 = 4;
__device__ __forceinline__ void sha2_dodec2(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                            const TwoLaneConst& c, const u32x4& a, const u32x4& b, const u32x4& d,
                                            const u32x4& e) {
    uint32_t t1, t2, t3, kk, p;
    asm volatile(KRK_SHA2_ROUND(R2, R1, R0, R3, w1) KRK_SHA2_ROUND(R3, R2, R1, R0, w2)
                 KRK_SHA2_ROUND(R0, R3, R2, R1, w3) KRK_SHA2_ROUND(R1, R0, R3, R2, w4)
                 KRK_SHA2_ROUND(R2, R1, R0, R3, w5) KRK_SHA2_ROUND(R3, R2, R1, R0, w6)
                 KRK_SHA2_ROUND(R0, R3, R2, R1, w7) KRK_SHA2_ROUND(R1, R0, R3, R2, w8)
                 KRK_SHA2_ROUND(R2, R1, R0, R3, w9) KRK_SHA2_ROUND(R3, R2, R1, R0, w10)
                 KRK_SHA2_ROUND(R0, R3, R2, R1, w11) KRK_SHA2_ROUND(R1, R0, R3, R2, w12)
                 KRK_SHA2_OPERANDS
                 : KRK_SHA2_CONSTS, [w1] "v"(a[3]), [w2] "v"(b[0]), [w3] "v"(b[1]), [w4] "v"(b[2]),
                   [w5] "v"(b[3]), [w6] "v"(d[0]), [w7] "v"(d[1]), [w8] "v"(d[2]), [w9] "v"(d[3]),
                   [w10] "v"(e[0]), [w11] "v"(e[1]), [w12] "v"(e[2]));
    (void)t3;
}


// Eight lanes a stream, blocks pipelined: the A quad runs rounds 62, 63 of block i
// while the E quad already runs rounds 0, 1 of block i + 1, so a block costs 64
// instruction-rounds instead of 66.  State crosses blocks in registers: R0..R3 (the
// history, same register roles as rounds2), z, and each half's chaining value hE
// (E quads: H4..H7, 0 on A lanes) / hA (A quads: H2, H3, H0, H1, 0 on E lanes) --
// masked to its own quad so that one unmasked add feeds one half forward and adds 0
// to the other.  Per block (instruction-rounds n = 2 .. 65 of block i):
//   n = 2 .. 63: both halves (E round n, A round n - 2);
//   F1 (E finished block i): R += hE (E's feed-forward); E's round 0 of block i + 1
//      reads d through the cross add as A's raw a61, so its z also takes the A
//      half's H3 (partner's hA[1], via DPP) and the feed-forward of h (hE[3]); A's
//      rounds 62, 63 read e63, e64 through the cross add from registers E has just
//      fed forward, so A's z gives back H5 now and H4 after n = 64;
//      hE <- R where i < this stream's block count;
//   n = 64: E round 0 of block i + 1 (W = its KW0 .. KW1), A round 62;
//   F2: E's round 1 reads raw a62 as d: z += partner's hA[0] (H2); A: z -= H4
//      (both in one register cc formed in F1);
//   n = 65: E round 1, A round 63;
//   F3 (A finished block i): A's round 0 of block i + 1 takes -d from z formed on raw
//      a61: z -= hA[1]; R += hA; hA <- R where i < the block count.
// A finished stream's lanes keep computing on garbage; their hE / hA stay frozen.
__device__ __forceinline__ void block2p(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                        uint32_t hE[4], uint32_t hA[4], uint32_t mineE, uint32_t mineA,
                                        uint32_t i, const uint32_t* lds, uint32_t cbase, uint32_t nbase,
                                        const TwoLaneConst& c, u32x4 k[kAhead2]) {
    constexpr int kRS = kAhead2 + 1;
    u32x4 wq[kRS];
#pragma unroll
    for (int j = 0; j < kAhead2; ++j) wq[j] = k[j];
    // Rounds n = 2 .. 61 in 15 asm blocks of four, n = 4j + 2 .. 4j + 5 (W: quad j's last
    // word, quad j + 1's first three), each W read between two blocks -- two rounds into
    // a W quad.  Issued right before a W quad's rounds a read cost ~16 cycles of the
    // wave's stream, two rounds in ~8, its code bytes (tools/micro/sha8lds.hip,
    // profiles/r02/micro_sha8lds.txt); and the read + its wait between two asm blocks
    // are the two wait states the hazard recognizer would otherwise pad there.
    constexpr int RS = kAhead2 + 3;
    u32x4 wr[RS];
#pragma unroll
    for (int j = 0; j < kAhead2; ++j) wr[j] = wq[j];
    auto rd = [&](int q) {  // W quad q of this block (q < 16) or q - 16 of the next block
        if (q < 16) wr[q % RS] = *reinterpret_cast<const u32x4*>(lds + cbase + 256 * q);
        else k[q - 16] = *reinterpret_cast<const u32x4*>(lds + nbase + 256 * (q - 16));
    };
#pragma unroll
    for (int j = 0; j < 15; j += 3) {
        rd(j + kAhead2);
        rd(j + kAhead2 + 1);
        rd(j + kAhead2 + 2);
        sha2_dodec2(R0, R1, R2, R3, z, c, wr[j % RS], wr[(j + 1) % RS], wr[(j + 2) % RS], wr[(j + 3) % RS]);
    }
    wq[15 % kRS] = wr[15 % RS];
    k[kAhead2 - 1] = *reinterpret_cast<const u32x4*>(lds + nbase + 256 * (kAhead2 - 1));
    {
        uint32_t t1, t2, t3, kk, p;  // n = 62, 63
        asm volatile(KRK_SHA2_ROUND(R2, R1, R0, R3, w3)
                     KRK_SHA2_ROUND(R3, R2, R1, R0, w4)
                     KRK_SHA2_OPERANDS
                     : KRK_SHA2_CONSTS, [w3] "v"(wq[15 % kRS][3]), [w4] "v"(k[0][0]));
    }
    {
        // F1, n = 64, F2, n = 65, F3.  The cross terms go through one DPP each: every
        // lane forms hA - hE of its own (E lanes: -hE, A lanes: hA) and reads its
        // partner's, so E picks up the A half's H2 / H3 and A gives back E's H4 / H5.
        // (v_subrev_u32_dpp swizzles its second operand on gfx950, tools/micro/dppsem.hip,
        // so it is not used.)  Every VGPR a DPP instruction reads is written at least two
        // instructions earlier.
        uint32_t t1, t2, t3, kk, p, cc, dd, c2, w1c;
        asm volatile("v_sub_u32_e32 %[cc], %[a0], %[e0]\n\t"   // own hA0 - hE0
                     "v_sub_u32_e32 %[dd], %[a1], %[e1]\n\t"   // own hA1 - hE1
                     "v_add_u32_e32 %[R0], %[e0], %[R0]\n\t"
                     "v_add_u32_e32 %[R3], %[e1], %[R3]\n\t"
                     "v_mov_b32_dpp %[c2], %[cc] row_mirror row_mask:0xf bank_mask:0xf\n\t"  // E: H2 of A, A: -H4
                     "v_add_u32_dpp %[z], %[dd], %[z] row_mirror row_mask:0xf bank_mask:0xf\n\t"  // E: +H3 of A, A: -H5
                     "v_add_u32_e32 %[R2], %[e2], %[R2]\n\t"
                     "v_add_u32_e32 %[R1], %[e3], %[R1]\n\t"
                     "v_add_u32_e32 %[z], %[e3], %[z]\n\t"
                     "v_cmp_lt_u32_e32 vcc, %[i], %[mineE]\n\t"
                     "v_cndmask_b32_e32 %[e0], %[e0], %[R0], vcc\n\t"
                     "v_cndmask_b32_e32 %[e1], %[e1], %[R3], vcc\n\t"
                     "v_cndmask_b32_e32 %[e2], %[e2], %[R2], vcc\n\t"
                     "v_cndmask_b32_e32 %[e3], %[e3], %[R1], vcc\n\t"
                     "v_add_u32_e32 %[w1c], %[c2], %[w1]\n\t"  // F2 folded into round 64's W
                     KRK_SHA2_ROUND(R0, R3, R2, R1, w1c)
                     KRK_SHA2_ROUND(R1, R0, R3, R2, w2)
                     "v_sub_u32_e32 %[z], %[z], %[a1]\n\t"
                     "v_add_u32_e32 %[R0], %[a0], %[R0]\n\t"
                     "v_add_u32_e32 %[R3], %[a1], %[R3]\n\t"
                     "v_add_u32_e32 %[R2], %[a2], %[R2]\n\t"
                     "v_add_u32_e32 %[R1], %[a3], %[R1]\n\t"
                     "v_cmp_lt_u32_e32 vcc, %[i], %[mineA]\n\t"
                     "v_cndmask_b32_e32 %[a0], %[a0], %[R0], vcc\n\t"
                     "v_cndmask_b32_e32 %[a1], %[a1], %[R3], vcc\n\t"
                     "v_cndmask_b32_e32 %[a2], %[a2], %[R2], vcc\n\t"
                     "v_cndmask_b32_e32 %[a3], %[a3], %[R1], vcc\n\t"
                     : [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [k] "=&v"(kk), [p] "=&v"(p), [cc] "=&v"(cc),
                       [dd] "=&v"(dd), [c2] "=&v"(c2), [w1c] "=&v"(w1c), [z] "+v"(z),
                       [R0] "+v"(R0), [R1] "+v"(R1), [R2] "+v"(R2), [R3] "+v"(R3), [e0] "+v"(hE[0]),
                       [e1] "+v"(hE[1]), [e2] "+v"(hE[2]), [e3] "+v"(hE[3]), [a0] "+v"(hA[0]), [a1] "+v"(hA[1]),
                       [a2] "+v"(hA[2]), [a3] "+v"(hA[3])
                     : KRK_SHA2_CONSTS, [w1] "v"(k[0][1]), [w2] "v"(k[0][2]), [i] "s"(i), [mineE] "v"(mineE),
                       [mineA] "v"(mineA)
                     : "vcc");
    }
}

// Instruction-rounds 0, 1 of a stream's first block (E rounds 0, 1; A idles and its
// two results are replaced by H1, H0: rounds2's start).
__device__ __forceinline__ void prologue2p(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                           const uint32_t h[4], bool is_e, const TwoLaneConst& c,
                                           const u32x4& k0) {
    {
        uint32_t t1, t2, t3, kk, p;
        asm volatile("s_nop 0\n\t"
                     "v_xad_u32 %[z], %[R1], %[ma], %[w0]\n\t"
                     KRK_SHA2_ROUND(R0, R3, R2, R1, w1)
                     KRK_SHA2_OPERANDS
                     : KRK_SHA2_CONSTS, [w0] "v"(k0[0]), [w1] "v"(k0[1]));
    }
    R1 = is_e ? R1 : h[3];
    {
        uint32_t t1, t2, t3, kk, p;
        asm volatile(KRK_SHA2_ROUND(R1, R0, R3, R2, w2)
                     KRK_SHA2_OPERANDS
                     : KRK_SHA2_CONSTS, [w2] "v"(k0[2]));
    }
    R2 = is_e ? R2 : h[2];
}
#undef KRK_SHA2_OPERANDS
#undef KRK_SHA2_CONSTS
#undef KRK_SHA8_OPERANDS
#undef KRK_SHA8_CONSTS

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, off, 64));
    return __builtin_amdgcn_readfirstlane(v);
}

// kTiming (diagnostic variant 2 only, wrong digests): the producer idles and the
// consumer runs its rounds on whatever the ring holds with no barriers -- the
// consumer's issue-bound time per block, to price the producer/consumer sync.
// kTwo: two lanes per stream (32 streams per workgroup, rounds2); the producer
// is unchanged -- both lanes of a stream build the same schedule into their own
// LDS column.
// kTiming 2 (diagnostic variants 5/6, wrong digests): the consumer exits at once and
// the producer runs alone (its barriers then count only itself) -- the producer's
// time per block.
//
// kTwo: the producer's A and E lanes of a stream build two different blocks per
// step (even and odd), so the producer's 64 lanes all do distinct work: built one
// block a step, it (47.6 MB/s a stream) could not keep up with the two-lane
// consumer (50 MB/s a stream).
//
// kGroups = 2: two producer/consumer pairs in one 4-wave workgroup, each with its own
// ring (128 KiB): the hardware puts the four waves of a workgroup on the four SIMDs
// of one CU, where two 2-wave workgroups sharing a CU also share SIMDs (47.9 vs 37.3
// MB/s a stream with two lanes).  The pairs share the workgroup barrier, so both run
// the workgroup's largest block count (jobs arrive sorted by length).
template <int kTiming, bool kTwo, int kGroups = 1>
__global__ void __launch_bounds__(128 * kGroups)
sha256_ws_kernel(const ShaJob* __restrict__ jobs, uint32_t n_jobs, uint8_t* __restrict__ out_digest,
                 uint32_t* __restrict__ out_state) {
    extern __shared__ __attribute__((aligned(16))) uint32_t ring_all[];
    constexpr int kNs = kTwo ? kSlots2 : kSlots;
    constexpr int kStep = kTwo ? 2 : 1;
    constexpr uint32_t kPer = kTwo ? 32u : 64u;  // streams per producer/consumer pair
    constexpr uint32_t kRingWords = uint32_t(kTwo ? kRing2 + 1 : kSlots) * kSlotWords;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const bool producer = wave < (uint32_t)kGroups;
    const uint32_t grp = wave % kGroups;
    uint32_t* ring = ring_all + grp * kRingWords;
    const uint32_t sbase = blockIdx.x * kPer * kGroups;
    const uint32_t me = kTwo ? two_lane_stream(lane) : lane;
    const uint32_t j = sbase + grp * kPer + me;
    const bool live = j < n_jobs;
    ShaJob job{};
    if (live) job = jobs[j];
    const uint32_t mine = live ? job_blocks(job) : 0u;
    // workgroup-uniform block count (every wave passes the same barriers)
    uint32_t nb = 0;
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
        const uint32_t jj = sbase + g * kPer + me;
        if (jj < n_jobs) nb = max(nb, g == (int)grp ? mine : job_blocks(jobs[jj]));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nb = max(nb, (uint32_t)__shfl_xor((int)nb, off, 64));
    nb = __builtin_amdgcn_readfirstlane(nb);

    if (producer && kTiming == 1) return;
    if (!producer && kTiming >= 2) return;
    if (producer) {
        // Two lanes per stream: the A lanes read W from the extra slot kRing2, all 1s
        // (rounds2).
        if (kTwo) {
#pragma unroll
            for (int q = 0; q < 16; ++q)
                *reinterpret_cast<u32x4*>(ring + kw_index(kRing2, q, lane)) = u32x4{1u, 1u, 1u, 1u};
        }
        // Loads are issued two steps ahead into a 3-deep register rotation (R0, R1, R2).
        u32x4 R0[kRaw], R1[kRaw], R2[kRaw];
        const uint64_t safe = reinterpret_cast<uint64_t>(jobs);
        const uint32_t par = kTwo && two_lane_is_e(lane) ? 1u : 0u;  // E lanes: odd blocks
        const uint32_t col = lane;                                    // each lane writes its own column
        uint32_t passed = 0;
        fetch(job, par, R0, safe);
        fetch(job, par + kStep, R1, safe);
        for (uint32_t b = 0; b < nb; b += 3 * kStep) {
            produce_step<kNs, kStep, kTiming == 3>(job, b, b + par, nb, col, ring, R0, R2, safe, passed);
            produce_step<kNs, kStep, kTiming == 3>(job, b + kStep, b + kStep + par, nb, col, ring, R1, R0, safe,
                                                   passed);
            produce_step<kNs, kStep, kTiming == 3>(job, b + 2 * kStep, b + 2 * kStep + par, nb, col, ring, R2, R1,
                                                   safe, passed);
        }
        // The consumer passes one barrier per step.
        while (passed < (nb + kStep - 1) / kStep) {
            __syncthreads();
            ++passed;
        }
    } else if (kTwo) {
        const bool is_e = two_lane_is_e(lane);
        const uint32_t half = is_e ? 4u : 0u;
        const TwoLaneConst c{is_e ? 6u : 2u, is_e ? 11u : 13u, is_e ? 25u : 22u, is_e ? 0u : ~0u, is_e ? 0u : 1u};
        // h[k] = H[4 + k] on E lanes, H[k ^ 2] on A lanes (rounds2's register order).
        uint32_t h[4];
        if (live && (job.flags & kShaFromState)) {
#pragma unroll
            for (int k = 0; k < 4; ++k) h[k] = out_state[8 * (uint64_t)job.out + half + (is_e ? k : k ^ 2)];
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) h[k] = is_e ? job.h[4 + k] : job.h[k ^ 2];  // no dynamic index: keeps job out of scratch
        }
        __builtin_amdgcn_s_setprio(3);
        // Blocks every live lane still needs (wave-uniform): no per-lane masking there.
        const uint32_t common = wave_min(live ? mine : ~0u);
        // kw2_base without the per-block slot arithmetic: the loop runs one producer
        // step (an even and an odd block, one slot) per iteration; vslot = the E
        // lanes' slot offset (the A lanes always read the all-1 slot, vslot = 0).
        const uint32_t aoff = is_e ? 0u : uint32_t(kRing2) * kSlotWords;
        const uint32_t base_even = aoff + (lane ^ 15u) * 4, base_odd = aoff + lane * 4;
        const uint32_t einc = is_e ? uint32_t(kSlotWords) : 0u;
        uint32_t vslot = 0, slot = 0;
        u32x4 kq[kAhead2] = {};
        // Blocks pipelined (block2p): 64 instruction-rounds a block, each half's chaining
        // value on its own lanes (0 on the other half).
        uint32_t hE[4], hA[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            hE[k] = is_e ? h[k] : 0u;
            hA[k] = is_e ? 0u : h[k];
        }
        const uint32_t mineE = is_e ? mine : 0u, mineA = is_e ? 0u : mine;
        uint32_t R0 = h[0], R3 = h[1], R2 = h[2], R1 = h[3], z = 0;
        (void)common;
        auto block = [&](uint32_t i, uint32_t cur, uint32_t nxt) {
            block2p(R0, R1, R2, R3, z, hE, hA, mineE, mineA, i, ring, cur, nxt, c, kq);
        };
        if (nb) {  // step 0's barrier, the first quads, and (pipelined) rounds 0, 1 of block 0
            if (kTiming == 0) __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
#pragma unroll
            for (int q = 0; q < kAhead2; ++q) kq[q] = *reinterpret_cast<const u32x4*>(ring + base_even + 256 * q);
            prologue2p(R0, R1, R2, R3, z, h, is_e, c, kq[0]);
        }
        for (uint32_t i = 0; i < nb; i += 2) {
            if (i) {
                if (kTiming == 0) __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
            }
            const uint32_t nslot = slot == kRing2 - 1 ? 0u : slot + 1;
            const uint32_t nvslot = slot == kRing2 - 1 ? 0u : vslot + einc;
            block(i, base_even + vslot, base_odd + vslot);
            if (i + 1 < nb) block(i + 1, base_odd + vslot, base_even + nvslot);
            slot = nslot;
            vslot = nvslot;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) h[k] = is_e ? hE[k] : hA[k];
        if (live) {
            uint32_t hs[4];  // back to H order (A lanes hold H[k ^ 2] in h[k])
#pragma unroll
            for (int k = 0; k < 4; ++k) hs[k] = is_e ? h[k] : h[k ^ 2];
            if (job.flags & kShaFinal) {
                uint8_t* o = out_digest + 32 * (uint64_t)job.out + 4 * half;
                if ((reinterpret_cast<uintptr_t>(o) & 15) == 0) {
                    reinterpret_cast<uint4*>(o)[0] =
                        make_uint4(bswap(hs[0]), bswap(hs[1]), bswap(hs[2]), bswap(hs[3]));
                } else {
                    for (int k = 0; k < 16; ++k) o[k] = (uint8_t)(hs[k >> 2] >> (24 - 8 * (k & 3)));
                }
            } else {
                uint32_t* o = out_state + 8 * (uint64_t)job.out + half;
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] = hs[k];
            }
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
        // The rounds are the long pole: win VALU issue arbitration should the
        // producer share this wave's SIMD.
        __builtin_amdgcn_s_setprio(3);
        // Blocks every live lane still needs (wave-uniform): no per-lane masking there.
        const uint32_t common = wave_min(live ? mine : ~0u);
        u32x4 k0{}, k1{};
        for (uint32_t i = 0; i < nb; ++i) {
            // The consumer writes no LDS, so its barrier needs no release fence (no
            // lgkmcnt drain): the quads prefetched below stay in flight across it.
            // Block i+1 is complete once this barrier has passed (the producer runs
            // kDepth-1 >= 1 blocks ahead of it), and its slot is not rewritten
            // before the barrier after next.
            if (kTiming == 0) __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (i == 0) {
                k0 = kw_quad(ring, 0, 0, lane);
                k1 = kw_quad(ring, 0, 1, lane);
            }
            uint32_t x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = h[k];
            rounds(x, ring, (int)(i % kSlots), lane, k0, k1);
            if (i + 1 < nb) {
                k0 = kw_quad(ring, (int)((i + 1) % kSlots), 0, lane);
                k1 = kw_quad(ring, (int)((i + 1) % kSlots), 1, lane);
            }
            if (i < common) {
#pragma unroll
                for (int k = 0; k < 8; ++k) h[k] = x[k];
            } else if (i < mine) {
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

// Eight lanes per stream (KRK_SHA8_ROUND above): a workgroup holds kGroups
// producer/consumer pairs over 8 streams each.  The producer's 64 lanes build 64
// different blocks per step -- lane p block b + p / 8 of stream p % 8 -- into its own
// column of the step's ring slot, so a step is 8 blocks a stream and the pair passes
// one barrier per 8 blocks (the producer runs 1/8 of the time it did with two lanes a
// stream, where a step was 2 blocks).  Ring: 3 slots of one step + the all-1 slot the
// A quads read W from, 64 KiB a pair.  The consumer's E quad of stream s reads block
// jj of a slot at column jj * 8 + s (every active lane of the quad the same address:
// an LDS broadcast), its A quad the all-1 slot.
// kTiming 1 (diagnostic build only, WRONG digests): the producer returns at once and
// the consumer runs its rounds on whatever the ring holds with no barriers -- the
// consumer's own time per block.
template <int kTiming, int kGroups>
__global__ void __launch_bounds__(128 * kGroups)
sha256_w8_kernel(const ShaJob* __restrict__ jobs, uint32_t n_jobs, uint8_t* __restrict__ out_digest,
                 uint32_t* __restrict__ out_state) {
    extern __shared__ __attribute__((aligned(16))) uint32_t ring_all[];
    constexpr int kStep8 = 8, kRing8 = 3, kNs = kStep8 * kRing8;
    constexpr uint32_t kPer = 8;  // streams per pair
    constexpr uint32_t kRingWords = uint32_t(kRing8 + 1) * kSlotWords + kOnesPad8;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const bool producer = wave < (uint32_t)kGroups;
    const uint32_t grp = wave % kGroups;
    uint32_t* ring = ring_all + grp * kRingWords;
    const uint32_t sbase = blockIdx.x * kPer * kGroups;
    const uint32_t quad = (lane >> 2) & 3;
    const uint32_t me = producer ? (lane & 7) : (lane >> 4) * 2 + (quad & 1);
    const uint32_t j = sbase + grp * kPer + me;
    const bool live = j < n_jobs;
    ShaJob job{};
    if (live) job = jobs[j];
    const uint32_t mine = live ? job_blocks(job) : 0u;
    uint32_t nb = 0;
#pragma unroll
    for (int g = 0; g < kGroups; ++g) {
        const uint32_t jj = sbase + g * kPer + me;
        if (jj < n_jobs) nb = max(nb, g == (int)grp ? mine : job_blocks(jobs[jj]));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nb = max(nb, (uint32_t)__shfl_xor((int)nb, off, 64));
    nb = __builtin_amdgcn_readfirstlane(nb);

    if (producer && kTiming == 1) return;
    if (producer) {
#pragma unroll
        for (int q = 0; q < 16; ++q) *reinterpret_cast<u32x4*>(ring + kw_index(kRing8, q, lane)) = u32x4{1u, 1u, 1u, 1u};
        *reinterpret_cast<u32x4*>(ring + (kRing8 + 1) * kSlotWords + lane * 4) = u32x4{1u, 1u, 1u, 1u};  // pad
        u32x4 R0[kRaw], R1[kRaw], R2[kRaw];
        const uint64_t safe = reinterpret_cast<uint64_t>(jobs);
        const uint32_t par = lane >> 3;  // this lane's block within a step
        uint32_t passed = 0;
        fetch(job, par, R0, safe);
        fetch(job, par + kStep8, R1, safe);
        for (uint32_t b = 0; b < nb; b += 3 * kStep8) {
            produce_step<kNs, kStep8>(job, b, b + par, nb, lane, ring, R0, R2, safe, passed);
            produce_step<kNs, kStep8>(job, b + kStep8, b + kStep8 + par, nb, lane, ring, R1, R0, safe, passed);
            produce_step<kNs, kStep8>(job, b + 2 * kStep8, b + 2 * kStep8 + par, nb, lane, ring, R2, R1, safe, passed);
        }
        while (passed < (nb + kStep8 - 1) / kStep8) {
            __syncthreads();
            ++passed;
        }
        return;
    }
    const bool is_e = quad < 2;
    const uint32_t pos = lane & 3;
    const uint32_t half = is_e ? 4u : 0u;
    // this lane's Sigma rotation: E quads Sigma1 (6, 11, 25), A quads Sigma0 (2, 13, 22)
    const uint32_t r1 = is_e ? (pos == 1 ? 11u : pos == 2 ? 25u : 6u) : (pos == 1 ? 13u : pos == 2 ? 22u : 2u);
    const TwoLaneConst c{r1, 0u, 0u, is_e ? 0u : ~0u, is_e ? 0u : 1u};
    uint32_t h[4];  // H[4 + k] on E lanes, H[k ^ 2] on A lanes (rounds2's register order)
    if (live && (job.flags & kShaFromState)) {
#pragma unroll
        for (int k = 0; k < 4; ++k) h[k] = out_state[8 * (uint64_t)job.out + half + (is_e ? k : k ^ 2)];
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) h[k] = is_e ? job.h[4 + k] : job.h[k ^ 2];
    }
    __builtin_amdgcn_s_setprio(3);
    // Word offsets: E lanes read block jj of ring slot sl at column jj * 8 + me, i.e.
    // lbase + sl * kSlotWords + jj * 32; A lanes always the all-1 slot.
    // A lanes: one broadcast address in the all-1 slot, column 8 (jj + 1), 32 banks
    // away from the E lanes' eight columns of the same block (the same banks at a
    // different address were a 2-way conflict on every read: 9 % of the LDS cycles).
    const uint32_t lbase = is_e ? me * 4u : uint32_t(kRing8) * kSlotWords + 32u;
    const uint32_t binc = 32u, sinc = is_e ? uint32_t(kSlotWords) : 0u;
    // voff: this lane's offset of block i (E: slot base vslot + jj * 32; A: 0)
    uint32_t voff = 0, vslot = 0, slot = 0;
    u32x4 kq[kAhead8] = {};
    // Blocks pipelined (block8p): 64 instruction-rounds a block; each half's chaining
    // value lives on its own lanes (0 on the other half).
    uint32_t hE[4], hA[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        hE[k] = is_e ? h[k] : 0u;
        hA[k] = is_e ? 0u : h[k];
    }
    const uint32_t mineE = is_e ? mine : 0u, mineA = is_e ? 0u : mine;
    uint32_t R0 = h[0], R3 = h[1], R2 = h[2], R1 = h[3], z = 0;
    auto block = [&](uint32_t i, uint32_t cur, uint32_t nxt) {
        block8p(R0, R1, R2, R3, z, hE, hA, mineE, mineA, i, ring, cur, nxt, c, kq);
    };
    // kU blocks an iteration (a step's 8 blocks never straddle an iteration): one block
    // an iteration ran at 52.9 MB/s a stream, two at 55.0 (fewer taken branches and
    // less loop bookkeeping per block); with the W read groups, four 59.1 vs two 58.8,
    // eight 59.1 (profiles/r02/sha8_unroll.jsonl).
    constexpr uint32_t kU = KRK_SHA8_UNROLL;
    static_assert(kU == 1 || kU == 2 || kU == 4 || kU == 8, "blocks per iteration divide a step");
    if (nb) {  // step 0's barrier, the first quads, and (pipelined) rounds 0, 1 of block 0
        if (kTiming == 0) __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#pragma unroll
        for (int q = 0; q < kAhead8; ++q) kq[q] = *reinterpret_cast<const u32x4*>(ring + lbase + 256 * q);
        prologue8p(R0, R1, R2, R3, z, h, is_e, c, kq[0]);
    }
    for (uint32_t i = 0; i < nb; i += kU) {
        const uint32_t jj = i & (kStep8 - 1);
        if (jj == 0 && i) {
            if (kTiming == 0) __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        }
        const bool last = jj == kStep8 - kU;
        const uint32_t nvslot = slot == kRing8 - 1 ? 0u : vslot + sinc;
        uint32_t o = voff;
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t on = (u == kU - 1 && last) ? nvslot : o + binc;
            if (u == 0 || i + u < nb) block(i + u, lbase + o, lbase + on);
            o = on;
        }
        voff = o;
        if (last) {
            slot = slot == kRing8 - 1 ? 0u : slot + 1;
            vslot = nvslot;
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) h[k] = is_e ? hE[k] : hA[k];
    if (live && pos == 0) {
        uint32_t hs[4];  // back to H order
#pragma unroll
        for (int k = 0; k < 4; ++k) hs[k] = is_e ? h[k] : h[k ^ 2];
        if (job.flags & kShaFinal) {
            uint8_t* o = out_digest + 32 * (uint64_t)job.out + 4 * half;
            if ((reinterpret_cast<uintptr_t>(o) & 15) == 0) {
                reinterpret_cast<uint4*>(o)[0] = make_uint4(bswap(hs[0]), bswap(hs[1]), bswap(hs[2]), bswap(hs[3]));
            } else {
                for (int k = 0; k < 16; ++k) o[k] = (uint8_t)(hs[k >> 2] >> (24 - 8 * (k & 3)));
            }
        } else {
            uint32_t* o = out_state + 8 * (uint64_t)job.out + half;
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = hs[k];
        }
    }
}

// Launch plans.  Production (every plan bit-exact):
//   KRK_SHA_PLAN_1LANE        one lane per stream, one producer/consumer pair per workgroup
//   KRK_SHA_PLAN_2LANE        two lanes per stream, one pair per workgroup
//   KRK_SHA_PLAN_1LANE_2PAIR  one lane, two pairs per 4-wave workgroup
//   KRK_SHA_PLAN_2LANE_2PAIR  two lanes, two pairs per workgroup
//   KRK_SHA_PLAN_8LANE        eight lanes per stream (sha256_w8_kernel), one pair per workgroup
//   KRK_SHA_PLAN_8LANE_2PAIR  eight lanes, two pairs per workgroup
//   KRK_SHA_PLAN_AUTO         auto_plan() below
// The plan is process-wide state set by krk_set_sha_plan (or KRK_SHA_PLAN read once,
// at the first launch); it is not re-read per launch.  The timing diagnostics
// (rounds-only consumer, producer-only, no-load producer: WRONG digests) and the
// one-lane-does-everything kernel exist only in the diagnostic build (make diag,
// -DKRK_DIAG), selected there with plan numbers 100 + the old variant number.
static std::atomic<int> g_sha_plan{-1};

static int sha_plan() {
    int p = g_sha_plan.load(std::memory_order_relaxed);
    if (p >= 0) return p;
    const char* e = KRK_AB_ENV("KRK_SHA_PLAN");  // krk_set_sha_plan is the run-time setter
    int want = e ? atoi(e) : KRK_SHA_PLAN_AUTO;
    if (!sha_plan_valid(want)) want = KRK_SHA_PLAN_AUTO;
    int expect = -1;
    g_sha_plan.compare_exchange_strong(expect, want);
    return g_sha_plan.load(std::memory_order_relaxed);
}

bool sha_plan_valid(int p) {
    if (p >= KRK_SHA_PLAN_AUTO && p <= KRK_SHA_PLAN_8LANE_2PAIR) return true;
#ifdef KRK_DIAG
    return p >= 100 && p <= 108;
#else
    return false;
#endif
}

void set_sha_plan(int p) { g_sha_plan.store(p, std::memory_order_relaxed); }

// Streams up to which two lanes per stream win: two two-lane workgroups (64 KiB of
// LDS each) per CU.  Measured (tools/probe_perf.py, profiles/r01/sha_compact_ring.jsonl):
// 8,192 streams 47.9 MB/s a stream two-lane vs 35.9 one-lane; 16,384 streams 37.3 vs
// 35.5 (two workgroups then share a CU's SIMDs).  Beyond that the two-lane grid would
// run in waves of workgroups.
static uint32_t device_cus() {
    static uint32_t n = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) {
            hipDeviceProp_t p;
            if (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0) cus = p.multiProcessorCount;
        }
        return (uint32_t)cus;
    }();
    return n;
}
static uint32_t two_lane_max_streams() { return device_cus() * 64u; }

// Automatic plan: eight lanes a stream up to 16 x CUs streams (two 64 KiB pairs per
// CU; at 4,096 streams 52.6 MB/s a stream vs 49.8 with two lanes, at 8,192 the
// eight-lane grid runs in two waves of workgroups and halves, tools/probe_perf.py);
// two lanes, one pair per workgroup up to 32 x CUs; two lanes, two pairs per
// workgroup up to 64 x CUs; one lane, two pairs per workgroup beyond.
static int auto_plan(uint32_t n_jobs) {
    if (n_jobs <= device_cus() * 16u) return KRK_SHA_PLAN_8LANE;
    if (n_jobs <= device_cus() * 32u) return KRK_SHA_PLAN_2LANE;
    return n_jobs <= two_lane_max_streams() ? KRK_SHA_PLAN_2LANE_2PAIR : KRK_SHA_PLAN_1LANE_2PAIR;
}

static int resolve_plan(uint32_t n_jobs) {
    const int p = sha_plan();
    return p == KRK_SHA_PLAN_AUTO ? auto_plan(n_jobs) : p;
}

static bool plan_two_lanes(int p) {
    return p == KRK_SHA_PLAN_2LANE || p == KRK_SHA_PLAN_2LANE_2PAIR || p == 103 || p == 104 || p == 106 ||
           p == 107;
}

static bool plan_eight_lanes(int p) { return p == KRK_SHA_PLAN_8LANE || p == KRK_SHA_PLAN_8LANE_2PAIR || p == 108; }

int sha_plan_for(uint32_t n_jobs) { return resolve_plan(n_jobs); }

int sha_lanes_for(uint32_t n_jobs) {
    const int p = resolve_plan(n_jobs);
    return plan_eight_lanes(p) ? 8 : plan_two_lanes(p) ? 2 : 1;
}

template <int kTiming, int kGroups>
static hipError_t launch_w8(const ShaJob* jobs, uint32_t n_jobs, uint8_t* out_digest, uint32_t* out_state,
                            hipStream_t s) {
    constexpr size_t lds = size_t(kGroups) * (4 * kSlotWords + kOnesPad8) * 4;  // 3 ring slots + the all-1 slot: 65 KiB a pair
    auto* k = &sha256_w8_kernel<kTiming, kGroups>;
    static std::once_flag once;
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [k] {
        attr_err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    });
    if (attr_err != hipSuccess) return attr_err;
    constexpr uint32_t per = 8u * kGroups;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(k, dim3((n_jobs + per - 1) / per), dim3(128 * kGroups), lds, s, jobs, n_jobs, out_digest,
                       out_state);
    return hipGetLastError();
}

template <int kTiming, bool kTwo, int kGroups>
static hipError_t launch_ws(const ShaJob* jobs, uint32_t n_jobs, uint8_t* out_digest, uint32_t* out_state,
                            hipStream_t s) {
    constexpr size_t lds = size_t(kGroups) * size_t(kTwo ? kRing2 + 1 : kSlots) * kSlotWords * 4;  // 64 KiB a pair
    auto* k = &sha256_ws_kernel<kTiming, kTwo, kGroups>;
    static std::once_flag once;  // host threads may launch concurrently (re-entrant C ABI)
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [k] {
        attr_err = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    });
    if (attr_err != hipSuccess) return attr_err;
    constexpr uint32_t per = (kTwo ? 32u : 64u) * kGroups;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(k, dim3((n_jobs + per - 1) / per), dim3(128 * kGroups), lds, s, jobs, n_jobs, out_digest,
                       out_state);
    return hipGetLastError();
}

hipError_t launch_sha256(const ShaJob* jobs, uint32_t n_jobs, uint8_t* out_digest,
                         uint32_t* out_state, hipStream_t s) {
    if (!n_jobs) return hipSuccess;
    return launch_sha256_plan(resolve_plan(n_jobs), jobs, n_jobs, out_digest, out_state, s);
}

hipError_t launch_sha256_plan(int plan, const ShaJob* jobs, uint32_t n_jobs, uint8_t* out_digest,
                              uint32_t* out_state, hipStream_t s) {
    if (!n_jobs) return hipSuccess;
    t_launch_plan = plan;
    t_launch_units = n_jobs;
    switch (plan) {
        case KRK_SHA_PLAN_1LANE: return launch_ws<0, false, 1>(jobs, n_jobs, out_digest, out_state, s);
        case KRK_SHA_PLAN_2LANE: return launch_ws<0, true, 1>(jobs, n_jobs, out_digest, out_state, s);
        case KRK_SHA_PLAN_1LANE_2PAIR: return launch_ws<0, false, 2>(jobs, n_jobs, out_digest, out_state, s);
        case KRK_SHA_PLAN_2LANE_2PAIR: return launch_ws<0, true, 2>(jobs, n_jobs, out_digest, out_state, s);
        case KRK_SHA_PLAN_8LANE: return launch_w8<0, 1>(jobs, n_jobs, out_digest, out_state, s);
        case KRK_SHA_PLAN_8LANE_2PAIR: return launch_w8<0, 2>(jobs, n_jobs, out_digest, out_state, s);
#ifdef KRK_DIAG
        // diagnostics (WRONG digests except 100): rounds-only consumer (102 one lane, 104 two
        // lanes), producer-only (105 / 106), producer without global loads (107)
        case 100:
            if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
            hipLaunchKernelGGL(sha256_multi_kernel, dim3((n_jobs + 63) / 64), dim3(64), 0, s, jobs, n_jobs,
                               out_digest, out_state);
            return hipGetLastError();
        case 101: return launch_ws<0, false, 1>(jobs, n_jobs, out_digest, out_state, s);
        case 102: return launch_ws<1, false, 1>(jobs, n_jobs, out_digest, out_state, s);
        case 103: return launch_ws<0, true, 1>(jobs, n_jobs, out_digest, out_state, s);
        case 104: return launch_ws<1, true, 1>(jobs, n_jobs, out_digest, out_state, s);
        case 105: return launch_ws<2, false, 1>(jobs, n_jobs, out_digest, out_state, s);
        case 106: return launch_ws<2, true, 1>(jobs, n_jobs, out_digest, out_state, s);
        case 107: return launch_ws<3, true, 1>(jobs, n_jobs, out_digest, out_state, s);
        case 108: return launch_w8<1, 1>(jobs, n_jobs, out_digest, out_state, s);  // eight-lane rounds only
#endif
        default: return hipErrorInvalidValue;
    }
}

// Host-offloaded digests into their batch slots (offload.cpp): record j = 4-byte blob
// index + 32-byte digest; one byte per thread (digests_dev has no alignment promise).
__global__ void __launch_bounds__(256) digest_scatter_kernel(const uint8_t* __restrict__ rec, uint32_t n,
                                                             uint8_t* __restrict__ digests) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n * 32) return;
    const uint8_t* r = rec + 36 * (t / 32);
    const uint32_t idx = (uint32_t)r[0] | ((uint32_t)r[1] << 8) | ((uint32_t)r[2] << 16) | ((uint32_t)r[3] << 24);
    digests[32ull * idx + t % 32] = r[4 + t % 32];
}

hipError_t launch_digest_scatter(const uint8_t* rec, uint32_t n, uint8_t* digests, hipStream_t s) {
    if (!n) return hipSuccess;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(digest_scatter_kernel, dim3((n * 32 + 255) / 256), dim3(256), 0, s, rec, n, digests);
    return hipGetLastError();
}

}  // namespace krk
