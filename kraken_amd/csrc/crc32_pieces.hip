// crc32_pieces.hip -- piece CRC-32/IEEE for gfx950 (core.calcPieceSums,
// core/metainfo.go:158-179; PieceHash = crc32.NewIEEE, core/piece_hash.go:22-24).
//
// Work: one wave per work item, a run of <= 256 KiB inside one piece.  One launch
// takes items from two sources (CrcWork): runs of whole pieces, expanded here on
// the device (a whole piece's items and constants depend only on the piece
// length), and explicit CrcItems built on the host (partial pieces, stream
// windows, seeded crc32.Update calls).
//
// Two lane layouts (CrcLaunchCfg.variant):
//  * strided (0, 1): a wave step covers 4 KiB; lane l owns the 64-byte segment
//    [step*4096 + 64l, +64), loaded as 4 x 16 B; one CRC chain per lane, and the
//    lane's virtual stream holds 4032 zero bytes between two of its segments.
//  * coalesced (2, 3): each 1 KiB quarter k of a step is ONE fully coalesced wave
//    load (lane l: bytes [1024k + 16l, +16)); lane l runs four independent chains,
//    one per quarter (ILP 4 on the LDS lookups), 4080 zero bytes apart.
// Each chain runs slicing-by-4 (1 LDS lookup per byte); a zero gap is one
// 4-lookup shift-table step.  At the end every chain is shifted to the item end
// (GF(2) multiply by a per-lane constant), the wave XOR-reduces, and lane 0 shifts
// to the piece end and atomically XORs into sums[piece].  XOR is order-free, so
// the items of one piece may run on any wave, XCD or launch.
//
// Tables live in LDS, replicated so that the lanes of a ds_read_b32 half-wave hit
// distinct banks.  Production (variants 7, 8): the byte-addressable layout of TabP,
// where a lookup address is one v_perm_b32.  The diagnostic build (KRK_DIAG) adds the
// measured alternatives: replicated R times and interleaved (word (t*256+e)*R + r,
// lane l reads replica l % R), the coalesced layout, nontemporal loads and load-only
// timing kernels.  DESIGN.md §4.1 has the measurements of every variant.
#include <mutex>

#include "kernels.hpp"
#include "crc_math.hpp"
#include "device_util.hpp"

namespace krk {

template <int R>
struct Tab {
    const uint32_t* lo;  // T0, T1 (and T2, T3 for R <= 16)
    const uint32_t* hi;  // T2 base for R == 32 (offset field is 16-bit)
    __device__ __forceinline__ uint32_t t(int k, uint32_t idx) const {
        if (R >= 32 && k >= 2) return hi[((k - 2) * 256 + idx) * R];
        return lo[(k * 256 + idx) * R];
    }
    // One slicing-by-4 word step: c' = raw(c ^ w, 4 bytes).
    __device__ __forceinline__ uint32_t word(uint32_t c) const {
        return xor3(t(3, c & 0xFF), t(2, (c >> 8) & 0xFF), t(1, (c >> 16) & 0xFF)) ^ t(0, c >> 24);
    }
    __device__ __forceinline__ uint32_t byte(uint32_t c, uint32_t b) const {
        return t(0, (c ^ b) & 0xFF) ^ (c >> 8);
    }
};

// Byte-addressable table layout (variants 7, 8): entry e of slicing table k,
// replica r = lane % RP, at LDS byte e*256 + (k % TPR)*RP*4 + r*4 + (k / TPR)*65536,
// TPR = 64 / RP tables per 256-byte row.  A lookup address is then ONE v_perm_b32
// (byte e -> bits 8-15, the lane's replica offset -> bits 0-7, the region bit from
// the selector) and the table's place in the row rides in the ds_read offset field,
// instead of extract + shift + add.  RP = 32 (128 KiB): bank = (address / 4) mod 32
// = r, the 32 lanes of a ds_read_b32 half-wave never conflict.  RP = 16 (64 KiB):
// lanes l and l + 16 share a bank (2-way), but two workgroups fit a CU.
typedef const __attribute__((address_space(3))) uint32_t* lds_u32p;

template <int RP>
struct TabP {
    static constexpr int TPR = 64 / RP;
    uint32_t loff;  // (1 << 16) | (lane % RP) * 4: byte 0 = replica offset, byte 2 = region 1
    // The tables start at LDS byte 0 (the kernel's only LDS is its dynamic array; checked
    // at kernel start), so the perm result is the ds_read address as it stands.
    __device__ __forceinline__ uint32_t at(uint32_t a, int off) const { return *(lds_u32p)(size_t)(a + off); }
    // byte0 <- loff.byte0, byte1 <- x.byte J, byte2 <- REGION ? loff.byte2 : 0, byte3 <- 0
    template <int J, int REGION>
    __device__ __forceinline__ uint32_t addr(uint32_t x) const {
        constexpr uint32_t sel = 0x0C000000u | ((REGION ? 0x02u : 0x0Cu) << 16) | ((4u + J) << 8);
        return __builtin_amdgcn_perm(x, loff, sel);
    }
    // table k looked up with byte J of x
    template <int J, int K>
    __device__ __forceinline__ uint32_t t(uint32_t x) const {
        return at(addr<J, (K / TPR)>(x), (K % TPR) * RP * 4);
    }
    // T3[byte 0] ^ T2[byte 1] ^ T1[byte 2] ^ T0[byte 3]
    __device__ __forceinline__ uint32_t word(uint32_t c) const {
        return xor3(t<0, 3>(c), t<1, 2>(c), t<2, 1>(c)) ^ t<3, 0>(c);
    }
    __device__ __forceinline__ uint32_t byte(uint32_t c, uint32_t b) const { return t<0, 0>(c ^ b) ^ (c >> 8); }
};

template <int RG>
__device__ __forceinline__ uint32_t gap_shift(uint32_t c, const uint32_t* G) {
    return xor3(G[(0 * 256 + (c & 0xFF)) * RG], G[(1 * 256 + ((c >> 8) & 0xFF)) * RG],
                G[(2 * 256 + ((c >> 16) & 0xFF)) * RG]) ^ G[(3 * 256 + (c >> 24)) * RG];
}

template <class TT>
__device__ __forceinline__ uint32_t seg16(uint32_t c, const u32x4& v, const TT& T) {
    c = T.word(c ^ v.x);
    c = T.word(c ^ v.y);
    c = T.word(c ^ v.z);
    c = T.word(c ^ v.w);
    return c;
}

// Up to 4 little-endian words holding n valid bytes (n <= 16) into register c.
template <class TT, int NW>
__device__ __forceinline__ uint32_t feed_words(uint32_t c, const uint32_t* w, uint32_t n, const TT& T) {
#pragma unroll
    for (int j = 0; j < NW; ++j) {
        const int keep = (int)n - 4 * j;
        if (keep >= 4) {
            c = T.word(c ^ w[j]);
        } else if (keep > 0) {
            for (int b = 0; b < keep; ++b) c = T.byte(c, (w[j] >> (8 * b)) & 0xFF);
        }
    }
    return c;
}

// ------------------------------------------------------------ strided layout
// One wave step for this lane: skip the 4032-byte gap, then its 64 own bytes.
template <class TT, int RG, bool LOADONLY = false>
__device__ __forceinline__ uint32_t step64(uint32_t c, const u32x4& v0, const u32x4& v1, const u32x4& v2,
                                           const u32x4& v3, const TT& T, const uint32_t* G) {
    if (LOADONLY)  // timing diagnostic (variant 4): the loads without the table work
        return c ^ xor3(v0.x ^ v0.y ^ v0.z ^ v0.w, v1.x ^ v1.y ^ v1.z ^ v1.w, v2.x ^ v2.y ^ v2.z ^ v2.w) ^ v3.x ^
               v3.y ^ v3.z ^ v3.w;
    c = gap_shift<RG>(c, G);
    c = seg16(c, v0, T);
    c = seg16(c, v1, T);
    c = seg16(c, v2, T);
    return seg16(c, v3, T);
}

// This lane's share of bytes [base, base+len), shifted to the item end.
// One 16-byte load; NT marks it nontemporal (global_load ... nt: the bytes are read
// once, so they need not displace anything in L2 / MALL).
template <bool NT>
__device__ __forceinline__ u32x4 ld16(gptr<u32x4> p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

typedef __attribute__((address_space(3))) uint32_t* lds_u32w;

// LDS-DMA ring of one wave (variant 20): step s's 4 KiB land in slot
// s & 1 by four global_load_lds_dwordx4 (1 KiB each; lane l's source is its own 16 bytes k of
// the step, so slot word [k][l] is what the register path loads into v_k of lane l and the
// consumer's ds_read_b128 are bank-conflict free); the next step's four are in flight while
// this one's lookups run.  NT: nontemporal (aux bit 1).
template <bool NT>
__device__ __forceinline__ void glds_issue(uint64_t src, lds_u32w slot) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
        __builtin_amdgcn_global_load_lds((const void*)(src + 16 * k), (__attribute__((address_space(3))) void*)(slot + 256 * k),
                                         16, 0, NT ? 2 : 0);
}

template <class TT, int RG, bool LOADONLY = false, bool NT = false, bool DEEP = false, int RING = 2>
__device__ __forceinline__ uint32_t lane_crc_strided(uint64_t base, uint32_t len, uint32_t lane, const TT& T,
                                                     const uint32_t* G, uint32_t lane_mul,
                                                     const uint32_t* x8pow, lds_u32w ring = nullptr) {
    uint32_t c = 0;
    uint32_t end = 0;  // end offset (in item) of this lane's last processed byte + 1
    const uint32_t nfull = len / kStep;
    if ((base & 15) == 0) {
        if (nfull > 0 && ring) {
            // RING - 1 steps in flight: steps s+1 .. s+RING-1 are loading while step s computes
            const uint64_t src = base + lane * kSeg;
            for (uint32_t k = 0; k + 1 < (uint32_t)RING && k < nfull; ++k)
                glds_issue<NT>(src + uint64_t(k) * kStep, ring + k * 1024);
            for (uint32_t s = 0; s < nfull; ++s) {
                const uint32_t nx = s + RING - 1;  // the step whose loads go out now
                if (nx < nfull) glds_issue<NT>(src + uint64_t(nx) * kStep, ring + (nx % RING) * 1024);
                // wait for step s: the loads issued after it may stay in flight
                const uint32_t after = min(nfull - 1, nx) - s;
                if (after >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
                else if (after == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                else if (after == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const __attribute__((address_space(3))) u32x4* q =
                    (const __attribute__((address_space(3))) u32x4*)(ring + (s % RING) * 1024) + lane;
                const u32x4 v0 = q[0], v1 = q[64], v2 = q[128], v3 = q[192];
                c = step64<TT, RG, LOADONLY>(c, v0, v1, v2, v3, T, G);
            }
            end = (nfull - 1) * kStep + (lane + 1) * kSeg;
        } else if (nfull > 0) {
            gptr<u32x4> p = as_global<u32x4>(base + lane * kSeg);
            constexpr uint32_t S = kStep / 16;
            if constexpr (DEEP) {
                // Three register sets in rotation: the loads of step s + 2 are in flight
                // while step s's lookups run (8 KiB a wave ahead instead of 4).
                u32x4 a0, a1, a2, a3, b0, b1, b2, b3, e0, e1, e2, e3;
                a0 = ld16<NT>(p); a1 = ld16<NT>(p + 1); a2 = ld16<NT>(p + 2); a3 = ld16<NT>(p + 3);
                if (nfull > 1) {
                    gptr<u32x4> q = p + S;
                    b0 = ld16<NT>(q); b1 = ld16<NT>(q + 1); b2 = ld16<NT>(q + 2); b3 = ld16<NT>(q + 3);
                }
                uint32_t s = 0;
                for (; s + 3 <= nfull; s += 3) {
                    gptr<u32x4> q = p + (s + 2) * S;
                    e0 = ld16<NT>(q); e1 = ld16<NT>(q + 1); e2 = ld16<NT>(q + 2); e3 = ld16<NT>(q + 3);
                    c = step64<TT, RG, LOADONLY>(c, a0, a1, a2, a3, T, G);
                    if (s + 3 < nfull) {
                        q = p + (s + 3) * S;
                        a0 = ld16<NT>(q); a1 = ld16<NT>(q + 1); a2 = ld16<NT>(q + 2); a3 = ld16<NT>(q + 3);
                    }
                    c = step64<TT, RG, LOADONLY>(c, b0, b1, b2, b3, T, G);
                    if (s + 4 < nfull) {
                        q = p + (s + 4) * S;
                        b0 = ld16<NT>(q); b1 = ld16<NT>(q + 1); b2 = ld16<NT>(q + 2); b3 = ld16<NT>(q + 3);
                    }
                    c = step64<TT, RG, LOADONLY>(c, e0, e1, e2, e3, T, G);
                }
                if (s < nfull) c = step64<TT, RG, LOADONLY>(c, a0, a1, a2, a3, T, G);
                if (s + 1 < nfull) c = step64<TT, RG, LOADONLY>(c, b0, b1, b2, b3, T, G);
            } else {
                // Two register sets in ping-pong: the next step's 4 x 16 B are in
                // flight while the current step's lookups run.
                u32x4 a0 = ld16<NT>(p), a1 = ld16<NT>(p + 1), a2 = ld16<NT>(p + 2), a3 = ld16<NT>(p + 3);
                u32x4 b0, b1, b2, b3;
                uint32_t s = 0;
                for (; s + 2 <= nfull; s += 2) {
                    gptr<u32x4> q = p + (s + 1) * S;
                    b0 = ld16<NT>(q); b1 = ld16<NT>(q + 1); b2 = ld16<NT>(q + 2); b3 = ld16<NT>(q + 3);
                    c = step64<TT, RG, LOADONLY>(c, a0, a1, a2, a3, T, G);
                    if (s + 2 < nfull) {
                        q = p + (s + 2) * S;
                        a0 = ld16<NT>(q); a1 = ld16<NT>(q + 1); a2 = ld16<NT>(q + 2); a3 = ld16<NT>(q + 3);
                    }
                    c = step64<TT, RG, LOADONLY>(c, b0, b1, b2, b3, T, G);
                }
                if (s < nfull) c = step64<TT, RG, LOADONLY>(c, a0, a1, a2, a3, T, G);
            }
            end = (nfull - 1) * kStep + (lane + 1) * kSeg;
        }
        const uint32_t ts = nfull * kStep + lane * kSeg;
        if (ts < len) {
            const uint32_t nb = min(kSeg, len - ts);
            uint32_t w[16];
            load_bytes64(base + ts, nb, w);
            c = feed_words<TT, 16>(gap_shift<RG>(c, G), w, nb, T);
            end = ts + nb;
        }
    } else {
        // Unaligned run (odd piece lengths, caller-provided pointers): same lane
        // structure, aligned-dword loads re-assembled in registers.
        const uint32_t nsteps = (len + kStep - 1) / kStep;
        for (uint32_t s = 0; s < nsteps; ++s) {
            const uint32_t ss = s * kStep + lane * kSeg;
            if (ss < len) {
                const uint32_t nb = min(kSeg, len - ss);
                uint32_t w[16];
                load_bytes64(base + ss, nb, w);
                c = feed_words<TT, 16>(gap_shift<RG>(c, G), w, nb, T);
                end = ss + nb;
            }
        }
    }
    const uint32_t d = len - end;
    uint32_t m = lane_mul;
    if (d != (63 - lane) * kSeg) m = x8n(d, x8pow);
    return end ? gf2_mulmod(c, m) : 0u;
}

// ---------------------------------------------------------- coalesced layout
template <class TT, int RG, bool LOADONLY = false>
__device__ __forceinline__ void step_coal(uint32_t c[4], const u32x4 v[4], const TT& T, const uint32_t* G) {
#pragma unroll
    for (int k = 0; k < 4; ++k)
        c[k] = LOADONLY ? c[k] ^ xor3(v[k].x, v[k].y, v[k].z) ^ v[k].w : seg16(gap_shift<RG>(c[k], G), v[k], T);
}

template <class TT, int RG, bool LOADONLY = false>
__device__ __forceinline__ uint32_t lane_crc_coal(uint64_t base, uint32_t len, uint32_t lane, const TT& T,
                                                  const uint32_t* G, const uint32_t lm[4], const uint32_t* x8pow) {
    uint32_t c[4] = {0u, 0u, 0u, 0u};
    uint32_t end[4] = {0u, 0u, 0u, 0u};
    const uint32_t nfull = len / kStep;
    uint32_t s0 = 0;  // first step left to the generic loop below
    if ((base & 15) == 0 && nfull > 0) {
        gptr<u32x4> p = as_global<u32x4>(base + lane * 16);
        constexpr uint32_t S = kStep / 16;
        u32x4 a[4], b[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] = p[64 * k];
        uint32_t s = 0;
        for (; s + 2 <= nfull; s += 2) {
            gptr<u32x4> q = p + (s + 1) * S;
#pragma unroll
            for (int k = 0; k < 4; ++k) b[k] = q[64 * k];
            step_coal<TT, RG, LOADONLY>(c, a, T, G);
            if (s + 2 < nfull) {
                q = p + (s + 2) * S;
#pragma unroll
                for (int k = 0; k < 4; ++k) a[k] = q[64 * k];
            }
            step_coal<TT, RG, LOADONLY>(c, b, T, G);
        }
        if (s < nfull) step_coal<TT, RG, LOADONLY>(c, a, T, G);
#pragma unroll
        for (int k = 0; k < 4; ++k) end[k] = (nfull - 1) * kStep + 1024 * k + 16 * lane + 16;
        s0 = nfull;
    }
    // The partial last step, or every step of an unaligned run.
    const uint32_t nsteps = (len + kStep - 1) / kStep;
    for (uint32_t s = s0; s < nsteps; ++s) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t ss = s * kStep + 1024 * k + 16 * lane;
            if (ss < len) {
                const uint32_t nb = min(16u, len - ss);
                uint32_t w[4];
                load_bytes16(base + ss, nb, w);
                c[k] = feed_words<TT, 4>(gap_shift<RG>(c[k], G), w, nb, T);
                end[k] = ss + nb;
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (end[k]) {
            const uint32_t d = len - end[k];
            const uint32_t m = d == kGapC - 1024 * k - 16 * lane ? lm[k] : x8n(d, x8pow);
            acc ^= gf2_mulmod(c[k], m);
        }
    }
    return acc;
}

// --------------------------------------------------------------- item source
struct ItemRef {
    uint64_t ptr;
    uint32_t len, out, mul, xr;
};

// Item `it` (wave-uniform) of the launch.
__device__ __forceinline__ ItemRef fetch_item(const CrcWork& w, uint32_t it) {
    if (it >= w.run_items) {
        const CrcItem ci = w.items[it - w.run_items];
        return {ci.ptr, ci.len, ci.out, ci.mul, ci.xr};
    }
    uint32_t lo = 0, hi = w.n_runs;  // last run with item_base <= it
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (w.runs[mid].item_base <= it) lo = mid;
        else hi = mid;
    }
    const CrcRun r = w.runs[lo];
    const uint32_t j = it - r.item_base;
    const uint32_t pc = j / r.ipp, jj = j - pc * r.ipp;
    const uint64_t q = uint64_t(jj) * kItemBytes;
    const uint64_t nx = min(q + kItemBytes, r.plen);
    return {r.ptr + uint64_t(pc) * r.plen + q, (uint32_t)(nx - q), r.out + pc, w.consts[r.cpat + jj],
            jj == 0 ? w.consts[r.cpat + r.ipp] : 0u};
}

// A wave's next item: the static stride (it + n_waves), or, with the work queue, the
// next unclaimed item (one atomicAdd by lane 0, broadcast) -- a wave on a CU that
// started late or runs slower (beside another kernel) simply claims fewer items.
template <bool QUEUE>
__device__ __forceinline__ uint32_t next_item(const CrcWork& w, uint32_t it, uint32_t n_waves, uint32_t lane) {
    if constexpr (QUEUE) {
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(w.next, 1u);
        return __builtin_amdgcn_readfirstlane(__shfl(v, 0, 64));
    } else {
        return it + n_waves;
    }
}

template <class TT, int RG, bool COAL, bool LOADONLY, bool NT, bool DEEP, bool QUEUE = false, int RING = 2>
__device__ __forceinline__ void item_loop(const CrcWork& w, const TT& T, const uint32_t* G, const uint32_t lm[4],
                                          const uint32_t* x8pow, uint32_t lane, uint32_t wave0, uint32_t n_waves,
                                          uint32_t* sums, lds_u32w ring = nullptr) {
    const uint32_t n_items = w.run_items + w.n_items;
    // every wave leaves once the queue head passes n_items (no wave waits on another)
    for (uint32_t it = QUEUE ? next_item<true>(w, 0, 0, lane) : wave0; it < n_items;
         it = next_item<QUEUE>(w, it, n_waves, lane)) {
        const ItemRef ci = fetch_item(w, it);
        uint32_t c = COAL ? lane_crc_coal<TT, RG, LOADONLY>(ci.ptr, ci.len, lane, T, G, lm, x8pow)
                          : lane_crc_strided<TT, RG, LOADONLY, NT, DEEP, RING>(ci.ptr, ci.len, lane, T, G, lm[0], x8pow, ring);
        // Wave XOR-reduction.
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) c ^= __shfl_xor(c, off, 64);
        if (lane == 0) {
            const uint32_t v = gf2_mulmod(c, ci.mul) ^ ci.xr;
            atomicXor(&sums[ci.out], v);
        }
    }
}

template <int R, int RG, int BLOCK, bool COAL, bool LOADONLY = false, int PERM = 0, bool NT = false, bool DEEP = false,
          bool QUEUE = false, int GLDS = 0>
__global__ void __launch_bounds__(BLOCK)
crc_items_kernel(CrcWork w, const uint32_t* __restrict__ tabs, uint32_t* __restrict__ sums) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr int TW = 1024 * (PERM ? PERM : R);
    constexpr int GW = 1024 * RG;
    constexpr int GT = COAL ? kTabGC : kTabG;
    if constexpr (PERM != 0) {
        for (int i = threadIdx.x; i < TW; i += BLOCK) {  // 16384 words (64 KiB) per region
            const int region = i >> 14, e = (i & 16383) >> 6, kk = (i & 63) / PERM;
            lds[i] = tabs[kTabT + (region * (64 / PERM) + kk) * 256 + e];
        }
    } else {
        for (int i = threadIdx.x; i < TW; i += BLOCK) lds[i] = tabs[kTabT + i / R];
    }
    for (int i = threadIdx.x; i < GW; i += BLOCK) lds[TW + i] = tabs[GT + i / RG];
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63;
    const uint32_t* G = lds + TW + (lane % RG);
    const uint32_t* x8pow = tabs + kTabX8Pow;
    uint32_t lm[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) lm[k] = COAL ? tabs[kTabLaneMulC + 64 * k + lane] : tabs[kTabLaneMul + lane];

    constexpr uint32_t WPB = BLOCK / 64;
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * WPB + threadIdx.x / 64);
    const uint32_t n_waves = gridDim.x * WPB;
    if constexpr (PERM != 0) {
        if ((uint32_t)(size_t)(lds_u32p)lds != 0) __builtin_trap();
        TabP<PERM> T;
        T.loff = (1u << 16) | ((lane % PERM) << 2);
        // GLDS: the wave's ring of GLDS 4 KiB steps after the tables
        lds_u32w ring = GLDS ? (lds_u32w)(lds + TW + GW) + (threadIdx.x / 64) * (GLDS * 1024) : nullptr;
        item_loop<TabP<PERM>, RG, COAL, LOADONLY, NT, DEEP, QUEUE, (GLDS ? GLDS : 2)>(w, T, G, lm, x8pow, lane, wave0,
                                                                                 n_waves, sums, ring);
    } else {
        Tab<R> T;
        T.lo = lds + (lane % R);
        T.hi = lds + 2 * 256 * R + (lane % R);
        item_loop<Tab<R>, RG, COAL, LOADONLY, NT, DEEP, QUEUE>(w, T, G, lm, x8pow, lane, wave0, n_waves, sums);
    }
}

template <int R, int RG, int BLOCK, bool COAL, bool LOADONLY = false, int PERM = 0, bool NT = false,
          bool DEEP = false, bool QUEUE = false, int GLDS = 0>
static hipError_t launch_variant(const CrcWork& w, const uint32_t* tabs, uint32_t* sums, int cus,
                                 int blocks_per_cu, hipStream_t s) {
    constexpr size_t lds = size_t(1024) * ((PERM ? PERM : R) + RG) * 4 + size_t(BLOCK / 64) * GLDS * 4096;
    static std::once_flag once;  // host threads may launch concurrently (re-entrant C ABI)
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [] {
        attr_err = hipFuncSetAttribute(reinterpret_cast<const void*>(&crc_items_kernel<R, RG, BLOCK, COAL, LOADONLY, PERM, NT, DEEP, QUEUE, GLDS>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    });
    if (attr_err != hipSuccess) return attr_err;
    const uint32_t wpb = BLOCK / 64;
    const uint64_t n_items = uint64_t(w.run_items) + w.n_items;
    uint64_t want = (n_items + wpb - 1) / wpb;
    uint64_t cap = uint64_t(cus) * blocks_per_cu;
    uint32_t grid = (uint32_t)(want < cap ? want : cap);
    if (grid == 0) return hipSuccess;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL((crc_items_kernel<R, RG, BLOCK, COAL, LOADONLY, PERM, NT, DEEP, QUEUE, GLDS>), dim3(grid), dim3(BLOCK), lds, s, w, tabs, sums);
    return hipGetLastError();
}

// Production launch variants (bit-exact): 16 = strided layout, byte-addressable tables
// with 32 replicas (144 KiB of LDS, one 1024-thread workgroup per CU) and the work
// queue, the default (+2.5-3 % over the static stride: 6.03-6.09 TB/s on 4 MiB pieces,
// 6.05 on 256 KiB, tools/crc_try.sh); 7 = the same with a static item stride; 8 = 7
// with 16 replicas (80 KiB, two workgroups per CU); 14 / 17 = 7 / 16 with three load
// sets in rotation; 15 = 14 with 8 gap-table replicas (160 KiB).  Every other layout
// measured in DESIGN.md 4.1 -- and the load-only timing diagnostics, which give WRONG
// sums -- is compiled only into the diagnostic build (make diag, -DKRK_DIAG).
bool crc_variant_valid(int v) {
#ifdef KRK_DIAG
    return v >= 0 && v <= 23;
#else
    return v == 7 || v == 8 || v == 14 || v == 15 || v == 16 || v == 17;
#endif
}

hipError_t launch_crc_items(const CrcWork& w, const uint32_t* tabs, uint32_t* sums, const CrcLaunchCfg& cfg,
                            hipStream_t s) {
    if (uint64_t(w.run_items) + w.n_items == 0) return hipSuccess;
    t_launch_units = uint64_t(w.run_items) + w.n_items;
    switch (cfg.variant) {
        case 7:
            return launch_variant<32, 4, 1024, false, false, 32>(w, tabs, sums, cfg.cus, 1, s);
        case 8:
            return launch_variant<16, 4, 1024, false, false, 16>(w, tabs, sums, cfg.cus, 2, s);
        case 14:  // 7 with three load sets in rotation (two steps of loads in flight)
            return launch_variant<32, 4, 1024, false, false, 32, false, true>(w, tabs, sums, cfg.cus, 1, s);
        case 15:  // 14 with 8 gap-table replicas (160 KiB of LDS: fewer bank conflicts on the gap lookups)
            return launch_variant<32, 8, 1024, false, false, 32, false, true>(w, tabs, sums, cfg.cus, 1, s);
        case 16:  // 7 with the work queue (items claimed by atomicAdd instead of a static stride)
            return w.next ? launch_variant<32, 4, 1024, false, false, 32, false, false, true>(w, tabs, sums, cfg.cus, 1, s)
                          : hipErrorInvalidValue;
        case 17:  // 14 with the work queue
            return w.next ? launch_variant<32, 4, 1024, false, false, 32, false, true, true>(w, tabs, sums, cfg.cus, 1, s)
                          : hipErrorInvalidValue;
#ifdef KRK_DIAG
        // LDS-DMA (bit-exact, measured in DESIGN.md 4.1): R16 byte-addressable
        // tables (64 KiB) + 4 gap replicas (16 KiB) + a two-step ring per wave (8 KiB), 10 waves
        // (160 KiB), work queue; 21 = the same with nt loads
        case 20:
            return w.next ? launch_variant<16, 4, 640, false, false, 16, false, false, true, 2>(w, tabs, sums, cfg.cus, 1, s)
                          : hipErrorInvalidValue;
        case 21:
            return w.next ? launch_variant<16, 4, 640, false, false, 16, true, false, true, 2>(w, tabs, sums, cfg.cus, 1, s)
                          : hipErrorInvalidValue;
        case 22:  // 6 waves x a three-step ring (two steps in flight a wave, 48 KiB a CU; 152 KiB)
            return w.next ? launch_variant<16, 4, 384, false, false, 16, false, false, true, 3>(w, tabs, sums, cfg.cus, 1, s)
                          : hipErrorInvalidValue;
        case 23:  // 5 waves x a four-step ring (three in flight a wave, 60 KiB a CU; 160 KiB)
            return w.next ? launch_variant<16, 4, 320, false, false, 16, false, false, true, 4>(w, tabs, sums, cfg.cus, 1, s)
                          : hipErrorInvalidValue;
        case 0:  // strided, interleaved R16 tables, 80 KiB LDS: two 512-thread blocks per CU
            return launch_variant<16, 4, 512, false>(w, tabs, sums, cfg.cus, 2, s);
        case 1:  // 144 KiB LDS: one 1024-thread block per CU
            return launch_variant<32, 4, 1024, false>(w, tabs, sums, cfg.cus, 1, s);
        case 2:  // coalesced, 80 KiB LDS: two 512-thread blocks per CU
            return launch_variant<16, 4, 512, true>(w, tabs, sums, cfg.cus, 2, s);
        case 3:  // coalesced, 144 KiB LDS: one 1024-thread block per CU
            return launch_variant<32, 4, 1024, true>(w, tabs, sums, cfg.cus, 1, s);
        case 4:  // timing diagnostic: variant 0's loads and occupancy without the lookups (wrong sums)
            return launch_variant<16, 4, 512, false, true>(w, tabs, sums, cfg.cus, 2, s);
        case 5:  // strided, 80 KiB LDS per 1024-thread block, two per CU: 32 waves/CU
            return launch_variant<16, 4, 1024, false>(w, tabs, sums, cfg.cus, 2, s);
        case 6:  // strided, R8 tables (40 KiB), four 512-thread blocks per CU: 32 waves/CU
            return launch_variant<8, 2, 512, false>(w, tabs, sums, cfg.cus, 4, s);
        case 9:  // as 7 with nontemporal data loads
            return launch_variant<32, 4, 1024, false, false, 32, true>(w, tabs, sums, cfg.cus, 1, s);
        case 10:  // timing diagnostic: variant 9's loads and occupancy without the lookups (wrong sums)
            return launch_variant<32, 4, 1024, false, true, 32, true>(w, tabs, sums, cfg.cus, 1, s);
        case 11:  // timing diagnostic: variant 7's loads and occupancy without the lookups (wrong sums)
            return launch_variant<32, 4, 1024, false, true, 32, false>(w, tabs, sums, cfg.cus, 1, s);
        case 12:  // coalesced, byte-addressable tables (144 KiB), one 1024-thread block per CU
            return launch_variant<32, 4, 1024, true, false, 32>(w, tabs, sums, cfg.cus, 1, s);
        case 13:  // timing diagnostic: variant 12's loads and occupancy without the lookups (wrong sums)
            return launch_variant<32, 4, 1024, true, true, 32>(w, tabs, sums, cfg.cus, 1, s);
#endif
        default:
            return hipErrorInvalidValue;
    }
}

__global__ void crc_verify_kernel(const uint32_t* sums, const uint32_t* expected, uint8_t* ok,
                                  uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ok[i] = sums[i] == expected[i];
}

hipError_t launch_crc_verify(const uint32_t* sums, const uint32_t* expected, uint8_t* ok,
                             uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    if (const hipError_t p_ = launch_precheck(); p_ != hipSuccess) return p_;
    hipLaunchKernelGGL(crc_verify_kernel, dim3((n + 255) / 256), dim3(256), 0, s, sums, expected,
                       ok, n);
    return hipGetLastError();
}

}  // namespace krk
