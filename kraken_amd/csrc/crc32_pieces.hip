// crc32_pieces.hip -- piece CRC-32/IEEE for gfx950 (core.calcPieceSums,
// core/metainfo.go:158-179; PieceHash = crc32.NewIEEE, core/piece_hash.go:22-24).
//
// Layout of the work: one wave per CrcItem (<= 256 KiB inside one piece).  A wave
// step covers 4 KiB: lane l owns the 64-byte segment [step*4096 + 64l, +64) and
// loads it as 4 x 16-byte global loads (a wave step reads one contiguous 4 KiB).
// Each lane runs slicing-by-4 over its own bytes; between two of its segments the
// lane's virtual stream holds 4032 zero bytes, applied as one shift-by-4032 table
// step (4 lookups per 64 bytes).  At the end every lane shifts its register to the
// item end (one GF(2) multiply by a per-lane constant), the wave XOR-reduces, and
// lane 0 shifts to the piece end and atomically XORs into sums[piece].
//
// Tables live in LDS, replicated R times and interleaved (word (t*256+e)*R + r) so
// lane l reads replica l % R: with R = 32 the 32 lanes of a ds_read_b32 half-wave
// hit 32 distinct banks (conflict-free); R = 16 allows at most 2-way.
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

template <int RG>
__device__ __forceinline__ uint32_t gap_shift(uint32_t c, const uint32_t* G) {
    return xor3(G[(0 * 256 + (c & 0xFF)) * RG], G[(1 * 256 + ((c >> 8) & 0xFF)) * RG],
                G[(2 * 256 + ((c >> 16) & 0xFF)) * RG]) ^ G[(3 * 256 + (c >> 24)) * RG];
}

template <int R>
__device__ __forceinline__ uint32_t seg16(uint32_t c, const u32x4& v, const Tab<R>& T) {
    c = T.word(c ^ v.x);
    c = T.word(c ^ v.y);
    c = T.word(c ^ v.z);
    c = T.word(c ^ v.w);
    return c;
}

// One wave step for this lane: skip the 4032-byte gap, then its 64 own bytes.
template <int R, int RG>
__device__ __forceinline__ uint32_t step64(uint32_t c, const u32x4& v0, const u32x4& v1, const u32x4& v2,
                                           const u32x4& v3, const Tab<R>& T, const uint32_t* G) {
    c = gap_shift<RG>(c, G);
    c = seg16(c, v0, T);
    c = seg16(c, v1, T);
    c = seg16(c, v2, T);
    return seg16(c, v3, T);
}

// Bytes [p, p+n) into register c, n <= kSeg, any alignment (see load_bytes64).
template <int R>
__device__ __forceinline__ uint32_t seg_tail(uint32_t c, uint64_t p, uint32_t n, const Tab<R>& T) {
    uint32_t w[16];
    load_bytes64(p, n, w);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int keep = (int)n - 4 * j;
        if (keep >= 4) {
            c = T.word(c ^ w[j]);
        } else if (keep > 0) {
            for (int b = 0; b < keep; ++b) c = T.byte(c, (w[j] >> (8 * b)) & 0xFF);
        }
    }
    return c;
}

template <int R, int RG, int BLOCK>
__global__ void __launch_bounds__(BLOCK)
crc_items_kernel(const CrcItem* __restrict__ items, uint32_t n_items,
                 const uint32_t* __restrict__ tabs, uint32_t* __restrict__ sums) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr int TW = 1024 * R;
    constexpr int GW = 1024 * RG;
    for (int i = threadIdx.x; i < TW; i += BLOCK) lds[i] = tabs[kTabT + i / R];
    for (int i = threadIdx.x; i < GW; i += BLOCK) lds[TW + i] = tabs[kTabG + i / RG];
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63;
    Tab<R> T;
    T.lo = lds + (lane % R);
    T.hi = lds + 2 * 256 * R + (lane % R);
    const uint32_t* G = lds + TW + (lane % RG);
    const uint32_t lane_mul = tabs[kTabLaneMul + lane];
    const uint32_t* x8pow = tabs + kTabX8Pow;

    constexpr uint32_t WPB = BLOCK / 64;
    const uint32_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * WPB + threadIdx.x / 64);
    const uint32_t n_waves = gridDim.x * WPB;

    for (uint32_t it = wave0; it < n_items; it += n_waves) {
        const CrcItem ci = items[it];
        const uint64_t base = ci.ptr;
        const uint32_t len = ci.len;
        uint32_t c = 0;
        uint32_t end = 0;  // end offset (in item) of this lane's last processed byte + 1
        const uint32_t nfull = len / kStep;

        if ((ci.ptr & 15) == 0) {
            if (nfull > 0) {
                // Two register sets in ping-pong: the next step's 4 x 16 B are in
                // flight while the current step's lookups run.
                gptr<u32x4> p = as_global<u32x4>(base + lane * kSeg);
                constexpr uint32_t S = kStep / 16;
                u32x4 a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
                u32x4 b0, b1, b2, b3;
                uint32_t s = 0;
                for (; s + 2 <= nfull; s += 2) {
                    gptr<u32x4> q = p + (s + 1) * S;
                    b0 = q[0]; b1 = q[1]; b2 = q[2]; b3 = q[3];
                    c = step64<R, RG>(c, a0, a1, a2, a3, T, G);
                    if (s + 2 < nfull) {
                        q = p + (s + 2) * S;
                        a0 = q[0]; a1 = q[1]; a2 = q[2]; a3 = q[3];
                    }
                    c = step64<R, RG>(c, b0, b1, b2, b3, T, G);
                }
                if (s < nfull) c = step64<R, RG>(c, a0, a1, a2, a3, T, G);
                end = (nfull - 1) * kStep + (lane + 1) * kSeg;
            }
            const uint32_t ts = nfull * kStep + lane * kSeg;
            if (ts < len) {
                const uint32_t nb = min(kSeg, len - ts);
                c = gap_shift<RG>(c, G);
                c = seg_tail(c, base + ts, nb, T);
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
                    c = gap_shift<RG>(c, G);
                    c = seg_tail(c, base + ss, nb, T);
                    end = ss + nb;
                }
            }
        }

        // Shift this lane's register to the item end.
        const uint32_t d = len - end;
        uint32_t m = lane_mul;
        if (d != (63 - lane) * kSeg) m = x8n(d, x8pow);
        c = end ? gf2_mulmod(c, m) : 0u;
        // Wave XOR-reduction.
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) c ^= __shfl_xor(c, off, 64);
        if (lane == 0) {
            const uint32_t v = gf2_mulmod(c, ci.mul) ^ ci.xr;
            atomicXor(&sums[ci.out], v);
        }
    }
}

template <int R, int RG, int BLOCK>
static hipError_t launch_variant(const CrcItem* items, uint32_t n_items, const uint32_t* tabs,
                                 uint32_t* sums, int cus, int blocks_per_cu, hipStream_t s) {
    constexpr size_t lds = size_t(1024) * (R + RG) * 4;
    static bool attr_set = false;
    if (!attr_set) {
        hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&crc_items_kernel<R, RG, BLOCK>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr_set = true;
    }
    const uint32_t wpb = BLOCK / 64;
    uint64_t want = (uint64_t(n_items) + wpb - 1) / wpb;
    uint64_t cap = uint64_t(cus) * blocks_per_cu;
    uint32_t grid = (uint32_t)(want < cap ? want : cap);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((crc_items_kernel<R, RG, BLOCK>), dim3(grid), dim3(BLOCK), lds, s, items,
                       n_items, tabs, sums);
    return hipGetLastError();
}

hipError_t launch_crc_items(const CrcItem* items, uint32_t n_items, const uint32_t* tabs,
                            uint32_t* sums, const CrcLaunchCfg& cfg, hipStream_t s) {
    if (n_items == 0) return hipSuccess;
    if (cfg.variant == 1)  // 144 KiB LDS: one 1024-thread block per CU
        return launch_variant<32, 4, 1024>(items, n_items, tabs, sums, cfg.cus, 1, s);
    // 80 KiB LDS: two 512-thread blocks per CU
    return launch_variant<16, 4, 512>(items, n_items, tabs, sums, cfg.cus, 2, s);
}

__global__ void crc_verify_kernel(const uint32_t* sums, const uint32_t* expected, uint8_t* ok,
                                  uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ok[i] = sums[i] == expected[i];
}

hipError_t launch_crc_verify(const uint32_t* sums, const uint32_t* expected, uint8_t* ok,
                             uint32_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(crc_verify_kernel, dim3((n + 255) / 256), dim3(256), 0, s, sums, expected,
                       ok, n);
    return hipGetLastError();
}

}  // namespace krk
