// Microbenchmark + correctness check for an EIGHT-lanes-per-stream SHA-256 round
// (candidate for sha256_multi.hip) against the production two-lane round.
//
// Two-lane round (production): 9 ops, all 8-byte encodings: 3 v_alignbit (the three
// rotations of Sigma), v_bitop3 xor3, v_bitop3 k, v_bitop3 F, v_xad z, DPP add, v_add3.
// Eight-lane round: every stream has an E quad and an A quad; the three active lanes of
// a quad hold the same history and rotate by ONE of the three Sigma amounts each, and
// two quad_perm DPP xors combine the three rotations (every active lane ends with the
// full Sigma): 8 ops a round (1 alignbit + 2 DPP xor instead of 3 alignbit + xor3).
// Lane layout in a DPP row of 16: quad 0 / 1 = E quads of streams 2r / 2r+1, quad
// 2 / 3 = their A quads; row_ror:8 pairs quad 0 with 2 and 1 with 3.  Lane 3 of each
// quad idles (it computes a single rotation; its results are never read).
//
// Each variant runs NB chained compressions of one 64-byte block per stream (W + K
// from LDS, read as production does: three quads ahead) and checks every stream's
// state against a host SHA-256 compression; cycles via s_memtime / s_memrealtime.
// Build: hipcc --offload-arch=gfx950 -O3 sha8lane.hip -o sha8lane
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static inline uint32_t hrotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static void host_compress(uint32_t h[8], const uint32_t kw[64]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int r = 0; r < 64; ++r) {
        uint32_t t1 = hh + (hrotr(e, 6) ^ hrotr(e, 11) ^ hrotr(e, 25)) + ((e & f) ^ (~e & g)) + kw[r];
        uint32_t t2 = (hrotr(a, 2) ^ hrotr(a, 13) ^ hrotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---- rounds ---------------------------------------------------------------
// Production two-lane round (sha256_multi.hip KRK_SHA2_ROUND).
#define ROUND2(X0, X1, X2, NX, WN)                                                      \
    "v_add_u32_dpp %[p], %[" #X1 "], %[z] row_mirror row_mask:0xf bank_mask:0xf\n\t"    \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                          \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                          \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                          \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_xad_u32 %[z], %[" #X2 "], %[ma], %[" #WN "]\n\t"                                \
    "v_add3_u32 %[" #NX "], %[t1], %[k], %[p]\n\t"

// Eight-lane round: t = this lane's rotation; the first DPP xor reads t three ops
// after it is written (two wait states), the second four.
#define ROUND8(X0, X1, X2, NX, WN)                                                      \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_xor_b32_dpp %[t2], %[t1], %[t1] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t" \
    "v_xor_b32_dpp %[t2], %[t1], %[t2] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t" \
    "v_add_u32_dpp %[p], %[" #X1 "], %[z] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"     \
    "v_xad_u32 %[z], %[" #X2 "], %[ma], %[" #WN "]\n\t"                                \
    "v_add3_u32 %[" #NX "], %[t2], %[k], %[p]\n\t"

struct LaneConst {
    uint32_t r1, r2, r3, ma, one_a;
};

#define OPS : [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [k] "=&v"(kk), [p] "=&v"(p), [z] "+v"(z), \
              [R0] "+v"(R0), [R1] "+v"(R1), [R2] "+v"(R2), [R3] "+v"(R3)
#define CONSTS [r1] "v"(c.r1), [r2] "v"(c.r2), [r3] "v"(c.r3), [ma] "v"(c.ma)

template <int V>
__device__ __forceinline__ void quad(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z,
                                     const LaneConst& c, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4) {
    uint32_t t1, t2, t3, kk, p;
    if (V == 0)
        asm volatile(ROUND2(R0, R3, R2, R1, w1) ROUND2(R1, R0, R3, R2, w2) ROUND2(R2, R1, R0, R3, w3)
                         ROUND2(R3, R2, R1, R0, w4) OPS
                     : CONSTS, [w1] "v"(w1), [w2] "v"(w2), [w3] "v"(w3), [w4] "v"(w4));
    else
        asm volatile(ROUND8(R0, R3, R2, R1, w1) ROUND8(R1, R0, R3, R2, w2) ROUND8(R2, R1, R0, R3, w3)
                         ROUND8(R3, R2, R1, R0, w4) OPS
                     : CONSTS, [w1] "v"(w1), [w2] "v"(w2), [w3] "v"(w3), [w4] "v"(w4));
}

template <int V>
__device__ __forceinline__ void one(uint32_t& X0, uint32_t& X1, uint32_t& X2, uint32_t& NX, uint32_t& z,
                                    const LaneConst& c, uint32_t w) {
    uint32_t t1, t2, t3, kk, p;
    uint32_t R0 = X0, R3 = X1, R2 = X2, R1 = NX;
    if (V == 0)
        asm volatile(ROUND2(R0, R3, R2, R1, w) OPS : CONSTS, [w] "v"(w));
    else
        asm volatile(ROUND8(R0, R3, R2, R1, w) OPS : CONSTS, [w] "v"(w));
    NX = R1;
}

// One block: 66 instruction-rounds, the A lanes two rounds behind the E lanes (the
// production rounds2 schedule).  h = (H4..H7) on E lanes, (H2, H3, H0, H1) on A lanes.
template <int V>
__device__ __forceinline__ void block(uint32_t h[4], const uint32_t* lds, uint32_t base, const LaneConst& c,
                                      bool is_e) {
    uint32_t R0 = h[0], R3 = h[1], R2 = h[2], R1 = h[3], z;
    u32x4 wq[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) wq[q] = *reinterpret_cast<const u32x4*>(lds + base + 256 * q);
    {
        uint32_t t1, t2, t3, kk, p;
        asm volatile("v_xad_u32 %[z], %[R1], %[ma], %[w0]\n\t" OPS : CONSTS, [w0] "v"(wq[0][0]));
    }
    one<V>(R0, R3, R2, R1, z, c, wq[0][1]);
    R1 = is_e ? R1 : h[3];
    one<V>(R1, R0, R3, R2, z, c, wq[0][2]);
    R2 = is_e ? R2 : h[2];
    one<V>(R2, R1, R0, R3, z, c, wq[0][3]);
    one<V>(R3, R2, R1, R0, z, c, wq[1][0]);
#pragma unroll
    for (int q = 1; q < 16; ++q) quad<V>(R0, R1, R2, R3, z, c, wq[q][1], wq[q][2], wq[q][3], q + 1 < 16 ? wq[q + 1][0] : c.one_a);
    uint32_t T1 = 0, T2 = 0;
    one<V>(R0, R3, R2, T1, z, c, c.one_a);
    one<V>(T1, R0, R3, T2, z, c, c.one_a);
    h[0] += R0;
    h[1] += R3;
    h[2] += is_e ? R2 : T2;
    h[3] += is_e ? R1 : T1;
}

// Lane roles.  V == 0: two lanes (row_mirror: A lane s, E lane 15 - s, 8 streams a
// row).  V == 1: eight lanes (quads 0/1 E, 2/3 A of streams 2r / 2r+1).
template <int V>
__device__ void roles(uint32_t lane, bool& is_e, uint32_t& stream, uint32_t& pos, uint32_t& spw) {
    if (V == 0) {
        is_e = (lane >> 3) & 1;
        stream = (lane >> 4) * 8 + (is_e ? 7 - (lane & 7) : (lane & 7));
        pos = 0;
        spw = 32;
    } else {
        const uint32_t q = (lane >> 2) & 3;
        is_e = q < 2;
        stream = (lane >> 4) * 2 + (q & 1);
        pos = lane & 3;
        spw = 8;
    }
}

template <int V>
__global__ void __launch_bounds__(64) run(const uint32_t* __restrict__ kw_all, const uint32_t* __restrict__ h0,
                                          uint32_t* __restrict__ out, uint32_t nb, unsigned long long* cyc) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[64 * 64 + 64];
    const uint32_t lane = threadIdx.x;
    bool is_e;
    uint32_t s, pos, spw;
    roles<V>(lane, is_e, s, pos, spw);
    const uint32_t stream = blockIdx.x * spw + s;
    // column `lane`: quad q of this lane at (q * 64 + lane) * 4 (production kw_index)
    for (int r = 0; r < 64; ++r) lds[((r >> 2) * 64 + lane) * 4 + (r & 3)] = is_e ? kw_all[stream * 64 + r] : 1u;
    __syncthreads();
    LaneConst c;
    if (V == 0) {
        c = LaneConst{is_e ? 6u : 2u, is_e ? 11u : 13u, is_e ? 25u : 22u, is_e ? 0u : ~0u, is_e ? 0u : 1u};
    } else {
        const uint32_t re[4] = {6, 11, 25, 6}, ra[4] = {2, 13, 22, 2};
        c = LaneConst{is_e ? re[pos] : ra[pos], 0u, 0u, is_e ? 0u : ~0u, is_e ? 0u : 1u};
    }
    uint32_t h[4];
    for (int k = 0; k < 4; ++k) h[k] = is_e ? h0[stream * 8 + 4 + k] : h0[stream * 8 + (k ^ 2)];
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), rt0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t i = 0; i < nb; ++i) block<V>(h, lds, lane * 4, c, is_e);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
    if (lane == 0 && blockIdx.x == 0) {
        cyc[0] = t1 - t0;
        cyc[1] = rt1 - rt0;
    }
    if (pos == 0)
        for (int k = 0; k < 4; ++k) out[stream * 8 + (is_e ? 4 + k : (k ^ 2))] = h[k];
}

int main() {
    const int waves = 4, nb = 2000;
    const int smax = waves * 32;
    uint32_t* kw = (uint32_t*)malloc(smax * 64 * 4);
    uint32_t* h0 = (uint32_t*)malloc(smax * 8 * 4);
    uint32_t* res = (uint32_t*)malloc(smax * 8 * 4);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < smax * 64; ++i) { x = x * 6364136223846793005ull + 1442695040888963407ull; kw[i] = (uint32_t)(x >> 32); }
    for (int i = 0; i < smax * 8; ++i) { x = x * 6364136223846793005ull + 1442695040888963407ull; h0[i] = (uint32_t)(x >> 32); }
    uint32_t *dkw, *dh0, *dout;
    unsigned long long* dcyc;
    hipMalloc(&dkw, smax * 64 * 4);
    hipMalloc(&dh0, smax * 8 * 4);
    hipMalloc(&dout, smax * 8 * 4);
    hipMalloc(&dcyc, 16);
    hipMemcpy(dkw, kw, smax * 64 * 4, hipMemcpyHostToDevice);
    hipMemcpy(dh0, h0, smax * 8 * 4, hipMemcpyHostToDevice);
    const char* names[2] = {"two-lane (production round, 9 ops)", "eight-lane (quad Sigma, 8 ops)"};
    for (int v = 0; v < 2; ++v) {
        const int spw = v == 0 ? 32 : 8;
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(dout, 0, smax * 8 * 4);
            if (v == 0) hipLaunchKernelGGL(run<0>, 1, 64, 0, 0, dkw, dh0, dout, nb, dcyc);
            else hipLaunchKernelGGL(run<1>, 1, 64, 0, 0, dkw, dh0, dout, nb, dcyc);
            if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
            unsigned long long cy[2];
            hipMemcpy(cy, dcyc, 16, hipMemcpyDeviceToHost);
            hipMemcpy(res, dout, spw * 8 * 4, hipMemcpyDeviceToHost);
            int bad = 0;
            for (int s = 0; s < spw; ++s) {
                uint32_t h[8];
                memcpy(h, h0 + s * 8, 32);
                for (int i = 0; i < nb; ++i) host_compress(h, kw + s * 64);
                if (memcmp(h, res + s * 8, 32)) ++bad;
            }
            const double secs = cy[1] * 1e-8;  // s_memrealtime: 100 MHz
            printf("%-38s streams %2d  bad %d  memtime/block %.1f  ns/block %.1f  clock %.3f GHz  MB/s/stream %.2f\n",
                   names[v], spw, bad, (double)cy[0] / nb, secs * 1e9 / nb, cy[0] / secs / 1e9, 64.0 * nb / secs / 1e6);
        }
    }
    return 0;
}
