// What the W reads cost the eight-lane SHA-256 round (sha256_multi.hip KRK_SHA8_ROUND)
// for one lone wave: 4 rounds a quad, W of the quad from a ds_read_b128 issued three
// quads ahead (production kAhead = 3), against W from registers; variants place the
// read after the quad's second round, read for a broadcast address, or read from
// only the E lanes' distinct addresses.  Timing only (no digest).
// Build: hipcc --offload-arch=gfx950 -O3 sha8lds.hip -o sha8lds
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ROUND8(X0, X1, X2, NX, WN)                                                      \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_xor_b32_dpp %[t2], %[t1], %[t1] quad_perm:[1,2,0,3] row_mask:0xf bank_mask:0xf\n\t" \
    "v_xor_b32_dpp %[t2], %[t1], %[t2] quad_perm:[2,0,1,3] row_mask:0xf bank_mask:0xf\n\t" \
    "v_add_u32_dpp %[p], %[" #X1 "], %[z] row_ror:8 row_mask:0xf bank_mask:0xf\n\t"     \
    "v_xad_u32 %[z], %[" #X2 "], %[ma], %[" #WN "]\n\t"                                \
    "v_add3_u32 %[" #NX "], %[t2], %[k], %[p]\n\t"

#define OPS                                                                                                   \
    : [t1] "=&v"(t1), [t2] "=&v"(t2), [k] "=&v"(kk), [p] "=&v"(p), [z] "+v"(z), [R0] "+v"(R0), [R1] "+v"(R1), \
      [R2] "+v"(R2), [R3] "+v"(R3)
#define CON [r1] "v"(r1), [ma] "v"(ma)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void half1(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z, uint32_t r1,
                                      uint32_t ma, uint32_t w1, uint32_t w2) {
    uint32_t t1, t2, kk, p;
    asm volatile(ROUND8(R0, R3, R2, R1, w1) ROUND8(R1, R0, R3, R2, w2) OPS : CON, [w1] "v"(w1), [w2] "v"(w2));
}
__device__ __forceinline__ void half2(uint32_t& R0, uint32_t& R1, uint32_t& R2, uint32_t& R3, uint32_t& z, uint32_t r1,
                                      uint32_t ma, uint32_t w3, uint32_t w4) {
    uint32_t t1, t2, kk, p;
    asm volatile(ROUND8(R2, R1, R0, R3, w3) ROUND8(R3, R2, R1, R0, w4) OPS : CON, [w3] "v"(w3), [w4] "v"(w4));
}

template <int V>
__global__ void __launch_bounds__(64) run(unsigned long long* out, unsigned* sink) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[16 * 64 * 4 + 64];
    const uint32_t l = threadIdx.x;
    for (int i = l; i < 16 * 64 * 4; i += 64) lds[i] = i * 2654435761u;
    __syncthreads();
    uint32_t R0 = l, R1 = 2 * l, R2 = 3 * l, R3 = 5 * l, z = 7;
    const uint32_t r1 = (l & 3) == 1 ? 11 : (l & 3) == 2 ? 25 : 6, ma = (l & 8) ? ~0u : 0u;
    // V 1, 2: production pattern (E lanes 8 distinct 16-B columns, A lanes one broadcast column)
    // V 3: every lane one address; V 4: every lane its own column (64 distinct)
    uint32_t col = (l & 8) ? 8u : ((l >> 4) * 2 + ((l >> 2) & 1));
    if (V == 3) col = 0;
    if (V == 4) col = l;
    const uint32_t* base = lds + col * 4;
    constexpr int kRS = 4;
    u4 wq[kRS];
#pragma unroll
    for (int j = 0; j < kRS; ++j) wq[j] = u4{l + j, 3u * j, 5u, 7u};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 256; ++it) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const u4 cur = wq[q % kRS];
            if (V == 1 || V == 3 || V == 4)  // read three quads ahead, before the quad (production)
                wq[(q + 3) % kRS] = *reinterpret_cast<const u4*>(base + 256 * ((q + 3) & 15));
            half1(R0, R1, R2, R3, z, r1, ma, cur.x, cur.y);
            if (V == 2)  // read three quads ahead, in the middle of the quad
                wq[(q + 3) % kRS] = *reinterpret_cast<const u4*>(base + 256 * ((q + 3) & 15));
            half2(R0, R1, R2, R3, z, r1, ma, cur.z, cur.w);
        }
    }
    const unsigned long long t1c = __builtin_amdgcn_s_memtime();
    if (l == 0) out[0] = t1c - t0;
    sink[l] = R0 + R1 + R2 + R3 + z + wq[0].x + wq[1].y + wq[2].z + wq[3].w;
}

int main() {
    unsigned long long* o;
    unsigned* s;
    hipMalloc(&o, 8);
    hipMalloc(&s, 256);
    const char* nm[5] = {"W from registers", "read 3 quads ahead, before the quad", "read 3 ahead, mid-quad",
                         "read 3 ahead, one broadcast address", "read 3 ahead, 64 distinct columns"};
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < 5; ++v) {
            switch (v) {
                case 0: hipLaunchKernelGGL(run<0>, 1, 64, 0, 0, o, s); break;
                case 1: hipLaunchKernelGGL(run<1>, 1, 64, 0, 0, o, s); break;
                case 2: hipLaunchKernelGGL(run<2>, 1, 64, 0, 0, o, s); break;
                case 3: hipLaunchKernelGGL(run<3>, 1, 64, 0, 0, o, s); break;
                case 4: hipLaunchKernelGGL(run<4>, 1, 64, 0, 0, o, s); break;
            }
            unsigned long long c = 0;
            hipMemcpy(&c, o, 8, hipMemcpyDeviceToHost);
            if (rep) printf("%-40s %.2f cycles/round\n", nm[v], c / (256.0 * 64));
        }
    return 0;
}
