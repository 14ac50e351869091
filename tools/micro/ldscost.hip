// Issue cost of LDS reads inside a VALU-dense stream for one lone wave (gfx950): per
// iteration 8 independent 8-byte VALU ops (v_add3) plus one LDS read whose result is
// waited for one iteration later -- the shape of the SHA-256 consumer (16 reads a
// block among ~530 VALU).  Variants: no read, ds_read_b32 / b64 / b128, two b64, a b128
// with every lane on one address (broadcast), and a b128 issued with half the lanes.
// Cycles via s_memtime.  Build: hipcc --offload-arch=gfx950 -O3 ldscost.hip -o ldscost
#include <hip/hip_runtime.h>
#include <stdio.h>

#define V8 "v_add3_u32 %[a0], %[a0], %[k], %[k]\n\tv_add3_u32 %[a1], %[a1], %[k], %[k]\n\t" \
           "v_add3_u32 %[a2], %[a2], %[k], %[k]\n\tv_add3_u32 %[a3], %[a3], %[k], %[k]\n\t" \
           "v_add3_u32 %[a4], %[a4], %[k], %[k]\n\tv_add3_u32 %[a5], %[a5], %[k], %[k]\n\t" \
           "v_add3_u32 %[a6], %[a6], %[k], %[k]\n\tv_add3_u32 %[a7], %[a7], %[k], %[k]\n\t"

template <int V>
__global__ void __launch_bounds__(64) k(unsigned long long* out, unsigned* sink) {
    __shared__ __attribute__((aligned(16))) unsigned lds[64 * 64 * 4];
    const unsigned l = threadIdx.x;
    for (int i = l; i < 64 * 64 * 4; i += 64) lds[i] = i;
    __syncthreads();
    unsigned a0 = l, a1 = l + 1, a2 = l + 2, a3 = l + 3, a4 = l + 4, a5 = l + 5, a6 = l + 6, a7 = l + 7, kk = 3;
    unsigned addr = V == 5 ? 0u : l * 16u;  // byte address
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    u4 d = {0, 0, 0, 0}, e = {0, 0, 0, 0};
    const unsigned long long hmask = 0x00000000FFFFFFFFull;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 4096; ++it) {
        if (V == 0)
            asm volatile(V8 : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4),
                         [a5] "+v"(a5), [a6] "+v"(a6), [a7] "+v"(a7) : [k] "v"(kk));
        if (V == 1)
            asm volatile("s_waitcnt lgkmcnt(6)\n\tds_read_b32 %[d], %[ad] offset:1024\n\t" V8
                         : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4), [a5] "+v"(a5),
                           [a6] "+v"(a6), [a7] "+v"(a7), [d] "=&v"(d.x)
                         : [k] "v"(kk), [ad] "v"(addr));
        if (V == 2)
            asm volatile("s_waitcnt lgkmcnt(6)\n\tds_read_b64 %[d], %[ad] offset:1024\n\t" V8
                         : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4), [a5] "+v"(a5),
                           [a6] "+v"(a6), [a7] "+v"(a7), [d] "=&v"(*(unsigned long long*)&d)
                         : [k] "v"(kk), [ad] "v"(addr));
        if (V == 3 || V == 5)
            asm volatile("s_waitcnt lgkmcnt(6)\n\tds_read_b128 %[d], %[ad] offset:1024\n\t" V8
                         : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4), [a5] "+v"(a5),
                           [a6] "+v"(a6), [a7] "+v"(a7), [d] "=&v"(d)
                         : [k] "v"(kk), [ad] "v"(addr));
        if (V == 4)
            asm volatile("s_waitcnt lgkmcnt(6)\n\tds_read_b64 %[d], %[ad] offset:1024\n\t"
                         "v_add3_u32 %[a0], %[a0], %[k], %[k]\n\tv_add3_u32 %[a1], %[a1], %[k], %[k]\n\t"
                         "v_add3_u32 %[a2], %[a2], %[k], %[k]\n\tv_add3_u32 %[a3], %[a3], %[k], %[k]\n\t"
                         "ds_read_b64 %[e], %[ad] offset:1032\n\t"
                         "v_add3_u32 %[a4], %[a4], %[k], %[k]\n\tv_add3_u32 %[a5], %[a5], %[k], %[k]\n\t"
                         "v_add3_u32 %[a6], %[a6], %[k], %[k]\n\tv_add3_u32 %[a7], %[a7], %[k], %[k]\n\t"
                         : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4), [a5] "+v"(a5),
                           [a6] "+v"(a6), [a7] "+v"(a7), [d] "=&v"(*(unsigned long long*)&d),
                           [e] "=&v"(*(unsigned long long*)&e)
                         : [k] "v"(kk), [ad] "v"(addr));
        if (V == 6)  // half the lanes issue the read
            asm volatile("s_waitcnt lgkmcnt(6)\n\ts_mov_b64 exec, %[m]\n\tds_read_b128 %[d], %[ad] offset:1024\n\t"
                         "s_mov_b64 exec, -1\n\t" V8
                         : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [a4] "+v"(a4), [a5] "+v"(a5),
                           [a6] "+v"(a6), [a7] "+v"(a7), [d] "=&v"(d)
                         : [k] "v"(kk), [ad] "v"(addr), [m] "s"(hmask));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) out[0] = t1 - t0;
    sink[l] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + d.x + d.y + d.z + d.w + e.x + e.y;
}

int main() {
    unsigned long long* o;
    unsigned* s;
    hipMalloc(&o, 8);
    hipMalloc(&s, 256);
    const char* nm[7] = {"8 VALU only", "+ ds_read_b32", "+ ds_read_b64", "+ ds_read_b128", "+ 2x ds_read_b64",
                         "+ ds_read_b128 broadcast", "+ ds_read_b128, 32 lanes (exec)"};
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < 7; ++v) {
            switch (v) {
                case 0: hipLaunchKernelGGL(k<0>, 1, 64, 0, 0, o, s); break;
                case 1: hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, o, s); break;
                case 2: hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, o, s); break;
                case 3: hipLaunchKernelGGL(k<3>, 1, 64, 0, 0, o, s); break;
                case 4: hipLaunchKernelGGL(k<4>, 1, 64, 0, 0, o, s); break;
                case 5: hipLaunchKernelGGL(k<5>, 1, 64, 0, 0, o, s); break;
                case 6: hipLaunchKernelGGL(k<6>, 1, 64, 0, 0, o, s); break;
            }
            unsigned long long c = 0;
            hipMemcpy(&c, o, 8, hipMemcpyDeviceToHost);
            if (rep) printf("%-34s %.2f cycles/iteration\n", nm[v], c / 4096.0);
        }
    return 0;
}
