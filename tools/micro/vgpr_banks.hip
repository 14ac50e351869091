// Microbenchmark: issue cost of 3-source VOP3 ops (v_add3_u32, v_bitop3_b32,
// v_alignbit_b32) for one lone wave on gfx950, with the three sources in
// distinct VGPR banks (reg % 4) vs in the same bank.  Cycles via s_memtime.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int K>
__global__ void bench(unsigned long long* out) {
    unsigned long long t0, t1;
    asm volatile("v_mov_b32 v1, 1\n v_mov_b32 v2, 2\n v_mov_b32 v3, 3\n v_mov_b32 v4, 4\n"
                 "v_mov_b32 v8, 8\n v_mov_b32 v12, 12\n v_mov_b32 v5, 5\n v_mov_b32 v6, 6\n v_mov_b32 v7, 7\n"
                 ::: "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v12");
    t0 = __builtin_amdgcn_s_memtime();
    if (K == 0)  // add3, sources in banks 1,2,3 (independent results)
        asm volatile(REP64("v_add3_u32 v5, v1, v2, v3\n v_add3_u32 v6, v1, v2, v3\n v_add3_u32 v7, v1, v2, v3\n v_add3_u32 v9, v1, v2, v3\n")
                     ::: "v5", "v6", "v7", "v9");
    if (K == 1)  // add3, sources all in bank 0
        asm volatile(REP64("v_add3_u32 v5, v4, v8, v12\n v_add3_u32 v6, v4, v8, v12\n v_add3_u32 v7, v4, v8, v12\n v_add3_u32 v9, v4, v8, v12\n")
                     ::: "v5", "v6", "v7", "v9");
    if (K == 2)  // alignbit, same register twice (rotate)
        asm volatile(REP64("v_alignbit_b32 v5, v1, v1, 6\n v_alignbit_b32 v6, v2, v2, 11\n v_alignbit_b32 v7, v3, v3, 25\n v_alignbit_b32 v9, v1, v1, 2\n")
                     ::: "v5", "v6", "v7", "v9");
    if (K == 3)  // 2-source VOP2 add
        asm volatile(REP64("v_add_u32_e32 v5, v1, v2\n v_add_u32_e32 v6, v1, v2\n v_add_u32_e32 v7, v1, v2\n v_add_u32_e32 v9, v1, v2\n")
                     ::: "v5", "v6", "v7", "v9");
    if (K == 4)  // bitop3, banks 1,2,3
        asm volatile(REP64("v_bitop3_b32 v5, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v6, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v7, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v9, v1, v2, v3 bitop3:0x96\n")
                     ::: "v5", "v6", "v7", "v9");
    if (K == 5)  // bitop3, banks 0,0,0
        asm volatile(REP64("v_bitop3_b32 v5, v4, v8, v12 bitop3:0x96\n v_bitop3_b32 v6, v4, v8, v12 bitop3:0x96\n v_bitop3_b32 v7, v4, v8, v12 bitop3:0x96\n v_bitop3_b32 v9, v4, v8, v12 bitop3:0x96\n")
                     ::: "v5", "v6", "v7", "v9");
    if (K == 6)  // dependent chain of add3 (each uses the previous result), banks mixed
        asm volatile(REP64("v_add3_u32 v5, v5, v2, v3\n v_add3_u32 v5, v5, v2, v3\n v_add3_u32 v5, v5, v2, v3\n v_add3_u32 v5, v5, v2, v3\n")
                     ::: "v5");
    if (K == 7)  // chain with one independent op between dependents
        asm volatile(REP64("v_add3_u32 v5, v5, v2, v3\n v_add3_u32 v6, v1, v2, v3\n v_add3_u32 v5, v5, v2, v3\n v_add3_u32 v6, v1, v2, v3\n")
                     ::: "v5", "v6");
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 8);
    const char* names[] = {"add3 banks 1,2,3", "add3 banks 0,0,0", "alignbit rotate", "v_add_u32 (VOP2)",
                           "bitop3 banks 1,2,3", "bitop3 banks 0,0,0", "add3 dependent chain",
                           "add3 dep every other"};
    for (int rep = 0; rep < 2; ++rep) {
        for (int k = 0; k < 8; ++k) {
            switch (k) {
                case 0: hipLaunchKernelGGL(bench<0>, 1, 64, 0, 0, d); break;
                case 1: hipLaunchKernelGGL(bench<1>, 1, 64, 0, 0, d); break;
                case 2: hipLaunchKernelGGL(bench<2>, 1, 64, 0, 0, d); break;
                case 3: hipLaunchKernelGGL(bench<3>, 1, 64, 0, 0, d); break;
                case 4: hipLaunchKernelGGL(bench<4>, 1, 64, 0, 0, d); break;
                case 5: hipLaunchKernelGGL(bench<5>, 1, 64, 0, 0, d); break;
                case 6: hipLaunchKernelGGL(bench<6>, 1, 64, 0, 0, d); break;
                case 7: hipLaunchKernelGGL(bench<7>, 1, 64, 0, 0, d); break;
            }
            unsigned long long c = 0;
            hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
            if (rep) printf("%-24s %.2f cycles/instr\n", names[k], c / 256.0);
        }
    }
    return 0;
}
