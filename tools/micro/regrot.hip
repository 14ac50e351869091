// Why is a round whose result lands in a different register each round (x0 rotating
// through 4 registers) ~4x slower than the same round writing one register?  Explicit
// physical registers, lone wave, s_memtime cycles per round.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP4(x) x x x x
#define REP16(x) REP4(REP4(x))
// round: X0 read, NX written; everything else fixed (as the compiler allocated rcost)
#define RR(X0, NX) \
    "v_add_u32_e32 v14, v3, v1\n\t" \
    "v_alignbit_b32 v10, " X0 ", " X0 ", v5\n\t" \
    "v_alignbit_b32 v11, " X0 ", " X0 ", v6\n\t" \
    "v_alignbit_b32 v12, " X0 ", " X0 ", v7\n\t" \
    "v_bitop3_b32 v13, " X0 ", v3, v8 bitop3:0x2d\n\t" \
    "v_bitop3_b32 v10, v10, v11, v12 bitop3:0x96\n\t" \
    "v_bitop3_b32 v13, v13, v4, v3 bitop3:0xca\n\t" \
    "v_xad_u32 v1, v4, v8, v9\n\t" \
    "v_add3_u32 " NX ", v10, v13, v14\n\t"
#define INIT "v_mov_b32 v1, 1\n\tv_mov_b32 v2, 2\n\tv_mov_b32 v3, 3\n\tv_mov_b32 v4, 4\n\tv_mov_b32 v5, 5\n\t" \
             "v_mov_b32 v6, 6\n\tv_mov_b32 v7, 7\n\tv_mov_b32 v8, 8\n\tv_mov_b32 v9, 9\n\tv_mov_b32 v20, 20\n\t" \
             "v_mov_b32 v21, 21\n\tv_mov_b32 v22, 22\n\tv_mov_b32 v16, 16\n\tv_mov_b32 v17, 17\n\ts_nop 7\n\t"
#define CLOB "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v16", "v17", \
             "v20", "v21", "v22"

template <int K>
__global__ void k(unsigned long long* out) {
    asm volatile(INIT ::: CLOB);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < 64; ++it) {
        if (K == 0) asm volatile(REP16(RR("v2", "v2") RR("v2", "v2") RR("v2", "v2") RR("v2", "v2")) ::: CLOB);
        if (K == 1) asm volatile(REP16(RR("v2", "v20") RR("v20", "v21") RR("v21", "v22") RR("v22", "v2")) ::: CLOB);
        if (K == 2) asm volatile(REP16(RR("v2", "v20") RR("v20", "v2") RR("v2", "v20") RR("v20", "v2")) ::: CLOB);
        if (K == 3) asm volatile(REP16(RR("v2", "v16") RR("v16", "v17") RR("v17", "v22") RR("v22", "v2")) ::: CLOB);
        // the result read one round later AND again 1..3 rounds later (like x1/x2): x1 = v20 fixed
        if (K == 4) asm volatile(REP16(RR("v2", "v2") RR("v2", "v2") RR("v2", "v2") RR("v2", "v2")) ::: CLOB);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[K] = t1 - t0;
}

int main() {
    unsigned long long* d;
    hipMalloc(&d, 8 * 8);
    const char* nm[] = {"x0 in v2 always", "x0 rotates v2,v20,v21,v22", "x0 alternates v2,v20",
                        "x0 rotates v2,v16,v17,v22", "same as 0"};
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k<0>, 1, 64, 0, 0, d);
        hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, d);
        hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, d);
        hipLaunchKernelGGL(k<3>, 1, 64, 0, 0, d);
        hipLaunchKernelGGL(k<4>, 1, 64, 0, 0, d);
        hipDeviceSynchronize();
        unsigned long long h[8];
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        if (rep)
            for (int i = 0; i < 5; ++i) printf("%-30s %.2f cycles/round\n", nm[i], h[i] / (64.0 * 64));
    }
    return 0;
}
