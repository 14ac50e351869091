// DPP semantics probe on gfx950: row_ror:8 with v_add / v_sub / v_subrev / v_mov, dst ==
// src1, and back-to-back DPP ops writing and reading the same register.
// Build: hipcc --offload-arch=gfx950 -O3 dppsem.hip -o dppsem
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k(unsigned* out) {
    const unsigned l = threadIdx.x;
    unsigned a = 1000u + l, b = 100000u * (l + 1), z, m, s, r, c, q;
    z = b;
    asm volatile("s_nop 4\n\tv_add_u32_dpp %0, %1, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\ts_nop 4" : "+v"(z) : "v"(a));
    m = 0;
    asm volatile("s_nop 4\n\tv_mov_b32_dpp %0, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n\ts_nop 4" : "+v"(m) : "v"(a));
    s = b;
    asm volatile("s_nop 4\n\tv_subrev_u32_dpp %0, %1, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\ts_nop 4" : "+v"(s) : "v"(a));
    r = b;
    asm volatile("s_nop 4\n\tv_sub_u32_dpp %0, %1, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\ts_nop 4" : "+v"(r) : "v"(a));
    // chain: c = b; c += DPP(a); c -= DPP(a) (3 ops apart) -> b
    c = b;
    unsigned t0 = 0, t1 = 0;
    asm volatile("s_nop 4\n\t"
                 "v_add_u32_dpp %0, %3, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                 "v_add_u32_e32 %1, 1, %1\n\t"
                 "v_add_u32_e32 %2, 1, %2\n\t"
                 "v_subrev_u32_dpp %0, %3, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 4"
                 : "+v"(c), "+v"(t0), "+v"(t1) : "v"(a));
    // chain with only one op between
    q = b;
    asm volatile("s_nop 4\n\t"
                 "v_add_u32_dpp %0, %2, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                 "v_add_u32_e32 %1, 1, %1\n\t"
                 "v_subrev_u32_dpp %0, %2, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 4"
                 : "+v"(q), "+v"(t0) : "v"(a));
    out[l] = z;
    out[64 + l] = m;
    out[128 + l] = s;
    out[192 + l] = r;
    out[256 + l] = c;
    out[320 + l] = q + t0 * 0 + t1 * 0;
}

int main() {
    unsigned* d;
    unsigned h[384];
    hipMalloc(&d, sizeof h);
    hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    const char* nm[6] = {"add z=DPP(a)+z", "mov m=DPP(a)", "subrev s=s-DPP(a)", "sub r=DPP(a)-r", "chain +DPP -DPP (2 between)",
                         "chain +DPP -DPP (1 between)"};
    for (int v = 0; v < 6; ++v) {
        printf("%-28s", nm[v]);
        for (int l = 0; l < 16; ++l) printf(" %d:%d", l, (int)h[64 * v + l]);
        printf("\n");
    }
    return 0;
}
