// Which SIMD / CU does each wave of a multi-wave workgroup land on?  Reads HW_REG_HW_ID
// (gfx9 layout: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13]) per wave.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void hwid(unsigned* out, int spin) {
    unsigned v = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_REG_HW_ID, offset 0, 32 bits
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = v;
    // keep the waves resident for a while so later workgroups cannot reuse slots
    long t0 = clock64();
    while (clock64() - t0 < spin) {}
}

int main() {
    unsigned* d;
    hipMalloc(&d, 64 * 8 * 4);
    for (int threads : {128, 192, 256}) {
        hipMemset(d, 0xff, 64 * 8 * 4);
        hipLaunchKernelGGL(hwid, 32, threads, 0, 0, d, 200000);
        unsigned h[64 * 8];
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        printf("threads=%d\n", threads);
        for (int b = 0; b < 8; ++b) {
            printf("  wg %2d:", b);
            for (int w = 0; w < threads / 64; ++w) {
                unsigned v = h[b * 8 + w];
                printf("  [wave %u simd %u cu %u sh %u se %u]", v & 15, (v >> 4) & 3, (v >> 8) & 15, (v >> 12) & 1, (v >> 13) & 7);
            }
            printf("\n");
        }
    }
    return 0;
}
