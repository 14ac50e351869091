// Issue cost of VALU encodings / operand shapes for one lone wave on gfx950:
// does a VOP3 cost more with three distinct VGPR sources than with two?
// Cycles via s_memtime over 256 independent instructions.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP4(x) x x x x
#define REP64(x) REP4(REP4(REP4(x)))
#define BODY(I) for (int it = 0; it < 64; ++it) asm volatile(REP64(I "\n\t")                                                   \
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3)                          \
                             : "v"(a), "v"(b), "v"(c), "s"(sg))
// %0..%3 destinations (only %0 used; the rest keep the operands live), %4 a, %5 b, %6 c, %7 sgpr
// One two-lane round (production shape: x0 feeds the next round), variants for
// pricing: VGPR vs immediate shift amounts, DPP vs plain add.
#define SH_V(r) "%[" #r "]"
#define SH_I(r) "7"
#define DPPSFX(x) DPPSFX_##x
#define DPPSFX_ "\n\t"
#define RND_V_DPP \
    "v_add_u32_dpp %[p], %[x1], %[z] row_mirror row_mask:0xf bank_mask:0xf\n\t" \
    "v_alignbit_b32 %[t1], %[x0], %[x0], %[r1]\n\t" \
    "v_alignbit_b32 %[t2], %[x0], %[x0], %[r2]\n\t" \
    "v_alignbit_b32 %[t3], %[x0], %[x0], %[r3]\n\t" \
    "v_bitop3_b32 %[k], %[x0], %[x1], %[ma] bitop3:0x2d\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t" \
    "v_bitop3_b32 %[k], %[k], %[x2], %[x1] bitop3:0xca\n\t" \
    "v_xad_u32 %[z], %[x2], %[ma], %[w]\n\t" \
    "v_add3_u32 %[x0], %[t1], %[k], %[p]\n\t"
#define RND_I_DPP \
    "v_add_u32_dpp %[p], %[x1], %[z] row_mirror row_mask:0xf bank_mask:0xf\n\t" \
    "v_alignbit_b32 %[t1], %[x0], %[x0], 2\n\t" \
    "v_alignbit_b32 %[t2], %[x0], %[x0], 13\n\t" \
    "v_alignbit_b32 %[t3], %[x0], %[x0], 22\n\t" \
    "v_bitop3_b32 %[k], %[x0], %[x1], %[ma] bitop3:0x2d\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t" \
    "v_bitop3_b32 %[k], %[k], %[x2], %[x1] bitop3:0xca\n\t" \
    "v_xad_u32 %[z], %[x2], %[ma], %[w]\n\t" \
    "v_add3_u32 %[x0], %[t1], %[k], %[p]\n\t"
#define RND_V_ADD \
    "v_add_u32_e32 %[p], %[x1], %[z]\n\t" \
    "v_alignbit_b32 %[t1], %[x0], %[x0], %[r1]\n\t" \
    "v_alignbit_b32 %[t2], %[x0], %[x0], %[r2]\n\t" \
    "v_alignbit_b32 %[t3], %[x0], %[x0], %[r3]\n\t" \
    "v_bitop3_b32 %[k], %[x0], %[x1], %[ma] bitop3:0x2d\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t" \
    "v_bitop3_b32 %[k], %[k], %[x2], %[x1] bitop3:0xca\n\t" \
    "v_xad_u32 %[z], %[x2], %[ma], %[w]\n\t" \
    "v_add3_u32 %[x0], %[t1], %[k], %[p]\n\t"
#define RND_I_ADD \
    "v_add_u32_e32 %[p], %[x1], %[z]\n\t" \
    "v_alignbit_b32 %[t1], %[x0], %[x0], 2\n\t" \
    "v_alignbit_b32 %[t2], %[x0], %[x0], 13\n\t" \
    "v_alignbit_b32 %[t3], %[x0], %[x0], 22\n\t" \
    "v_bitop3_b32 %[k], %[x0], %[x1], %[ma] bitop3:0x2d\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t" \
    "v_bitop3_b32 %[k], %[k], %[x2], %[x1] bitop3:0xca\n\t" \
    "v_xad_u32 %[z], %[x2], %[ma], %[w]\n\t" \
    "v_add3_u32 %[x0], %[t1], %[k], %[p]\n\t"
#define RBODY(R) for (int it = 0; it < 64; ++it) asm volatile(REP64(R) \
        : [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [k] "=&v"(kk), [p] "=&v"(p), [z] "+v"(z), [x0] "+v"(x0) \
        : [x1] "v"(x1), [x2] "v"(x2), [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [ma] "v"(ma), [w] "v"(w))

template <int K>
__global__ void rcost(unsigned long long* out, unsigned* sink) {
    const unsigned l = threadIdx.x;
    unsigned t1, t2, t3, kk, p, z = 1, x0 = l, x1 = 3 * l, x2 = 5 * l, w = 9;
    const unsigned r1 = (l & 8) ? 6 : 2, r2 = (l & 8) ? 11 : 13, r3 = (l & 8) ? 25 : 22, ma = (l & 8) ? 0u : ~0u;
    asm volatile("s_nop 7\n\ts_nop 7" ::);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();
    if (K == 0) RBODY(RND_V_DPP);
    if (K == 1) RBODY(RND_I_DPP);
    if (K == 2) RBODY(RND_V_ADD);
    if (K == 3) RBODY(RND_I_ADD);
    const unsigned long long tt = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
    if (l == 0) {
        out[32 + K] = tt - t0;
        out[96 + K] = q1 - q0;
    }
    sink[l] = x0 + z;
}


// Rotating-register rounds (the production shape: x1/x2/x3 are earlier rounds' x0).
#define QR(X0, X1, X2, NX, DPPLINE) \
    DPPLINE \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t" \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t" \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t" \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t" \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t" \
    "v_xad_u32 %[z], %[" #X2 "], %[ma], %[w]\n\t" \
    "v_add3_u32 %[" #NX "], %[t1], %[k], %[p]\n\t"
#define DPP_X1(X1) "v_add_u32_dpp %[p], %[" #X1 "], %[z] row_mirror row_mask:0xf bank_mask:0xf\n\t"
#define ADD_X1(X1) "v_add_u32_e32 %[p], %[" #X1 "], %[z]\n\t"
#define DPP_C(X1) "v_add_u32_dpp %[p], %[w], %[z] row_mirror row_mask:0xf bank_mask:0xf\n\t"
#define QQ(D) QR(R0, R3, R2, R1, D(R3)) QR(R1, R0, R3, R2, D(R0)) QR(R2, R1, R0, R3, D(R1)) QR(R3, R2, R1, R0, D(R2))
#define QBODY(D) for (int it = 0; it < 64; ++it) asm volatile(REP4(REP4(QQ(D))) \
        : [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [k] "=&v"(kk), [p] "=&v"(p), [z] "+v"(z), \
          [R0] "+v"(R0), [R1] "+v"(R1), [R2] "+v"(R2), [R3] "+v"(R3) \
        : [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [ma] "v"(ma), [w] "v"(w))
template <int K>
__global__ void qcost(unsigned long long* out, unsigned* sink) {
    const unsigned l = threadIdx.x;
    unsigned t1, t2, t3, kk, p, z = 1, R0 = l, R1 = 3 * l, R2 = 5 * l, R3 = 7 * l, w = 9;
    const unsigned r1 = (l & 8) ? 6 : 2, r2 = (l & 8) ? 11 : 13, r3 = (l & 8) ? 25 : 22, ma = (l & 8) ? 0u : ~0u;
    asm volatile("s_nop 7\n\ts_nop 7" ::);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (K == 0) QBODY(DPP_X1);
    if (K == 1) QBODY(ADD_X1);
    if (K == 2) QBODY(DPP_C);
    const unsigned long long tt = __builtin_amdgcn_s_memtime();
    if (l == 0) out[40 + K] = tt - t0;
    sink[l] = R0 + R1 + R2 + R3 + z;
}


// Which rotating operand makes the round slow?  QV(X0, X1k, X1f, X2f, X2z, X1p, NX): the
// register each use reads (k's x1, F's x1, F's x2, z's x2, p's x1).
#define QV(X0, X1K, X1F, X2F, X2Z, X1P, NX) \
    "v_add_u32_e32 %[p], %[" #X1P "], %[z]\n\t" \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t" \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t" \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t" \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1K "], %[ma] bitop3:0x2d\n\t" \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t" \
    "v_bitop3_b32 %[k], %[k], %[" #X2F "], %[" #X1F "] bitop3:0xca\n\t" \
    "v_xad_u32 %[z], %[" #X2Z "], %[ma], %[w]\n\t" \
    "v_add3_u32 %[" #NX "], %[t1], %[k], %[p]\n\t"
// rotation R0..R3; C = constant register
#define VQ(a, b, c, d, e) QV(R0, a##3, b##3, c##2, d##2, e##3, R1) QV(R1, a##0, b##0, c##3, d##3, e##0, R2) \
                          QV(R2, a##1, b##1, c##0, d##0, e##1, R3) QV(R3, a##2, b##2, c##1, d##1, e##2, R0)
#define VBODY(Q) for (int it = 0; it < 64; ++it) asm volatile(REP4(REP4(Q)) \
        : [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3), [k] "=&v"(kk), [p] "=&v"(p), [z] "+v"(z), \
          [R0] "+v"(R0), [R1] "+v"(R1), [R2] "+v"(R2), [R3] "+v"(R3) \
        : [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [ma] "v"(ma), [w] "v"(w), [C0] "v"(c0), [C1] "v"(c1), \
          [C2] "v"(c2), [C3] "v"(c3))
template <int K>
__global__ void vcost(unsigned long long* out, unsigned* sink) {
    const unsigned l = threadIdx.x;
    unsigned t1, t2, t3, kk, p, z = 1, R0 = l, R1 = 3 * l, R2 = 5 * l, R3 = 7 * l, w = 9;
    const unsigned c0 = l + 1, c1 = l + 2, c2 = l + 3, c3 = l + 4;
    const unsigned r1 = (l & 8) ? 6 : 2, r2 = (l & 8) ? 11 : 13, r3 = (l & 8) ? 25 : 22, ma = (l & 8) ? 0u : ~0u;
    asm volatile("s_nop 7\n\ts_nop 7" ::);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (K == 0) VBODY(VQ(R, R, R, R, R));  // all rotating (production)
    if (K == 1) VBODY(VQ(C, R, R, R, R));  // k's x1 constant
    if (K == 2) VBODY(VQ(R, C, R, R, R));  // F's x1 constant
    if (K == 3) VBODY(VQ(R, R, C, R, R));  // F's x2 constant
    if (K == 4) VBODY(VQ(R, R, R, C, R));  // z's x2 constant
    if (K == 5) VBODY(VQ(R, R, R, R, C));  // p's x1 constant
    if (K == 6) VBODY(VQ(C, C, C, C, C));  // all constant
    const unsigned long long tt = __builtin_amdgcn_s_memtime();
    if (l == 0) out[48 + K] = tt - t0;
    sink[l] = R0 + R1 + R2 + R3 + z;
}

template <int K>
__global__ void cost(unsigned long long* out, unsigned* sink) {
    unsigned d0 = threadIdx.x, d1 = 1, d2 = 2, d3 = 3, a = threadIdx.x * 3, b = 7, c = 9, sg = 11;
    asm volatile("s_nop 7\n\ts_nop 7" ::);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (K == 0) BODY("v_alignbit_b32 %0, %4, %4, 6");
    if (K == 1) BODY("v_alignbit_b32 %0, %4, %4, %5");
    if (K == 2) BODY("v_alignbit_b32 %0, %4, %6, %5");
    if (K == 3) BODY("v_bitop3_b32 %0, %4, %5, %6 bitop3:0x96");
    if (K == 4) BODY("v_bitop3_b32 %0, %4, %4, %5 bitop3:0x96");
    if (K == 5) BODY("v_bitop3_b32 %0, %4, %4, %4 bitop3:0x96");
    if (K == 6) BODY("v_add3_u32 %0, %4, %5, %6");
    if (K == 7) BODY("v_add3_u32 %0, %4, %5, 5");
    if (K == 8) BODY("v_xad_u32 %0, %4, %5, %6");
    if (K == 9) BODY("v_add_u32_e32 %0, %4, %5");
    if (K == 10) BODY("v_add_u32_e64 %0, %4, %5");
    if (K == 11) BODY("v_add_u32_dpp %0, %4, %5 row_mirror row_mask:0xf bank_mask:0xf");
    if (K == 12) BODY("v_lshl_add_u32 %0, %4, 2, %5");
    if (K == 13) BODY("v_bitop3_b32 %0, %4, %5, %7 bitop3:0x96");
    if (K == 14) BODY("v_xor_b32_e32 %0, %4, %5");
    if (K == 15) BODY("v_cndmask_b32_e32 %0, %4, %5, vcc");
    // dependent chains (each op reads the previous result)
    if (K == 16) BODY("v_add_u32_e32 %0, %0, %5");
    if (K == 17) BODY("v_add3_u32 %0, %0, %5, %6");
    if (K == 18) BODY("v_alignbit_b32 %0, %0, %0, 7");
    if (K == 19) BODY("v_bitop3_b32 %0, %0, %5, %6 bitop3:0x96");
    if (K == 20) BODY("v_add_u32_dpp %0, %0, %5 row_mirror row_mask:0xf bank_mask:0xf\n\ts_nop 1");
    if (K == 21) BODY("s_nop 1");
    // two interleaved dependent chains
    if (K == 22) BODY("v_add3_u32 %0, %0, %5, %6\n\tv_add3_u32 %1, %1, %5, %6");
    // four interleaved dependent chains
    if (K == 23) BODY("v_add3_u32 %0, %0, %5, %6\n\tv_add3_u32 %1, %1, %5, %6\n\tv_add3_u32 %2, %2, %5, %6\n\tv_add3_u32 %3, %3, %5, %6");
    // dependent through a DPP source read (needs 2 wait states: here filled by 2 independent ops)
    if (K == 24) BODY("v_add_u32_dpp %0, %0, %5 row_mirror row_mask:0xf bank_mask:0xf\n\tv_add_u32_e32 %1, %1, %5\n\tv_add_u32_e32 %2, %2, %5");
    // encoding size vs operand count: a VOP2 add with a 32-bit literal is 8 bytes with two sources
    if (K == 25) BODY("v_add_u32_e32 %0, 0x12345, %5");
    if (K == 26) BODY("v_fma_f32 %0, %4, %5, %6");
    if (K == 27) BODY("v_mov_b32_e32 %0, 0x12345");
    if (K == 28) BODY("v_add_u32_e32 %0, %4, %5\n\tv_add3_u32 %1, %4, %5, %6");
    if (K == 29) BODY("v_add_u32_e32 %0, %4, %5\n\tv_add_u32_e32 %1, %4, %6\n\tv_add3_u32 %2, %4, %5, %6");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[K] = t1 - t0;
        out[64 + K] = r1 - r0;
    }
    sink[threadIdx.x] = d0 + d1 + d2 + d3;
}

template <int K>
void run(unsigned long long* d, unsigned* s) {
    hipLaunchKernelGGL(cost<K>, 1, 64, 0, 0, d, s);
}

int main() {
    unsigned long long* d;
    unsigned* sink;
    hipMalloc(&d, 128 * 8);
    hipMalloc(&sink, 64 * 4);
    const char* names[] = {"alignbit v,v,imm", "alignbit v,v,v", "alignbit v,v',v", "bitop3 3 vgprs",
                           "bitop3 2 vgprs", "bitop3 1 vgpr", "add3 3 vgprs", "add3 2 vgprs+imm",
                           "xad 3 vgprs", "add VOP2", "add VOP3 (e64)", "add DPP", "lshl_add v,imm,v",
                           "bitop3 2 vgprs+sgpr", "xor VOP2", "cndmask VOP2", "DEP add VOP2", "DEP add3",
                           "DEP alignbit", "DEP bitop3", "DEP dpp+s_nop1 (per pair)", "s_nop 1", "2 chains add3 (per pair)",
                           "4 chains add3 (per 4)", "DEP dpp + 2 indep (per 3)", "add VOP2 + literal (8B)",
                           "fma_f32 (VOP3 8B)", "mov VOP1 + literal (8B)", "add VOP2 + add3 (per pair)",
                           "2 add VOP2 + add3 (per 3)"};
    for (int rep = 0; rep < 3; ++rep) {
        run<0>(d, sink); run<1>(d, sink); run<2>(d, sink); run<3>(d, sink); run<4>(d, sink); run<5>(d, sink);
        run<6>(d, sink); run<7>(d, sink); run<8>(d, sink); run<9>(d, sink); run<10>(d, sink); run<11>(d, sink);
        run<12>(d, sink); run<13>(d, sink); run<14>(d, sink); run<15>(d, sink);
        run<16>(d, sink); run<17>(d, sink); run<18>(d, sink); run<19>(d, sink); run<20>(d, sink); run<21>(d, sink);
        run<22>(d, sink); run<23>(d, sink); run<24>(d, sink); run<25>(d, sink); run<26>(d, sink);
        run<27>(d, sink); run<28>(d, sink); run<29>(d, sink);
        hipLaunchKernelGGL(rcost<0>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(rcost<1>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(rcost<2>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(rcost<3>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(qcost<0>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(qcost<1>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(qcost<2>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(vcost<0>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(vcost<1>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(vcost<2>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(vcost<3>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(vcost<4>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(vcost<5>, 1, 64, 0, 0, d, sink);
        hipLaunchKernelGGL(vcost<6>, 1, 64, 0, 0, d, sink);
        hipDeviceSynchronize();
        unsigned long long h[128];
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        if (rep == 2)
            for (int k = 0; k < 30; ++k)
                printf("%-26s %.2f cycles/instr  (%.3f GHz)\n", names[k], h[k] / (256.0 * 64), h[k] / (h[64 + k] * 10.0));
        if (rep == 2) {
            const char* rn[] = {"round VGPR-shift DPP", "round imm-shift DPP", "round VGPR-shift add", "round imm-shift add"};
            for (int k = 0; k < 4; ++k)
                printf("%-26s %.2f cycles/round (%.3f GHz)\n", rn[k], h[32 + k] / (256.0 * 64), h[32 + k] / (h[96 + k] * 10.0));
            const char* qn[] = {"rotating, DPP of x1", "rotating, plain add of x1", "rotating, DPP of a const"};
            for (int k = 0; k < 3; ++k) printf("%-26s %.2f cycles/round\n", qn[k], h[40 + k] / (64.0 * 64));
            const char* vn[] = {"V all rotating", "V k.x1 const", "V F.x1 const", "V F.x2 const", "V z.x2 const",
                                "V p.x1 const", "V all const"};
            for (int k = 0; k < 7; ++k) printf("%-26s %.2f cycles/round\n", vn[k], h[48 + k] / (64.0 * 64));
        }
    }
    return 0;
}
