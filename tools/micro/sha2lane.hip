// Microbenchmark for the two-lanes-per-stream SHA-256 round (sha256_multi.hip):
//  * DPP row_shl/row_shr + bank_mask semantics on gfx950 (which lane reads which);
//  * issue cost of v_add_u32_dpp and v_xad_u32 for one lone wave;
//  * cycles per round of the 14-op one-lane round vs the 10-op two-lane round.
// Cycles via s_memtime.  Build: hipcc --offload-arch=gfx950 -O3 sha2lane.hip -o sha2lane
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP4(x) x x x x
#define REP16(x) REP4(REP4(x))
#define REP64(x) REP16(REP4(x))

__global__ void dpp_semantics(unsigned* out) {
    unsigned lane = threadIdx.x, a, b;
    a = 1000u;
    b = 2000u;
    // a <- src(lane+4) + 0 on banks 0,2 ; b <- src(lane-4) on banks 1,3
    asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %2, %3 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
                 "v_add_u32_dpp %1, %2, %3 row_shr:4 row_mask:0xf bank_mask:0xa\n\ts_nop 1"
                 : "+v"(a), "+v"(b)
                 : "v"(lane), "v"(0u));
    unsigned m = 3000u;
    asm volatile("s_nop 1\n\tv_add_u32_dpp %0, %1, %2 row_mirror row_mask:0xf bank_mask:0xf\n\ts_nop 1"
                 : "=&v"(m) : "v"(lane), "v"(0u));
    out[lane] = a;
    out[64 + lane] = b;
    out[128 + lane] = m;
}

template <int K>
__global__ void cost(unsigned long long* out, unsigned* sink) {
    unsigned long long t0, t1;
    unsigned v5 = threadIdx.x, v6 = 3, v7 = 7, v8 = 9, v9 = 11, v10 = 13;
    t0 = __builtin_amdgcn_s_memtime();
    if (K == 0)  // independent DPP adds
        asm volatile(REP64("v_add_u32_dpp %0, %4, %5 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
                           "v_add_u32_dpp %1, %4, %5 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
                           "v_add_u32_dpp %2, %4, %5 row_shl:4 row_mask:0xf bank_mask:0x5\n\t"
                           "v_add_u32_dpp %3, %4, %5 row_shl:4 row_mask:0xf bank_mask:0x5\n\t")
                     : "+v"(v5), "+v"(v8), "+v"(v9), "+v"(v10)
                     : "v"(v6), "v"(v7));
    if (K == 1)  // v_xad_u32
        asm volatile(REP64("v_xad_u32 %0, %4, %5, %4\n\tv_xad_u32 %1, %4, %5, %4\n\t"
                           "v_xad_u32 %2, %4, %5, %4\n\tv_xad_u32 %3, %4, %5, %4\n\t")
                     : "+v"(v5), "+v"(v8), "+v"(v9), "+v"(v10)
                     : "v"(v6), "v"(v7));
    if (K == 2)  // VOP3 add3 for comparison
        asm volatile(REP64("v_add3_u32 %0, %4, %5, %4\n\tv_add3_u32 %1, %4, %5, %4\n\t"
                           "v_add3_u32 %2, %4, %5, %4\n\tv_add3_u32 %3, %4, %5, %4\n\t")
                     : "+v"(v5), "+v"(v8), "+v"(v9), "+v"(v10)
                     : "v"(v6), "v"(v7));
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
    sink[threadIdx.x] = v5 + v8 + v9 + v10;
}

// One-lane round (the production KRK_SHA_ROUND body, 12 VOP3 + 2 VOP2).
#define ONE_ROUND                                                        \
    "v_alignbit_b32 %[r6], %[e], %[e], 6\n\t"                            \
    "v_alignbit_b32 %[r11], %[e], %[e], 11\n\t"                          \
    "v_alignbit_b32 %[r25], %[e], %[e], 25\n\t"                          \
    "v_bitop3_b32 %[ch], %[e], %[f], %[g] bitop3:0xca\n\t"               \
    "v_bitop3_b32 %[r6], %[r6], %[r11], %[r25] bitop3:0x96\n\t"          \
    "v_alignbit_b32 %[q2], %[a], %[a], 2\n\t"                            \
    "v_add3_u32 %[t1], %[hk], %[r6], %[ch]\n\t"                          \
    "v_alignbit_b32 %[q13], %[a], %[a], 13\n\t"                          \
    "v_add_u32_e32 %[e], %[d], %[t1]\n\t"                                \
    "v_alignbit_b32 %[q22], %[a], %[a], 22\n\t"                          \
    "v_bitop3_b32 %[mj], %[a], %[b], %[c] bitop3:0xe8\n\t"               \
    "v_bitop3_b32 %[q2], %[q2], %[q13], %[q22] bitop3:0x96\n\t"          \
    "v_add_u32_e32 %[hk], %[g], %[kw]\n\t"                               \
    "v_add3_u32 %[a], %[t1], %[q2], %[mj]\n\t"

// Two-lane round: 8 VOP3 + 2 DPP (see sha256_multi.hip for the algebra).
#define TWO_ROUND                                                        \
    "v_alignbit_b32 %[t1], %[x0], %[x0], %[r1]\n\t"                      \
    "v_alignbit_b32 %[t2], %[x0], %[x0], %[r2]\n\t"                      \
    "v_bitop3_b32 %[k], %[x0], %[x1], %[ma] bitop3:0x2d\n\t"             \
    "v_alignbit_b32 %[t3], %[x0], %[x0], %[r3]\n\t"                      \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"            \
    "v_bitop3_b32 %[k], %[k], %[x2], %[x1] bitop3:0xca\n\t"              \
    "v_add3_u32 %[v], %[t1], %[k], %[p]\n\t"                             \
    "v_xad_u32 %[p], %[x2], %[ma], %[c]\n\t"                             \
    "v_add_u32_dpp %[c], %[x0], %[kw] row_shr:4 row_mask:0xf bank_mask:0xa\n\t" \
    "v_add_u32_dpp %[v], %[v], %[v] row_shl:4 row_mask:0xf bank_mask:0x5\n\t"

template <int K>
__global__ void rounds(unsigned long long* out, unsigned* sink) {
    unsigned long long t0, t1;
    const unsigned l = threadIdx.x;
    unsigned a = l, b = l * 3, c = l * 5, d = l * 7, e = l * 9, f = l * 11, g = l * 13, hk = 17, kw = 19;
    unsigned r6, r11, r25, ch, q2, t1v, q13, q22, mj;
    unsigned x0 = l, x1 = 2 * l, x2 = 3 * l, p = 5, cc = 1, v = 0, k, tt1, tt2, tt3;
    const unsigned r1 = (l & 4) ? 6 : 2, r2 = (l & 4) ? 11 : 13, r3 = (l & 4) ? 25 : 22;
    const unsigned ma = (l & 4) ? 0u : ~0u;
    t0 = __builtin_amdgcn_s_memtime();
    if (K == 0) {
        asm volatile(REP64(ONE_ROUND)
                     : [r6] "=&v"(r6), [r11] "=&v"(r11), [r25] "=&v"(r25), [ch] "=&v"(ch), [q2] "=&v"(q2),
                       [t1] "=&v"(t1v), [q13] "=&v"(q13), [q22] "=&v"(q22), [mj] "=&v"(mj), [a] "+v"(a),
                       [e] "+v"(e), [hk] "+v"(hk)
                     : [b] "v"(b), [c] "v"(c), [d] "v"(d), [f] "v"(f), [g] "v"(g), [kw] "v"(kw));
    } else {
        asm volatile(REP64(TWO_ROUND)
                     : [t1] "=&v"(tt1), [t2] "=&v"(tt2), [t3] "=&v"(tt3), [k] "=&v"(k), [v] "+v"(v), [p] "+v"(p),
                       [c] "+v"(cc), [x0] "+v"(x0)
                     : [x1] "v"(x1), [x2] "v"(x2), [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [ma] "v"(ma),
                       [kw] "v"(kw));
    }
    t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) out[0] = t1 - t0;
    sink[l] = a + e + hk + x0 + v + p + cc;
}


// The production two-lane quad (true cross-round dependencies: R0..R3 rotate).
#define R2(X0, X1, X2, V, CW, CR, KWN, PRE, MID, POST)                                  \
    PRE                                                                                \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                          \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                          \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                          \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_add3_u32 %[" #V "], %[t1], %[k], %[p]\n\t"                                      \
    MID                                                                                \
    "v_add_u32_dpp %[" #CW "], %[" #X0 "], %[" #KWN "] row_shr:4 row_mask:0xf bank_mask:0xa\n\t" \
    "v_add_u32_dpp %[" #V "], %[" #V "], %[" #V "] row_shl:4 row_mask:0xf bank_mask:0x5\n\t" \
    POST
#define XADN(X2, CR) "v_xad_u32 %[p], %[" #X2 "], %[ma], %[" #CR "]\n\t"
// variant 2: production order (xad between add3 and the DPPs)
#define Q2 R2(R0, R3, R2, R1, C3, C1, kw, "", XADN(R2, C1), "") R2(R1, R0, R3, R2, C0, C2, kw, "", XADN(R3, C2), "") \
           R2(R2, R1, R0, R3, C1, C3, kw, "", XADN(R0, C3), "") R2(R3, R2, R1, R0, C2, C0, kw, "", XADN(R1, C0), "")
// variant 3: xad right after the V DPP (shields the DPP result), s_nop 0 before the V DPP
#define Q3 R2(R0, R3, R2, R1, C3, C1, kw, "", "s_nop 0\n\t", XADN(R2, C1)) R2(R1, R0, R3, R2, C0, C2, kw, "", "s_nop 0\n\t", XADN(R3, C2)) \
           R2(R2, R1, R0, R3, C1, C3, kw, "", "s_nop 0\n\t", XADN(R0, C3)) R2(R3, R2, R1, R0, C2, C0, kw, "", "s_nop 0\n\t", XADN(R1, C0))
// variant 4: production order + s_nop 0 after the V DPP
#define Q4 R2(R0, R3, R2, R1, C3, C1, kw, "", XADN(R2, C1), "s_nop 0\n\t") R2(R1, R0, R3, R2, C0, C2, kw, "", XADN(R3, C2), "s_nop 0\n\t") \
           R2(R2, R1, R0, R3, C1, C3, kw, "", XADN(R0, C3), "s_nop 0\n\t") R2(R3, R2, R1, R0, C2, C0, kw, "", XADN(R1, C0), "s_nop 0\n\t")

// variant 5: production order, V combine without DPP (prices the DPP latency)
#define R5(X0, X1, X2, V, CW, CR, KWN)                                                   \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                          \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                          \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                          \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_add3_u32 %[" #V "], %[t1], %[k], %[p]\n\t"                                      \
    XADN(X2, CR)                                                                       \
    "v_add_u32_dpp %[" #CW "], %[" #X0 "], %[" #KWN "] row_shr:4 row_mask:0xf bank_mask:0xa\n\t" \
    "v_add_u32_e32 %[" #V "], %[" #V "], %[" #V "]\n\t"
#define Q5 R5(R0, R3, R2, R1, C3, C1, kw) R5(R1, R0, R3, R2, C0, C2, kw) R5(R2, R1, R0, R3, C1, C3, kw) R5(R3, R2, R1, R0, C2, C0, kw)

// variant 6: skewed lanes (E runs round n while A runs round n-1): DPPs off the chain
#define R6(X0, X1, X2, X3)                                                               \
    "v_add_u32_e32 %[y], %[" #X3 "], %[kw]\n\t"                                         \
    "v_add_u32_dpp %[p], %[" #X2 "], %[y] row_shr:4 row_mask:0xf bank_mask:0xa\n\t"     \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                          \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                          \
    "v_sub_u32_dpp %[p], %[" #X0 "], %[" #X3 "] row_shl:4 row_mask:0xf bank_mask:0x5\n\t" \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                          \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_add3_u32 %[" #X3 "], %[t1], %[k], %[p]\n\t"
#define Q6 R6(R0, R3, R2, R1) R6(R1, R0, R3, R2) R6(R2, R1, R0, R3) R6(R3, R2, R1, R0)

// variant 7: skew-2 lanes, one unmasked row_mirror DPP per round (production)
#define R7(X0, X1, X2, X3)                                                               \
    "v_xad_u32 %[y], %[" #X3 "], %[ma], %[kw]\n\t"                                     \
    "v_add_u32_dpp %[p], %[" #X1 "], %[y] row_mirror row_mask:0xf bank_mask:0xf\n\t"   \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                          \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                          \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                          \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_add3_u32 %[" #X3 "], %[t1], %[k], %[p]\n\t"
#define Q7 R7(R0, R3, R2, R1) R7(R1, R0, R3, R2) R7(R2, R1, R0, R3) R7(R3, R2, R1, R0)

// variant 8: skew-2, z for the next round formed at the end of this one (no xad -> DPP back-to-back)
#define R8(X0, X1, X2, X3)                                                               \
    "v_add_u32_dpp %[p], %[" #X1 "], %[y] row_mirror row_mask:0xf bank_mask:0xf\n\t"   \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                          \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                          \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                          \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_xad_u32 %[y], %[" #X2 "], %[ma], %[kw]\n\t"                                     \
    "v_add3_u32 %[" #X3 "], %[t1], %[k], %[p]\n\t"
#define Q8 R8(R0, R3, R2, R1) R8(R1, R0, R3, R2) R8(R2, R1, R0, R3) R8(R3, R2, R1, R0)
// variant 9: as 7 with a VOP2 add in place of the xad (timing only: is it VOP3 -> DPP?)
#define R9(X0, X1, X2, X3)                                                               \
    "v_add_u32_e32 %[y], %[" #X3 "], %[kw]\n\t"                                         \
    "v_add_u32_dpp %[p], %[" #X1 "], %[y] row_mirror row_mask:0xf bank_mask:0xf\n\t"   \
    "v_alignbit_b32 %[t1], %[" #X0 "], %[" #X0 "], %[r1]\n\t"                          \
    "v_alignbit_b32 %[t2], %[" #X0 "], %[" #X0 "], %[r2]\n\t"                          \
    "v_alignbit_b32 %[t3], %[" #X0 "], %[" #X0 "], %[r3]\n\t"                          \
    "v_bitop3_b32 %[k], %[" #X0 "], %[" #X1 "], %[ma] bitop3:0x2d\n\t"                 \
    "v_bitop3_b32 %[t1], %[t1], %[t2], %[t3] bitop3:0x96\n\t"                          \
    "v_bitop3_b32 %[k], %[k], %[" #X2 "], %[" #X1 "] bitop3:0xca\n\t"                  \
    "v_add3_u32 %[" #X3 "], %[t1], %[k], %[p]\n\t"
#define Q9 R9(R0, R3, R2, R1) R9(R1, R0, R3, R2) R9(R2, R1, R0, R3) R9(R3, R2, R1, R0)

template <int K>
__global__ void quads(unsigned long long* out, unsigned* sink) {
    unsigned long long t0, t1, rt0, rt1;
    rt0 = __builtin_amdgcn_s_memrealtime();
    const unsigned l = threadIdx.x;
    unsigned R0 = l, R1 = 2 * l, R2v = 3 * l, R3 = 5 * l, C0 = 1, C1 = 1, C2 = 1, C3 = 1, p = 7, kw = 19;
    unsigned a, b, c, k;
    const unsigned r1 = (l & 4) ? 6 : 2, r2 = (l & 4) ? 11 : 13, r3 = (l & 4) ? 25 : 22;
    const unsigned ma = (l & 4) ? 0u : ~0u;
    t0 = __builtin_amdgcn_s_memtime();
#define QUAD_ASM(Q) asm volatile(REP16(Q)                                                                  \
                     : [t1] "=&v"(a), [t2] "=&v"(b), [t3] "=&v"(c), [k] "=&v"(k), [R0] "+v"(R0),       \
                       [R1] "+v"(R1), [R2] "+v"(R2v), [R3] "+v"(R3), [C0] "+v"(C0), [C1] "+v"(C1),     \
                       [C2] "+v"(C2), [C3] "+v"(C3), [p] "+v"(p)                                        \
                     : [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [ma] "v"(ma), [kw] "v"(kw))
    if (K == 2) QUAD_ASM(Q2);
    if (K == 3) QUAD_ASM(Q3);
    if (K == 4) QUAD_ASM(Q4);
    if (K == 5) QUAD_ASM(Q5);
    unsigned y;
#define QY(Q) asm volatile(REP16(Q)                                                                 \
                     : [t1] "=&v"(a), [t2] "=&v"(b), [t3] "=&v"(c), [k] "=&v"(k), [y] "+v"(y), [R0] "+v"(R0), \
                       [R1] "+v"(R1), [R2] "+v"(R2v), [R3] "+v"(R3), [p] "+v"(p)                               \
                     : [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [ma] "v"(ma), [kw] "v"(kw))
    y = 3;
    if (K == 8)
        for (int it = 0; it < 256; ++it) QY(Q8);
    if (K == 9) QY(Q9);
    if (K == 7)
        asm volatile(REP16(Q7)
                     : [t1] "=&v"(a), [t2] "=&v"(b), [t3] "=&v"(c), [k] "=&v"(k), [y] "=&v"(y), [R0] "+v"(R0),
                       [R1] "+v"(R1), [R2] "+v"(R2v), [R3] "+v"(R3), [p] "+v"(p)
                     : [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [ma] "v"(ma), [kw] "v"(kw));
    if (K == 6)
        asm volatile(REP16(Q6)
                     : [t1] "=&v"(a), [t2] "=&v"(b), [t3] "=&v"(c), [k] "=&v"(k), [y] "=&v"(y), [R0] "+v"(R0),
                       [R1] "+v"(R1), [R2] "+v"(R2v), [R3] "+v"(R3), [p] "+v"(p)
                     : [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [ma] "v"(ma), [kw] "v"(kw));
    t1 = __builtin_amdgcn_s_memtime();
    rt1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = rt1 - rt0;
    }
    sink[l] = R0 + R1 + R2v + R3 + C0 + C1 + C2 + C3 + p;
}

int main() {
    unsigned long long* d;
    unsigned *sink, *sem;
    hipMalloc(&d, 16);
    hipMalloc(&sink, 256 * 4);
    hipMalloc(&sem, 192 * 4);
    hipLaunchKernelGGL(dpp_semantics, 1, 64, 0, 0, sem);
    unsigned hs[192];
    hipMemcpy(hs, sem, sizeof hs, hipMemcpyDeviceToHost);
    printf("row_shl:4 bank_mask:0x5 (lane: value)  ");
    for (int i = 0; i < 32; ++i) printf("%d:%u ", i, hs[i]);
    printf("\nrow_shr:4 bank_mask:0xa (lane: value)  ");
    for (int i = 0; i < 32; ++i) printf("%d:%u ", i, hs[64 + i]);
    printf("\nrow_mirror (lane: value)  ");
    for (int i = 0; i < 32; ++i) printf("%d:%u ", i, hs[128 + i]);
    printf("\n");
    for (int rep = 0; rep < 2; ++rep) {
        const char* names[] = {"v_add_u32_dpp", "v_xad_u32", "v_add3_u32"};
        for (int k = 0; k < 3; ++k) {
            if (k == 0) hipLaunchKernelGGL(cost<0>, 1, 64, 0, 0, d, sink);
            if (k == 1) hipLaunchKernelGGL(cost<1>, 1, 64, 0, 0, d, sink);
            if (k == 2) hipLaunchKernelGGL(cost<2>, 1, 64, 0, 0, d, sink);
            unsigned long long c = 0;
            hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
            if (rep) printf("%-24s %.2f cycles/instr\n", names[k], c / 256.0);
        }
        for (int k = 0; k < 2; ++k) {
            if (k == 0) hipLaunchKernelGGL(rounds<0>, 1, 64, 0, 0, d, sink);
            if (k == 1) hipLaunchKernelGGL(rounds<1>, 1, 64, 0, 0, d, sink);
            unsigned long long c = 0;
            hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
            if (rep) printf("%-24s %.2f cycles/round\n", k ? "two-lane round (10 ops)" : "one-lane round (14 ops)", c / 64.0);
        }
        for (int k = 2; k < 10; ++k) {
            if (k == 2) hipLaunchKernelGGL(quads<2>, 1, 64, 0, 0, d, sink);
            if (k == 3) hipLaunchKernelGGL(quads<3>, 1, 64, 0, 0, d, sink);
            if (k == 4) hipLaunchKernelGGL(quads<4>, 1, 64, 0, 0, d, sink);
            if (k == 5) hipLaunchKernelGGL(quads<5>, 1, 64, 0, 0, d, sink);
            if (k == 6) hipLaunchKernelGGL(quads<6>, 1, 64, 0, 0, d, sink);
            if (k == 7) hipLaunchKernelGGL(quads<7>, 1, 64, 0, 0, d, sink);
            if (k == 8) hipLaunchKernelGGL(quads<8>, 1, 64, 0, 0, d, sink);
            if (k == 9) hipLaunchKernelGGL(quads<9>, 1, 64, 0, 0, d, sink);
            unsigned long long c = 0;
            hipMemcpy(&c, d, 8, hipMemcpyDeviceToHost);
            unsigned long long rt = 0;
            hipMemcpy(&rt, d + 1, 8, hipMemcpyDeviceToHost);
            if (k == 8) c /= 256;
            if (rep && k == 8) printf("clock during quads<8>: %.3f GHz (s_memtime %llu cycles / s_memrealtime %llu x 10 ns)\n", c * 256 / (rt * 10.0), c * 256, rt);
            const char* nm[] = {"", "", "dep quads, production", "dep quads, xad after DPP", "dep quads, nop after DPP", "dep quads, plain V add", "dep quads, skewed lanes", "dep quads, skew-2 mirror", "skew-2, z a round early", "skew-2, VOP2 z (timing)"};
            if (rep) printf("%-28s %.2f cycles/round\n", nm[k], c / 64.0);
        }
    }
    return 0;
}
