// Micro-benchmark: can the MFMA pipe take work off the VALU on gfx950?
// Loop bodies (per wave per iteration), every CU busy, W waves per SIMD:
//   A: 16 v_pk_fma_f32            (16 independent register pairs)
//   D: 32 v_fma_f32               (same flops as A, 32 independent registers)
//   B:  8 v_mfma_f32_4x4x1_16b_f32 (4 independent accumulators)
//   C: A and B interleaved (2 pk_fma per MFMA)
//   E: 16 pk_fma + 4 MFMA (4 pk_fma per MFMA)
// Operands live in loop-carried registers (no per-iteration moves). Reported:
// wall ms of the timed launch (relative costs are what matter: C vs A + B
// says whether the two pipes overlap).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

#define PK(i) "v_pk_fma_f32 %" #i ", %" #i ", %16, %17\n"
#define PK16 PK(0) PK(1) PK(2) PK(3) PK(4) PK(5) PK(6) PK(7) PK(8) PK(9) PK(10) PK(11) PK(12) PK(13) PK(14) PK(15)
#define PKOUT "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7), \
              "+v"(p8), "+v"(p9), "+v"(p10), "+v"(p11), "+v"(p12), "+v"(p13), "+v"(p14), "+v"(p15)
#define MF(acc, x, y) acc = __builtin_amdgcn_mfma_f32_4x4x1f32(x, y, acc, 0, 0, 0)

template <int MODE>
__global__ __launch_bounds__(256) void kern(float* out, int iters) {
    const float t = threadIdx.x * 1e-3f;
    f2 p0 = {t, t + 1}, p1 = p0 + 1, p2 = p0 + 2, p3 = p0 + 3, p4 = p0 + 4, p5 = p0 + 5,
       p6 = p0 + 6, p7 = p0 + 7, p8 = p0 + 8, p9 = p0 + 9, p10 = p0 + 10, p11 = p0 + 11,
       p12 = p0 + 12, p13 = p0 + 13, p14 = p0 + 14, p15 = p0 + 15;
    f2 mm = {0.999f, 0.999f}, cc = {1e-3f, 1e-3f};
    float x = t + 0.5f, y = t + 0.25f;
    asm volatile("" : "+v"(mm), "+v"(cc), "+v"(x), "+v"(y));
    f4 a0 = {t, t, t, t}, a1 = a0 + 1.f, a2 = a0 + 2.f, a3 = a0 + 3.f;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            asm volatile(PK16 : PKOUT : "v"(mm), "v"(cc));
        } else if (MODE == 1) {  // 32 v_fma_f32 on the 32 halves
            asm volatile(
#define F(i) "v_fma_f32 %" #i ", %" #i ", %32, %33\n"
                F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7) F(8) F(9) F(10) F(11) F(12) F(13) F(14) F(15)
                F(16) F(17) F(18) F(19) F(20) F(21) F(22) F(23) F(24) F(25) F(26) F(27) F(28) F(29)
                F(30) F(31)
#undef F
                : "+v"(p0.x), "+v"(p0.y), "+v"(p1.x), "+v"(p1.y), "+v"(p2.x), "+v"(p2.y),
                  "+v"(p3.x), "+v"(p3.y), "+v"(p4.x), "+v"(p4.y), "+v"(p5.x), "+v"(p5.y),
                  "+v"(p6.x), "+v"(p6.y), "+v"(p7.x), "+v"(p7.y), "+v"(p8.x), "+v"(p8.y),
                  "+v"(p9.x), "+v"(p9.y), "+v"(p10.x), "+v"(p10.y), "+v"(p11.x), "+v"(p11.y),
                  "+v"(p12.x), "+v"(p12.y), "+v"(p13.x), "+v"(p13.y), "+v"(p14.x), "+v"(p14.y),
                  "+v"(p15.x), "+v"(p15.y)
                : "v"(mm.x), "v"(cc.x));
        } else if (MODE == 2) {
            MF(a0, x, y); MF(a1, x, y); MF(a2, x, y); MF(a3, x, y);
            MF(a0, x, y); MF(a1, x, y); MF(a2, x, y); MF(a3, x, y);
        } else if (MODE == 3) {  // 8 MFMA + 16 pk_fma interleaved
            MF(a0, x, y);
            asm volatile(PK(0) PK(1) : PKOUT : "v"(mm), "v"(cc));
            MF(a1, x, y);
            asm volatile(PK(2) PK(3) : PKOUT : "v"(mm), "v"(cc));
            MF(a2, x, y);
            asm volatile(PK(4) PK(5) : PKOUT : "v"(mm), "v"(cc));
            MF(a3, x, y);
            asm volatile(PK(6) PK(7) : PKOUT : "v"(mm), "v"(cc));
            MF(a0, x, y);
            asm volatile(PK(8) PK(9) : PKOUT : "v"(mm), "v"(cc));
            MF(a1, x, y);
            asm volatile(PK(10) PK(11) : PKOUT : "v"(mm), "v"(cc));
            MF(a2, x, y);
            asm volatile(PK(12) PK(13) : PKOUT : "v"(mm), "v"(cc));
            MF(a3, x, y);
            asm volatile(PK(14) PK(15) : PKOUT : "v"(mm), "v"(cc));
        } else {  // 4 MFMA + 16 pk_fma
            MF(a0, x, y);
            asm volatile(PK(0) PK(1) PK(2) PK(3) : PKOUT : "v"(mm), "v"(cc));
            MF(a1, x, y);
            asm volatile(PK(4) PK(5) PK(6) PK(7) : PKOUT : "v"(mm), "v"(cc));
            MF(a2, x, y);
            asm volatile(PK(8) PK(9) PK(10) PK(11) : PKOUT : "v"(mm), "v"(cc));
            MF(a3, x, y);
            asm volatile(PK(12) PK(13) PK(14) PK(15) : PKOUT : "v"(mm), "v"(cc));
        }
    }
    f2 s = p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7 + p8 + p9 + p10 + p11 + p12 + p13 + p14 + p15;
    f4 q = a0 + a1 + a2 + a3;
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y + q.x + q.y + q.z + q.w;
}

template <int MODE>
float run(int W, int iters) {
    const int blocks = 256 * W;
    float* d;
    (void)hipMalloc(&d, (size_t)blocks * 256 * 4);
    hipLaunchKernelGGL(kern<MODE>, blocks, 256, 0, 0, d, iters / 10);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(kern<MODE>, blocks, 256, 0, 0, d, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    (void)hipFree(d);
    return best;
}

int main() {
    const int iters = 40000;
    for (int W : {2, 4, 6}) {
        const float A = run<0>(W, iters), D = run<1>(W, iters), B = run<2>(W, iters);
        const float C = run<3>(W, iters), E = run<4>(W, iters);
        // per SIMD: W waves x iters iterations
        const double it = (double)W * iters;
        const double ghz = 2.1;  // nominal, for a cycles view only
        printf("W=%d  A 16pk %.2f ms (%.2f cyc/pk)  D 32fma %.2f ms (%.2f cyc/fma)  "
               "B 8mfma %.2f ms (%.2f cyc/mfma)  C A+B interleaved %.2f ms (A+B=%.2f)  "
               "E 16pk+4mfma %.2f ms\n",
               W, A, A * 1e6 * ghz / it / 16, D, D * 1e6 * ghz / it / 32, B,
               B * 1e6 * ghz / it / 8, C, A + B, E);
    }
    return 0;
}
