// Micro-benchmark: do f16 MFMAs (the matrix cores) run beside packed-fp32
// VALU work on gfx950? (tools/ubench/valu_mfma.hip measured the f32
// v_mfma_f32_4x4x1f32: no overlap.) Loop bodies per wave per iteration, every
// CU busy, W waves per SIMD:
//   V: 16 v_pk_fma_f32 (16 independent register pairs)
//   M: K v_mfma_f32_32x32x16_f16 on 2 independent accumulators
//   X: V and M in the same wave, interleaved
//   S: even waves V only, odd waves 2x M only (same total work as X per wave pair)
// Reported: ms of the timed launch; X ~ max(V, M) means the pipes overlap.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

#define PK(i) "v_pk_fma_f32 %" #i ", %" #i ", %16, %17\n"
#define PK4(a, b, c, d) PK(a) PK(b) PK(c) PK(d)
#define PKOUT "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7), \
              "+v"(p8), "+v"(p9), "+v"(p10), "+v"(p11), "+v"(p12), "+v"(p13), "+v"(p14), "+v"(p15)
#define MF(acc) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, hb, acc, 0, 0, 0)

template <int MODE, int K>
__global__ __launch_bounds__(256) void kern(float* out, int iters) {
    const float t = threadIdx.x * 1e-3f;
    f2 p0 = {t, t + 1}, p1 = p0 + 1, p2 = p0 + 2, p3 = p0 + 3, p4 = p0 + 4, p5 = p0 + 5,
       p6 = p0 + 6, p7 = p0 + 7, p8 = p0 + 8, p9 = p0 + 9, p10 = p0 + 10, p11 = p0 + 11,
       p12 = p0 + 12, p13 = p0 + 13, p14 = p0 + 14, p15 = p0 + 15;
    f2 mm = {0.999f, 0.999f}, cc = {1e-3f, 1e-3f};
    h8 ha, hb;
    for (int i = 0; i < 8; ++i) {
        ha[i] = (_Float16)(t + i);
        hb[i] = (_Float16)(1e-3f * i);
    }
    asm volatile("" : "+v"(mm), "+v"(cc), "+v"(ha), "+v"(hb));
    f16v a0 = {}, a1 = {};
    a0[0] = t;
    const bool valu_wave = ((threadIdx.x >> 6) & 1) == 0;
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {
            asm volatile(PK4(0, 1, 2, 3) PK4(4, 5, 6, 7) PK4(8, 9, 10, 11) PK4(12, 13, 14, 15)
                         : PKOUT : "v"(mm), "v"(cc));
        } else if (MODE == 1) {
            for (int k = 0; k < K; k += 2) { MF(a0); MF(a1); }
        } else if (MODE == 2) {  // interleaved in one wave
            if (K >= 4) {
                MF(a0);
                asm volatile(PK4(0, 1, 2, 3) : PKOUT : "v"(mm), "v"(cc));
                MF(a1);
                asm volatile(PK4(4, 5, 6, 7) : PKOUT : "v"(mm), "v"(cc));
                MF(a0);
                asm volatile(PK4(8, 9, 10, 11) : PKOUT : "v"(mm), "v"(cc));
                MF(a1);
                asm volatile(PK4(12, 13, 14, 15) : PKOUT : "v"(mm), "v"(cc));
            } else {
                MF(a0);
                asm volatile(PK4(0, 1, 2, 3) PK4(4, 5, 6, 7) : PKOUT : "v"(mm), "v"(cc));
                MF(a1);
                asm volatile(PK4(8, 9, 10, 11) PK4(12, 13, 14, 15) : PKOUT : "v"(mm), "v"(cc));
            }
        } else {  // split by wave: VALU waves and MFMA waves
            if (valu_wave) {
                asm volatile(PK4(0, 1, 2, 3) PK4(4, 5, 6, 7) PK4(8, 9, 10, 11) PK4(12, 13, 14, 15)
                             PK4(0, 1, 2, 3) PK4(4, 5, 6, 7) PK4(8, 9, 10, 11) PK4(12, 13, 14, 15)
                             : PKOUT : "v"(mm), "v"(cc));
            } else {
                for (int k = 0; k < 2 * K; k += 2) { MF(a0); MF(a1); }
            }
        }
    }
    f2 s = p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7 + p8 + p9 + p10 + p11 + p12 + p13 + p14 + p15;
    float q = 0.0f;
    for (int i = 0; i < 16; ++i) q += a0[i] + a1[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s.x + s.y + q;
}

template <int MODE, int K>
float run(int W, int iters) {
    const int blocks = 256 * W;
    float* d;
    (void)hipMalloc(&d, (size_t)blocks * 256 * 4);
    hipLaunchKernelGGL((kern<MODE, K>), blocks, 256, 0, 0, d, iters / 10);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((kern<MODE, K>), blocks, 256, 0, 0, d, iters);
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
    const int iters = 20000;
    for (int W : {2, 3, 4, 6}) {
        const float V = run<0, 4>(W, iters);
        const float M2 = run<1, 2>(W, iters), X2 = run<2, 2>(W, iters), S2 = run<3, 2>(W, iters);
        const float M4 = run<1, 4>(W, iters), X4 = run<2, 4>(W, iters), S4 = run<3, 4>(W, iters);
        const double it = (double)W * iters;  // iterations per SIMD
        const double ghz = 2.4;
        printf("W=%d  V 16pk %.2f ms (%.2f cyc/pk) | M 2mfma %.2f ms (%.1f cyc/mfma)  X %.2f  "
               "S %.2f  (V+M=%.2f) | M 4mfma %.2f ms (%.1f cyc/mfma)  X %.2f  S %.2f  (V+M=%.2f)\n",
               W, V, V * 1e6 * ghz / it / 16, M2, M2 * 1e6 * ghz / it / 2, X2, S2, V + M2, M4,
               M4 * 1e6 * ghz / it / 4, X4, S4, V + M4);
    }
    return 0;
}
