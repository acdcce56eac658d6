// How gfx950's SQ counters see v_mfma_f32_32x32x16_f16 (for bench.py's SIMD
// issue roofline): does SQ_INSTS_VALU count MFMAs, what do SQ_ACTIVE_INST_VALU
// and SQ_VALU_MFMA_BUSY_CYCLES add per MFMA, and how many cycles of a SIMD's
// vector issue does one MFMA hold next to VALU work. Kernels (256 threads,
// 4 waves per SIMD like rt_render_kernel, fixed iteration counts):
//   k_mfma   8 independent MFMAs per iteration (matrix pipe bound)
//   k_fma    8 independent v_fma_f32 per iteration (VALU issue bound)
//   k_mix    1 MFMA + 8 v_fma_f32 per iteration
// Run under rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA
// SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F16
// GRBM_GUI_ACTIVE -- ./mfma_count ; tools/mfma_count.py reads the csv.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16x __attribute__((ext_vector_type(16)));
#define ITERS 4096

__global__ __launch_bounds__(256) void k_mfma(float* out) {
    h8v a, b;
    for (int k = 0; k < 8; ++k) {
        a[k] = (_Float16)(0.001f * (float)((threadIdx.x + k) & 7));
        b[k] = (_Float16)(0.001f * (float)((threadIdx.x * 3 + k) & 7));
    }
    f16x c0 = {}, c1 = {}, c2 = {}, c3 = {};
    for (int i = 0; i < ITERS; ++i) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, b, c3, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, b, c3, 0, 0, 0);
    }
    float s = 0.f;
    for (int k = 0; k < 16; ++k) s += c0[k] + c1[k] + c2[k] + c3[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fma(float* out, float a) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
          x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_fma_f32 %0, %0, %8, %8\n\tv_fma_f32 %1, %1, %8, %8\n\t"
            "v_fma_f32 %2, %2, %8, %8\n\tv_fma_f32 %3, %3, %8, %8\n\t"
            "v_fma_f32 %4, %4, %8, %8\n\tv_fma_f32 %5, %5, %8, %8\n\t"
            "v_fma_f32 %6, %6, %8, %8\n\tv_fma_f32 %7, %7, %8, %8"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(a));
    }
    out[blockIdx.x * 256 + threadIdx.x] = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
}

__global__ __launch_bounds__(256) void k_mix(float* out, float a) {
    h8v p, q;
    for (int k = 0; k < 8; ++k) {
        p[k] = (_Float16)(0.001f * (float)((threadIdx.x + k) & 7));
        q[k] = (_Float16)(0.001f * (float)((threadIdx.x * 3 + k) & 7));
    }
    f16x c = {};
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
          x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < ITERS; ++i) {
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(p, q, c, 0, 0, 0);
        asm volatile(
            "v_fma_f32 %0, %0, %8, %8\n\tv_fma_f32 %1, %1, %8, %8\n\t"
            "v_fma_f32 %2, %2, %8, %8\n\tv_fma_f32 %3, %3, %8, %8\n\t"
            "v_fma_f32 %4, %4, %8, %8\n\tv_fma_f32 %5, %5, %8, %8\n\t"
            "v_fma_f32 %6, %6, %8, %8\n\tv_fma_f32 %7, %7, %8, %8"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(a));
    }
    float s = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
    for (int k = 0; k < 16; ++k) s += c[k];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const unsigned blocks = ncu * 4;  // 16 waves per CU = 4 per SIMD
    float* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        float ms[3];
        for (int k = 0; k < 3; ++k) {
            hipEventRecord(e0);
            if (k == 0) hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, out);
            if (k == 1) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
            if (k == 2) hipLaunchKernelGGL(k_mix, dim3(blocks), dim3(256), 0, 0, out, 1.0f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms[k], e0, e1);
        }
        // instructions per SIMD: 4 waves x ITERS x per-iteration count
        const double per_simd = 4.0 * ITERS;
        printf("rep %d: k_mfma %.3f ms (%.2f ns per MFMA per SIMD), k_fma %.3f ms (%.2f ns per "
               "v_fma), k_mix %.3f ms (%.2f ns per iteration)\n",
               rep, ms[0], ms[0] * 1e6 / (per_simd * 8), ms[1], ms[1] * 1e6 / (per_simd * 8), ms[2],
               ms[2] * 1e6 / per_simd);
    }
    return 0;
}
