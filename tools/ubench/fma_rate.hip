// Micro-benchmark: v_fma_f32 vs v_pk_fma_f32 issue rate on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_fma(float* out, float a, float b, int iters) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            x0 = __builtin_fmaf(x0, a, b); x1 = __builtin_fmaf(x1, a, b); x2 = __builtin_fmaf(x2, a, b); x3 = __builtin_fmaf(x3, a, b);
            x4 = __builtin_fmaf(x4, a, b); x5 = __builtin_fmaf(x5, a, b); x6 = __builtin_fmaf(x6, a, b); x7 = __builtin_fmaf(x7, a, b);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}
__global__ __launch_bounds__(256) void k_pk(float* out, float a, float b, int iters) {
    f2 x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    f2 va = {a, a}, vb = {b, b};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            x0 = __builtin_elementwise_fma(x0, va, vb); x1 = __builtin_elementwise_fma(x1, va, vb);
            x2 = __builtin_elementwise_fma(x2, va, vb); x3 = __builtin_elementwise_fma(x3, va, vb);
        }
    }
    f2 s = x0 + x1 + x2 + x3;
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}
int main() {
    float* d; hipMalloc(&d, 256 * 8192 * 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int iters = 4096; int grid = 256 * 8;
    for (int rep = 0; rep < 3; ++rep) {
        float ms;
        hipEventRecord(e0); hipLaunchKernelGGL(k_fma, grid, 256, 0, 0, d, 0.999f, 0.001f, iters); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        double fl = 2.0 * 8 * 8 * (double)iters * grid * 256;
        printf("v_fma_f32   : %.3f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
        hipEventRecord(e0); hipLaunchKernelGGL(k_pk, grid, 256, 0, 0, d, 0.999f, 0.001f, iters); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
        printf("v_pk_fma_f32: %.3f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
    }
    return 0;
}
