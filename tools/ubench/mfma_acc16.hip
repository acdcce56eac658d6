// Accuracy and operand layout of v_mfma_f32_16x16x32_f16 (32 products in one
// instruction) and v_mfma_f32_16x16x16f16 on gfx950 -- the hardware
// assumptions of a 16 x 16 form of the matrix-core filter (the margin proof
// allows <= 33 roundings of <= 2^-24 sum |p| each, rt_dev_intersect.h). Random
// f16 operands with mixed signs and exponents in [-6, 6], every product exact
// in f32 and every sum exact in double. Layout (cdna_hip_programming.md):
// lane l holds A[row l & 15][k = 8 (l >> 4) + j] and B[k = 8 (l >> 4) + j][col
// l & 15] (16x16x16: k = 4 (l >> 4) + j); D: col l & 15, row 4 (l >> 4) + i.
// A wrong layout shows as ratios far above the allowance.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef _Float16 h4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));

// per tile: A 16 x 32 row-major, B 32 x 16 row-major (k, col)
__global__ void tiles(const _Float16* A, const _Float16* B, float* D32, float* D16, int ntiles) {
    const int l = threadIdx.x, t = blockIdx.x;
    if (t >= ntiles) return;
    const _Float16* a = A + (size_t)t * 512;
    const _Float16* b = B + (size_t)t * 512;
    h8v a8, b8;
    h4v a4, b4;
    for (int j = 0; j < 8; ++j) {
        const int k = 8 * (l >> 4) + j;
        a8[j] = a[(l & 15) * 32 + k];
        b8[j] = b[k * 16 + (l & 15)];
    }
    for (int j = 0; j < 4; ++j) {  // 16x16x16: K 0..15 of the same tile
        const int k = 4 * (l >> 4) + j;
        a4[j] = a[(l & 15) * 32 + k];
        b4[j] = b[k * 16 + (l & 15)];
    }
    const f4v z = {};
    const f4v d32 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, z, 0, 0, 0);
    const f4v d16 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, z, 0, 0, 0);
    for (int i = 0; i < 4; ++i) {
        const int row = 4 * (l >> 4) + i, col = l & 15;
        D32[(size_t)t * 256 + row * 16 + col] = d32[i];
        D16[(size_t)t * 256 + row * 16 + col] = d16[i];
    }
}

int main() {
    const int ntiles = 16384;
    std::mt19937 rng(12345);
    std::uniform_real_distribution<double> m(1.0, 2.0);
    std::uniform_int_distribution<int> e(-6, 6), s(0, 1);
    std::vector<_Float16> A((size_t)ntiles * 512), B((size_t)ntiles * 512);
    for (auto* v : {&A, &B})
        for (auto& x : *v) x = (_Float16)((s(rng) ? -1.0 : 1.0) * std::ldexp(m(rng), e(rng)));
    _Float16 *dA, *dB;
    float *dD32, *dD16;
    (void)hipMalloc(&dA, A.size() * 2);
    (void)hipMalloc(&dB, B.size() * 2);
    (void)hipMalloc(&dD32, (size_t)ntiles * 256 * 4);
    (void)hipMalloc(&dD16, (size_t)ntiles * 256 * 4);
    (void)hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(tiles, ntiles, 64, 0, 0, dA, dB, dD32, dD16, ntiles);
    std::vector<float> D32((size_t)ntiles * 256), D16((size_t)ntiles * 256);
    (void)hipMemcpy(D32.data(), dD32, D32.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(D16.data(), dD16, D16.size() * 4, hipMemcpyDeviceToHost);
    double w32 = 0, w16 = 0;
    long rn32 = 0, rn16 = 0, n = 0;
    for (int t = 0; t < ntiles; ++t)
        for (int r = 0; r < 16; ++r)
            for (int c = 0; c < 16; ++c) {
                double ex32 = 0, ab32 = 0, ex16 = 0, ab16 = 0;
                for (int k = 0; k < 32; ++k) {
                    const double p = (double)A[(size_t)t * 512 + r * 32 + k] * (double)B[(size_t)t * 512 + k * 16 + c];
                    ex32 += p;
                    ab32 += std::fabs(p);
                    if (k < 16) {
                        ex16 += p;
                        ab16 += std::fabs(p);
                    }
                }
                const size_t i = (size_t)t * 256 + r * 16 + c;
                w32 = std::max(w32, std::fabs(D32[i] - ex32) / std::ldexp(ab32, -24));
                w16 = std::max(w16, std::fabs(D16[i] - ex16) / std::ldexp(ab16, -24));
                rn32 += D32[i] == (float)ex32;
                rn16 += D16[i] == (float)ex16;
                ++n;
            }
    printf("16x16x32 (32 products): worst |D - exact| / (2^-24 sum|p|) = %.3f, D == RN(exact) for %.4f of %ld\n",
           w32, (double)rn32 / n, n);
    printf("16x16x16 (16 products): worst ratio = %.3f, D == RN(exact) for %.4f\n", w16, (double)rn16 / n);
    printf("allowance 33 (32 products), 17 (16): %s\n", (w32 <= 33.0 && w16 <= 17.0) ? "holds" : "VIOLATED");
    return 0;
}
