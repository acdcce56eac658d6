// Accuracy of v_mfma_f32_32x32x16_f16's 16-product f32 sums on gfx950 -- the
// hardware assumption of the matrix-core filter's margin proof
// (rt_dev_intersect.h: "the f32 sums of the exact products add <= 31 * 2^-24
// of their magnitudes" over two chained MFMAs). Random f16 operands with
// mixed signs and exponents in [-6, 6] (cancellation-heavy), so every product
// is exact in f32 and every 16/32-term sum exact in double. Per tile element:
// err = |D - exact| / (2^-24 * sum |a_k b_k|). Reports the worst ratio for one
// MFMA (C = 0) and for two chained (C = the first's D), and the share of
// elements equal to RN_f32(exact). The proof needs ratio <= 15 (one MFMA) and
// <= 31 (two chained).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16x __attribute__((ext_vector_type(16)));

// A: 32 rows x 32 K (two K groups), B: 32 K x 32 columns, per tile, row-major
// host arrays; lane l holds row/column l & 31, K 8 (l >> 5) .. + 8 of a group.
__global__ void tiles(const _Float16* A, const _Float16* B, float* D1, float* D2, int ntiles) {
    const int l = threadIdx.x, t = blockIdx.x;
    if (t >= ntiles) return;
    const _Float16* a = A + (size_t)t * 32 * 32;
    const _Float16* b = B + (size_t)t * 32 * 32;
    h8v a0, a1, b0, b1;
    for (int i = 0; i < 8; ++i) {
        const int k = 8 * (l >> 5) + i;
        a0[i] = a[(l & 31) * 32 + k];
        a1[i] = a[(l & 31) * 32 + 16 + k];
        b0[i] = b[k * 32 + (l & 31)];
        b1[i] = b[(16 + k) * 32 + (l & 31)];
    }
    const f16x z = {};
    const f16x d1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, z, 0, 0, 0);
    const f16x d2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b1, d1, 0, 0, 0);
    for (int i = 0; i < 16; ++i) {  // row (i & 3) + 8 (i >> 2) + 4 (l >> 5), column l & 31
        const int row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5), col = l & 31;
        D1[(size_t)t * 1024 + row * 32 + col] = d1[i];
        D2[(size_t)t * 1024 + row * 32 + col] = d2[i];
    }
}

int main() {
    const int ntiles = 4096;
    std::mt19937 rng(12345);
    std::uniform_real_distribution<double> m(1.0, 2.0);
    std::uniform_int_distribution<int> e(-6, 6), s(0, 1);
    std::vector<_Float16> A((size_t)ntiles * 1024), B((size_t)ntiles * 1024);
    for (auto* v : {&A, &B})
        for (auto& x : *v) x = (_Float16)((s(rng) ? -1.0 : 1.0) * std::ldexp(m(rng), e(rng)));
    _Float16 *dA, *dB;
    float *dD1, *dD2;
    (void)hipMalloc(&dA, A.size() * 2);
    (void)hipMalloc(&dB, B.size() * 2);
    (void)hipMalloc(&dD1, A.size() * 4);
    (void)hipMalloc(&dD2, A.size() * 4);
    (void)hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(tiles, ntiles, 64, 0, 0, dA, dB, dD1, dD2, ntiles);
    std::vector<float> D1(A.size()), D2(A.size());
    (void)hipMemcpy(D1.data(), dD1, D1.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(D2.data(), dD2, D2.size() * 4, hipMemcpyDeviceToHost);
    double w1 = 0, w2 = 0;
    long rn1 = 0, rn2 = 0, n = 0;
    for (int t = 0; t < ntiles; ++t)
        for (int r = 0; r < 32; ++r)
            for (int c = 0; c < 32; ++c) {
                double ex1 = 0, ab1 = 0, ex2 = 0, ab2 = 0;
                for (int k = 0; k < 32; ++k) {
                    const double p = (double)A[(size_t)t * 1024 + r * 32 + k] *
                                     (double)B[(size_t)t * 1024 + k * 32 + c];
                    if (k < 16) {
                        ex1 += p;
                        ab1 += std::fabs(p);
                    }
                    ex2 += p;
                    ab2 += std::fabs(p);
                }
                const size_t i = (size_t)t * 1024 + r * 32 + c;
                w1 = std::max(w1, std::fabs(D1[i] - ex1) / (std::ldexp(ab1, -24)));
                w2 = std::max(w2, std::fabs(D2[i] - ex2) / (std::ldexp(ab2, -24)));
                rn1 += D1[i] == (float)ex1;
                rn2 += D2[i] == (float)ex2;
                ++n;
            }
    printf("one MFMA (16 products): worst |D - exact| / (2^-24 sum|p|) = %.3f, D == RN(exact) for %.4f of %ld\n",
           w1, (double)rn1 / n, n);
    printf("two chained (32 products): worst ratio = %.3f, D == RN(exact) for %.4f\n", w2,
           (double)rn2 / n);
    printf("proof's allowance: 15 (one), 31 (two chained): %s\n",
           (w1 <= 15.0 && w2 <= 31.0) ? "holds" : "VIOLATED");
    return 0;
}
