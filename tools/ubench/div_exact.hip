// Exactness checks of the correctly rounded f32 forms used by rt_kernels.hip
// (rt_math: recip_rn / div_rn / sqrt_rn) against the IEEE division and
// square root hipcc emits for a / b and sqrtf(x):
//   recip_rn(b) = fma(fma(-b, r0, 1), r0, r0), r0 = v_rcp_f32(b)  == RN(1/b)
//   div_rn(a, b, y=recip_rn(b)) = fma(-fma(b, q, -a), y, q), q = a*y  (Markstein)
//   sqrt_rn(x)  = v_sqrt_f32 then the +-1 ulp residual correction
// Domain (the kernel guards everything else onto the IEEE path):
//   |b| in [2^-60, 2^60]; |a| in [2^-60, 2^60] (so a/b and the residual stay
//   normal), or a == +-0 when b > 0; x == 0 or x in [2^-100, 2^100].
// Part 1: recip_rn on every significand at 5 exponents.
// Part 2: 2^33 random (a, b) pairs over the domain, zeros of both signs included.
// Part 3: sqrt_rn on every significand at both exponent parities, at 6 exponents, and 0.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#include "../../bevy_raytrace_amd/csrc/rt_math.h"

__global__ void recip_all(int e, unsigned long long* bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const float b = __uint_as_float(((uint32_t)(127 + e) << 23) | m);
    for (int s = 0; s < 2; ++s) {
        const float bb = s ? -b : b;
        if (__float_as_uint(rt_recip_rn(bb)) != __float_as_uint(1.0f / bb)) atomicAdd(bad, 1ull);
    }
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void div_random(uint32_t seed, unsigned long long* bad, unsigned long long* tested) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned long long nb = 0;
    for (int k = 0; k < 64; ++k) {
        const uint32_t h1 = hash32(i * 64u + k + seed * 0x9E3779B9u);
        const uint32_t h2 = hash32(h1 ^ 0xA511E9B3u);
        const uint32_t h3 = hash32(h2 + 0x3C6EF372u);
        const uint32_t ea = 127 + (h1 >> 25) % 121 - 60;    // |a| exponent in [-60, 60]
        const uint32_t eb = 127 + (h2 >> 25) % 121 - 60;    // |b| exponent in [-60, 60]
        float a = __uint_as_float(((h3 & 1) << 31) | (ea << 23) | (h1 & 0x7FFFFF));
        const float b = __uint_as_float(((h3 >> 1 & 1) << 31) | (eb << 23) | (h2 & 0x7FFFFF));
        // zeros of both signs over a positive denominator (the contract: a +0
        // numerator over b < 0 would come out +0, not -0; callers with b < 0
        // never pass a zero numerator)
        if ((h3 & 0x3F0) == 0 && b > 0.0f) a = (h3 & 1) ? -0.0f : 0.0f;
        const float y = rt_recip_rn(b);
        if (__float_as_uint(rt_div_rn(a, b, y)) != __float_as_uint(a / b)) ++nb;
    }
    if (nb) atomicAdd(bad, nb);
    if (threadIdx.x == 0) atomicAdd(tested, 64ull * blockDim.x);
}

__global__ void sqrt_all(int e, unsigned long long* bad) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const float x = __uint_as_float(((uint32_t)(127 + e) << 23) | m);
    if (__float_as_uint(rt_sqrt_rn(x)) != __float_as_uint(sqrtf(x))) atomicAdd(bad, 1ull);
    if (m == 0 && __float_as_uint(rt_sqrt_rn(0.0f)) != __float_as_uint(sqrtf(0.0f))) atomicAdd(bad, 1ull);
}

int main() {
    unsigned long long *bad, *tested, nb, nt;
    hipMalloc(&bad, 8); hipMalloc(&tested, 8);
    int rc = 0;
    for (int e : {0, -60, 60, -1, 1}) {
        hipMemset(bad, 0, 8);
        hipLaunchKernelGGL(recip_all, dim3((1 << 23) / 256), dim3(256), 0, 0, e, bad);
        hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        printf("recip_rn exponent %d: %llu of %u (both signs) differ from IEEE 1/b\n", e, nb, 2u << 23);
        rc |= nb != 0;
    }
    hipMemset(bad, 0, 8); hipMemset(tested, 0, 8);
    for (uint32_t s = 0; s < 32; ++s)
        hipLaunchKernelGGL(div_random, dim3(16384), dim3(256), 0, 0, s, bad, tested);
    hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost); hipMemcpy(&nt, tested, 8, hipMemcpyDeviceToHost);
    printf("div_rn: %llu of %llu random (a, b) pairs differ from IEEE a/b\n", nb, nt);
    rc |= nb != 0;
    for (int e : {0, 1, -100, -99, 99, 100}) {
        hipMemset(bad, 0, 8);
        hipLaunchKernelGGL(sqrt_all, dim3((1 << 23) / 256), dim3(256), 0, 0, e, bad);
        hipMemcpy(&nb, bad, 8, hipMemcpyDeviceToHost);
        printf("sqrt_rn exponent %d: %llu of %u differ from IEEE sqrtf\n", e, nb, 1u << 23);
        rc |= nb != 0;
    }
    printf(rc ? "FAIL\n" : "PASS\n");
    return rc;
}
