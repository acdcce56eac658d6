// rt_math.h — correctly rounded f32 division and square root for the hot
// path, in fewer VALU than the general IEEE expansions hipcc emits (11 VALU
// per divide: div_scale x2, rcp, 5 fma/mul, div_fmas, div_fixup; 16 per sqrt
// with the denormal scaling and class fix-ups), valid on a restricted domain:
//   rt_recip_rn(b)        == RN(1/b)   for |b| in [2^-60, 2^60]   (3 VALU)
//   rt_div_rn(a, b, y)    == RN(a/b)   given y = rt_recip_rn(b), |a| in
//                                      [2^-60, 2^60], or a == +-0 with b > 0
//                                      (over b < 0 a +0 numerator gives +0,
//                                      not -0)                    (3 VALU)
//   (so the quotient and the residual stay normal: outside that, e.g.
//    |a| = 2^100 over |b| = 2^-60, the form over/underflows where IEEE does not)
//   rt_sqrt_rn(x)         == RN(sqrt x) for x == 0 or x in [2^-100, 2^100] (8 VALU)
// Checked on the GPU (tools/ubench/div_exact.hip): recip on every significand
// (both signs, 5 exponents), division on 2^33 random pairs over the domain
// incl. signed zeros, sqrt on every significand at both exponent parities.
// Callers keep IEEE results everywhere: operands outside the domain take the
// plain IEEE operation (rt_dev_math.h guards).
#pragma once

#include <hip/hip_runtime.h>

// One Newton step on the 1-ulp hardware reciprocal.
__device__ __forceinline__ float rt_recip_rn(float b) {
    const float r0 = __builtin_amdgcn_rcpf(b);
    return __builtin_fmaf(__builtin_fmaf(-b, r0, 1.0f), r0, r0);
}

// Markstein's correction with the residual taken as b*q - a (exact), so that a
// signed zero numerator over a positive denominator keeps its sign:
// q = a*y; q' = q - (b*q - a)*y.
__device__ __forceinline__ float rt_div_rn(float a, float b, float y) {
    const float q = a * y;
    const float r = __builtin_fmaf(b, q, -a);
    return __builtin_fmaf(-r, y, q);
}

// Hardware square root, then the +-1 ulp candidate whose residual brackets x.
__device__ __forceinline__ float rt_sqrt_rn(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x);
    const float rp = __builtin_fmaf(-sp, s, x);
    float r = rm <= 0.0f ? sm : s;
    r = rp > 0.0f ? sp : r;
    return r;
}

// Domain predicates (one compare each on |v|; NaN fails every one).
__device__ __forceinline__ bool rt_den_ok(float b) {
    return __builtin_fabsf(b) >= 0x1p-60f && __builtin_fabsf(b) <= 0x1p60f;
}
// (for a numerator over a POSITIVE denominator)
__device__ __forceinline__ bool rt_num_ok(float a) {
    return a == 0.0f || (__builtin_fabsf(a) >= 0x1p-60f && __builtin_fabsf(a) <= 0x1p60f);
}
__device__ __forceinline__ bool rt_sqrt_ok(float x) {
    return x == 0.0f || (x >= 0x1p-100f && x <= 0x1p100f);
}
