// rt_dev_math.h -- f32 vector helpers, the correctly rounded short-form wrappers,
// hash3, camera rays (generate.wgsl), sky / reflect (shade.wgsl)
// (included by rt_kernels.hip only: one translation unit, device code)
#pragma once

namespace {

struct v3 {
    float x, y, z;
};

__device__ __forceinline__ v3 mk(float x, float y, float z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ v3 scale(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(v3 a, v3 b) {
    float r = a.x * b.x;
    r = r + a.y * b.y;
    r = r + a.z * b.z;
    return r;
}
__device__ __forceinline__ float length(v3 a) { return sqrtf(dot(a, a)); }
__device__ __forceinline__ v3 normalize(v3 a) {
    float l = length(a);
    return mk(a.x / l, a.y / l, a.z / l);
}

// ---- the hot path's correctly rounded ops (rt_math.h): the short forms on
// their checked domain; lanes outside it recompute with the plain IEEE op in
// a branch the wave skips when no lane needs it. The result is the IEEE one
// in every case (GPU parity tests; rt_debug_math + tests/test_gpu_math.py on
// zeros, denormals, huge, inf and NaN operands).
#if defined(RT_NO_FAST_MATH) || defined(RT_SHADE_IEEE)  // A/B: plain IEEE operations
__device__ __forceinline__ float sqrt_x(float x) { return sqrtf(x); }
__device__ __forceinline__ float length_x(v3 a) { return sqrtf(dot(a, a)); }
__device__ __forceinline__ float div_x(float n, float b, float) { return n / b; }
__device__ __forceinline__ float recip_or_nan(float b) { return b; }
__device__ __forceinline__ v3 div3_x(v3 v, float b) { return mk(v.x / b, v.y / b, v.z / b); }
__device__ __forceinline__ v3 normalize_x(v3 v) { return normalize(v); }
__device__ __forceinline__ v3 normalize_seed(v3 v) { return normalize(v); }
#else
// Each guard's ballot takes a single compare (no && / ||): the compare's lane
// mask is then the ballot, with no round trip through a VGPR.
__device__ __forceinline__ float sqrt_x(float x) {
    float r = rt_sqrt_rn(x);
    // x outside [2^-100, 2^100] (0, NaN, inf, < 0: IEEE) as one unsigned compare
    const bool bad = __float_as_uint(x) - 0x0D800000u > 0x71800000u - 0x0D800000u;
    if (rt_ballot(bad) != 0) {
        if (bad) r = sqrtf(rt_cold(x));
    }
    return r;
}
__device__ __forceinline__ float length_x(v3 a) { return sqrt_x(dot(a, a)); }

// n / b for a denominator b > 0 with yb = rt_recip_rn(b), or yb = NaN when b
// is outside rt_recip_rn's domain (every lane then takes the IEEE divide).
__device__ __forceinline__ float div_x(float n, float b, float yb) {
    float r = rt_div_rn(n, b, yb);
    const bool ok = yb == yb && rt_num_ok(n);
    if (rt_ballot(!ok) != 0) {
        if (!ok) r = n / b;
    }
    return r;
}
__device__ __forceinline__ float recip_or_nan(float b) {
    return b > 0.0f && rt_den_ok(b) ? rt_recip_rn(b) : __builtin_nanf("");
}

// v / b componentwise, any sign of b: short form when b and every component
// lie within [2^-40, 2^40] in magnitude (no zeros, so the sign rule of
// rt_div_rn does not arise). The range test runs on the magnitudes' bit
// patterns (integer min/max: same order as the floats, NaN above inf), so no
// canonicalising float min/max is needed.
__device__ __forceinline__ v3 div3_x(v3 v, float b) {
    const float y = rt_recip_rn(b);
    v3 r = mk(rt_div_rn(v.x, b, y), rt_div_rn(v.y, b, y), rt_div_rn(v.z, b, y));
    const uint32_t ax = __float_as_uint(v.x) & 0x7FFFFFFFu, ay = __float_as_uint(v.y) & 0x7FFFFFFFu;
    const uint32_t az = __float_as_uint(v.z) & 0x7FFFFFFFu, ab = __float_as_uint(b) & 0x7FFFFFFFu;
    const uint32_t lo = min(min(min(ax, ay), az), ab), hi = max(max(max(ax, ay), az), ab);
    const bool small = lo < 0x2B800000u /* 2^-40 */, big = hi > 0x53800000u /* 2^40 */;
    if ((rt_ballot(small) | rt_ballot(big)) != 0) {
        if (small || big) {
            const float bb = rt_cold(b);
            r = mk(v.x / bb, v.y / bb, v.z / bb);
        }
    }
    return r;
}

// normalize(v) = v / sqrt(dot(v, v)): short form when every squared component
// is at least 2^-80 and dot(v, v) <= 2^80 (false for NaN / inf): then every
// |v_i| >= 2^-40 (1 - 2^-24), dot(v, v) lies in rt_sqrt_rn's domain, the
// length l in [2^-40, 2^40] > 0 and every numerator in rt_div_rn's. The
// squares are dot's own products, so the guard costs a v_min3 and 2 compares.
__device__ __forceinline__ v3 normalize_x(v3 v) {
    const float px = v.x * v.x, py = v.y * v.y, pz = v.z * v.z;
    const float d2 = (px + py) + pz;  // = dot(v, v), same op order
    const float l = rt_sqrt_rn(d2);
    const float y = rt_recip_rn(l);
    v3 r = mk(rt_div_rn(v.x, l, y), rt_div_rn(v.y, l, y), rt_div_rn(v.z, l, y));
    const bool small = !(fminf(fminf(px, py), pz) >= 0x1p-80f), big = !(d2 <= 0x1p80f);
    if ((rt_ballot(small) | rt_ballot(big)) != 0) {
        if (small || big) r = normalize(mk(rt_cold(v.x), v.y, v.z));
    }
    return r;
}

// normalize(hash3(n)) needs no guard: hash3's components are k / 2^31 with k
// odd (shade.wgsl:105-116: n is odd after the first step), so each lies in
// [2^-31, 1], dot in [3*2^-62, 3] and the length in [2^-31, 2].
__device__ __forceinline__ v3 normalize_seed(v3 v) {
    const float l = rt_sqrt_rn(dot(v, v));
    const float y = rt_recip_rn(l);
    return mk(rt_div_rn(v.x, l, y), rt_div_rn(v.y, l, y), rt_div_rn(v.z, l, y));
}
#endif  // RT_NO_FAST_MATH

// shade.wgsl:105-116
__device__ __forceinline__ v3 hash3(uint32_t n) {
    n = (n << 13) ^ n;
    n = n * (n * n * 15731u + 789221u) + 1376312589u;
    uint32_t kx = n * n;
    uint32_t ky = n * (n * 16807u);
    uint32_t kz = n * (n * 48271u);
    const float den = 2147483648.0f;
    return mk((float)(kx & 0x7fffffffu) / den, (float)(ky & 0x7fffffffu) / den,
              (float)(kz & 0x7fffffffu) / den);
}

// generate.wgsl:66-129 (lens offset 0: origin = camera translation).
__device__ __forceinline__ void primary_ray(const KParams& P, uint32_t x, uint32_t y, v3& o,
                                            v3& d) {
    float px = (float)x, py = (float)y;
    v3 dir = mk(((px - P.half_w) * P.tan_half) / P.aspect,
                ((-py + P.half_h) * P.tan_half) / P.aspect, -1.0f);
    dir = normalize(dir);
    float denom = dot(dir, mk(0.0f, 0.0f, -1.0f));
    v3 fpnt = scale(dir, P.focus_plane / denom);
    v3 origin = mk(0.0f, 0.0f, 0.0f);
    dir = normalize(sub(fpnt, origin));
    const float* T = P.T;
    o = add(origin, mk(T[12], T[13], T[14]));
    d.x = ((T[0] * dir.x + T[4] * dir.y) + T[8] * dir.z) + T[12] * 0.0f;
    d.y = ((T[1] * dir.x + T[5] * dir.y) + T[9] * dir.z) + T[13] * 0.0f;
    d.z = ((T[2] * dir.x + T[6] * dir.y) + T[10] * dir.z) + T[14] * 0.0f;
}

// rt_sincos of the opt-in thin-lens sampling (include/rt_hip.h): Cody-Waite
// reduction by pi/2, Taylor polynomials, quadrant swap; plain f32 ops in the
// oracle's order (oracle/rt_oracle.c rto_sincos).
__device__ __forceinline__ void rt_sincos(float theta, float& s, float& c) {
    const float q = rintf(theta * 0x1.45f306p-1f);
    float r = theta - q * 0x1.92p+0f;
    r = r - q * 0x1.fb5444p-12f;
    r = r - q * 0x1.68cp-39f;
    const float r2 = r * r;
    const float sr = r + r * (r2 * (-0x1.555556p-3f +
                                    r2 * (0x1.111112p-7f +
                                          r2 * (-0x1.a01a02p-13f + r2 * 0x1.71de3ap-19f))));
    const float cr = 1.0f + r2 * (-0x1p-1f +
                                  r2 * (0x1.555556p-5f +
                                        r2 * (-0x1.6c16c2p-10f +
                                              r2 * (0x1.a01a02p-16f + r2 * -0x1.27e4fcp-22f))));
    switch ((int)q & 3) {
        case 0: s = sr; c = cr; break;
        case 1: s = cr; c = -sr; break;
        case 2: s = -sr; c = -cr; break;
        default: s = -cr; c = sr; break;
    }
}

// Opt-in camera sampling (RT_FLAG_JITTER / RT_FLAG_THIN_LENS, rt_hip.h):
// generate.wgsl:66-129 with a jittered pixel position and/or a lens sample
// fed to thin_lens_ray (generate.wgsl:85-107) verbatim. idx = the seed index.
__device__ __forceinline__ void sampled_primary_ray(const KParams& P, uint32_t x, uint32_t y,
                                                 uint32_t idx, v3& o, v3& d) {
    float px = (float)x, py = (float)y;
    if (P.flags & RT_FLAG_JITTER) {
        const v3 j = hash3(idx * RT_JITTER_HASH_MUL);
        px = px + (j.x - 0.5f);
        py = py + (j.y - 0.5f);
    }
    v3 dir = mk(((px - P.half_w) * P.tan_half) / P.aspect,
                ((-py + P.half_h) * P.tan_half) / P.aspect, -1.0f);
    dir = normalize(dir);
    const float denom = dot(dir, mk(0.0f, 0.0f, -1.0f));
    const v3 fpnt = scale(dir, P.focus_plane / denom);
    v3 origin = mk(0.0f, 0.0f, 0.0f);
    if (P.flags & RT_FLAG_THIN_LENS) {
        const v3 l = hash3(idx * RT_LENS_HASH_MUL);
        const float pi2 = 2.0f * 3.14159265358979f;
        const float theta = pi2 * l.x + pi2;
        const float sr = sqrtf(l.y);
        float sn, cs;
        rt_sincos(theta, sn, cs);
        const float a = (cs * sr) * P.coc, b = (sn * sr) * P.coc;
        origin = add(mk(1.0f * a, 0.0f * a, 0.0f * a), mk(0.0f * b, 1.0f * b, 0.0f * b));
    }
    dir = normalize(sub(fpnt, origin));
    const float* T = P.T;
    o = add(origin, mk(T[12], T[13], T[14]));
    d.x = ((T[0] * dir.x + T[4] * dir.y) + T[8] * dir.z) + T[12] * 0.0f;
    d.y = ((T[1] * dir.x + T[5] * dir.y) + T[9] * dir.z) + T[13] * 0.0f;
    d.z = ((T[2] * dir.x + T[6] * dir.y) + T[10] * dir.z) + T[14] * 0.0f;
}

// shade.wgsl:189-197
__device__ __forceinline__ v3 sky(v3 d) {
    v3 unit = normalize(d);
    float t = 0.5f * unit.y + 1.0f;
    float omt = (1.0f - t) * 1.0f;
    return mk(omt + t * 0.5f, omt + t * 0.7f, omt + t * 1.0f);
}

__device__ __forceinline__ v3 reflect(v3 v, v3 n) {  // shade.wgsl:132-134
    float k = 2.0f * dot(v, n);
    return sub(v, scale(n, k));
}


}  // namespace
