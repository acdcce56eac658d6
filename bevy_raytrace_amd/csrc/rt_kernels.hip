// rt_kernels.hip — the MI355X (gfx950) path-tracer kernels.
//
// ONE persistent kernel replaces the reference's whole WGSL chain
//   clear.wgsl:71-87 -> generate.wgsl:109-130 -> 3 x (prepass.wgsl:55-63,
//   intersect.wgsl:145-163, shade.wgsl:199-258) -> collect.wgsl:99-125
// dispatched by RayTraceNode::run (src/ray_trace_node.rs:195-224). Nothing is
// exchanged through HBM between stages: each lane keeps its whole path state
// (ray, throughput, seed, sample-block sum) in VGPRs.
//
// Work decomposition: a launch covers F frames; its work
// queue holds (frame, pixel, sample block of RT_SAMPLE_BLOCK samples) *block
// items* followed by single-sample *tail items* (so no lane holds a long item
// when the queue runs dry). Waves take chunks of items with one atomic
// (prefetched a chunk ahead); a lane whose path ends starts the next sample of
// its item, a lane whose item ends stores its block sum (or, for a tail item,
// each sample's colour) and takes the next item (wave-ballot refill), so lanes
// do not idle while the wave's longest path finishes. rt_collect_kernel folds
// a pixel's slots in sample order -- the oracle's summation order.
//
// Intersection (the hot loop, intersect.wgsl:133-143): every sphere of the
// list is tested for every live ray (brute force). The list is read as groups
// of 8 spheres (SoA cx[8] cy[8] cz[8] S[8]) with scalar loads and fed to
// hand-scheduled v_pk_fma_f32 as SGPR pairs (filter8: 28 packed FMAs + a
// v_max3 chain + 1 compare per group):
//   H - T = hb^2 + r^2 - (1 - m)|o - c|^2 + mu (|o|^2 + |c|^2),  hb = dn.(o - c)
// H < T proves the reference's discriminant (intersect.wgsl:102) is negative.
// Lanes queue their candidate groups (group, 8-bit mask) in LDS; after the
// walk each lane runs the reference's exact op sequence (intersect.wgsl:
// 97-115) on its own candidates in list order with the strict `<` tie-break
// (:137), so the result is bit-identical to the brute-force reference loop.
//
// Floating point: compiled with -ffp-contract=off; every expression below
// except the explicit FMAs of the filter is one IEEE f32 round-to-nearest op
// in the same order as oracle/rt_oracle.c. Divides and square roots are
// correctly rounded: the short forms of rt_math.h where their domain is
// proved (exact test) or checked per lane (shading), IEEE otherwise.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_internal.h"
#include "rt_math.h"

// Wave ballot on a bool straight into the intrinsic: HIP's __ballot(int)
// round-trips the lane mask through a VGPR (v_cndmask + v_cmp, 2 VALU) when
// the predicate comes from another block.
__device__ __forceinline__ uint64_t rt_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Keeps a rare fallback in its branch: LLVM prices sqrt / fdiv as one IR
// instruction and speculates them out of the branch (then the backend's
// 11-17 instruction IEEE expansion runs on every pass, measured). A volatile
// asm cannot be speculated.
__device__ __forceinline__ float rt_cold(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

#define VERY_FAR 1e20f
#define EPSILON 0.001f

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
#ifdef RT_FAST_NOGUARD  // measurement only (NOT exact): no IEEE fallback lanes
#define RT_GUARD_ON 0
#else
#define RT_GUARD_ON 1
#endif
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
    if (RT_GUARD_ON && rt_ballot(bad) != 0) {
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
    if (RT_GUARD_ON && rt_ballot(!ok) != 0) {
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
    if (RT_GUARD_ON && (rt_ballot(small) | rt_ballot(big)) != 0) {
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
    if (RT_GUARD_ON && (rt_ballot(small) | rt_ballot(big)) != 0) {
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

// ---- diagnostic build only (-DRT_PROFILE): per-wave phase clocks (s_memtime)
// and wave-level event counts, summed into a debug buffer. Never compiled into
// the product library.
#ifdef RT_PROFILE
struct Prof {
    unsigned long long c[16];
    unsigned long long last;
};
#define PROF_DECL Prof prof_ = {};
#define PROF_START() (prof_.last = __builtin_amdgcn_s_memtime())
#define PROF_MARK(i)                                            \
    do {                                                        \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        prof_.c[i] += t_ - prof_.last;                          \
        prof_.last = t_;                                        \
    } while (0)
#define PROF_ADD(i, v) (prof_.c[i] += (v))
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off));
    return v;
}
#else
#define PROF_DECL
#define PROF_START()
#define PROF_MARK(i)
#define PROF_ADD(i, v)
#endif

// Exact reference test of one sphere (intersect.wgsl:97-115 + :137).
// s.w = RN(radius*radius) = sqr(s.radius); r2p = s.w * (1 + 2^-20).
#ifdef RT_PROFILE
__device__ uint32_t g_prof_dummy;
#define EXACT_COUNT(k) (ecnt[k]++)
#define EXACT_ARGS , uint32_t* ecnt
#define EXACT_PASS , ecnt
#else
#define EXACT_COUNT(k)
#define EXACT_ARGS
#define EXACT_PASS
#endif
// FAST (wave-uniform, ray_fast below): the short correctly-rounded forms of
// rt_math.h, unguarded. Their domains hold without per-candidate checks:
// the scene (rt_api.cpp scene_fast_ok) has |centre_i| <= 2^30 and
// r^2 in [2^-40, 2^60], the ray |origin_i| <= 2^32 and a in [2^-20, 2^20], so
// qq < 2^67, |half_b| < 2^44, dis < 2^88 and the numerators < 2^45. Low ends:
//  - qq < 2^-100 (incl. 0): lo^2 < 2^-99 is below half an ulp of s.w >= 2^-40,
//    so c = -s.w whichever lo (IEEE or short) the square root returned;
//  - dis < 2^-100: the IEEE sqrtf (a rare branch; dis < 0 returns as before);
//  - |numerator| < 2^-60 (incl. +-0): IEEE and short quotients both have
//    |root| < 2^-40 < EPSILON and are rejected alike.
// Otherwise the IEEE operations (sqrtf, '/'). ya = rt_recip_rn(a) when FAST.
template <bool FAST>
__device__ __forceinline__ void exact_body(float4 s, int idx, v3 o, v3 d, float a, float ya,
                                           float& best_t, int& best_i EXACT_ARGS) {
    EXACT_COUNT(0);
    const v3 oc = mk(o.x - s.x, o.y - s.y, o.z - s.z);
    const float half_b = dot(oc, d);
    const float qq = dot(oc, oc);
    // Cheap certain-miss: centre behind the origin (half_b >= 0) and origin
    // outside (qq >= r^2 (1 + 2^-20) => c >= 0 after the sqrt/square round
    // trip). Then dis <= half_b^2, sqrt(dis) <= half_b, and both roots are
    // <= 0 < EPSILON, exactly as the full evaluation below would find.
    if (half_b >= 0.0f && qq >= s.w * (1.0f + 0x1p-20f)) return;
    EXACT_COUNT(1);
    const float lo = FAST ? rt_sqrt_rn(qq) : sqrtf(qq);
    const float c = lo * lo - s.w;
    const float dis = half_b * half_b - a * c;
    float sqrtd;
    if (FAST) {
        if (dis < 0x1p-100f) {
            if (dis < 0.0f) return;
            sqrtd = sqrtf(rt_cold(dis));
        } else {
            sqrtd = rt_sqrt_rn(dis);
        }
    } else {
        if (dis < 0.0f) return;
        sqrtd = sqrtf(dis);
    }
    float root = FAST ? rt_div_rn(-half_b - sqrtd, a, ya) : (-half_b - sqrtd) / a;
    if (root < EPSILON || VERY_FAR < root) {
        root = FAST ? rt_div_rn(-half_b + sqrtd, a, ya) : (-half_b + sqrtd) / a;
        if (root < EPSILON || VERY_FAR < root) return;
    }
    if (root < best_t) {
        best_t = root;
        best_i = idx;
    }
}

__device__ __forceinline__ void exact_test(float4 s, int idx, v3 o, v3 d, float a, float ya,
                                           bool fast, float& best_t, int& best_i EXACT_ARGS) {
    if (fast)
        exact_body<true>(s, idx, o, d, a, ya, best_t, best_i EXACT_PASS);
    else
        exact_body<false>(s, idx, o, d, a, ya, best_t, best_i EXACT_PASS);
}

// The ray side of the short-math domain (exact_body), for the whole wave.
__device__ __forceinline__ bool ray_fast(uint32_t scene_fast, v3 o, float a) {
#ifdef RT_NO_FAST_MATH
    return false;
#else
    // (a NaN origin component makes every exact test of the lane NaN in both
    // forms: no hit either way)
    const float om = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    return scene_fast != 0 && (rt_ballot(!(om <= 0x1p32f)) | rt_ballot(!(a >= 0x1p-20f)) |
                               rt_ballot(!(a <= 0x1p20f))) == 0;
#endif
}

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(4))) const float4 cfloat4;  // scalar-cache reads

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bc(float x) { return f2{x, x}; }

// Per-ray constants of the expanded-form filter (see file header / DESIGN.md):
//   G' = (k1 - dn.c)^2 + S + K + o2.c
//      = hb^2 + r^2 - (1 - m) |o - c|^2 + mu (|o|^2 + |c|^2)
// with hb = dn.(o - c), dn ~ d/|d|, S = r^2 - (1 - m - mu)|c|^2 (per sphere,
// host), k1 = dn.o, K = -(1 - m - mu)|o|^2, o2 = 2(1 - m) o (per ray).
// m = 2^-16 bounds the exact path's rounding relative to |o - c|^2 + r^2,
// mu = 2^-17 the expanded form's cancellation relative to |o|^2 + |c|^2.
struct RayF {
    f2 dx, dy, dz, o2x, o2y, o2z, k1;  // dx,dy,dz hold -dn
    float T;                           // candidate threshold -K
};

__device__ __forceinline__ RayF ray_filter_consts(v3 o, v3 d) {
    const float rs = __builtin_amdgcn_rsqf(dot(d, d));  // approximate 1/|d| (covered by m)
    const float dnx = d.x * rs, dny = d.y * rs, dnz = d.z * rs;
    const float m = 0x1p-16f, mu = 0x1p-17f;
    const float oo = __builtin_fmaf(o.z, o.z, __builtin_fmaf(o.y, o.y, o.x * o.x));
    const float k1 = __builtin_fmaf(dnz, o.z, __builtin_fmaf(dny, o.y, dnx * o.x));
    const float two = 2.0f * (1.0f - m);
    RayF r;
    r.dx = bc(-dnx); r.dy = bc(-dny); r.dz = bc(-dnz);  // negated: hb = k1 + (-dn).c
    r.o2x = bc(two * o.x); r.o2y = bc(two * o.y); r.o2z = bc(two * o.z);
    r.k1 = bc(k1);
    r.T = (1.0f - m - mu) * oo;
    return r;
}

// Filter two spheres at once: 7 packed fp32 FMAs (v_pk_fma_f32: two f32 FMAs
// per lane per issue, tools/ubench/fma_rate.hip). Returns H = hb^2 + S + o2.c;
// the sphere is a candidate iff H >= T, the ray's threshold (an exact
// comparison). The C++ form of filter8 (builds without RT_ASM_FILTER).
__device__ __forceinline__ f2 filter2(f2 cx, f2 cy, f2 cz, f2 S, const RayF& r) {
    // every op has ONE SGPR-pair operand (sphere data) -- the constant-bus limit
    const f2 hb = pk_fma(r.dz, cz, pk_fma(r.dy, cy, pk_fma(r.dx, cx, r.k1)));  // k1 - dn.c
    return pk_fma(r.o2x, cx, pk_fma(r.o2y, cy, pk_fma(r.o2z, cz, pk_fma(hb, hb, S))));
}

// The same filter for a whole group of 8 spheres in hand-scheduled VOP3P:
// the ray constants live ONCE in 4 VGPR pairs (r0 = (-dnx, -dny),
// r1 = (-dnz, k1), r2 = (o2x, o2y), r3 = (o2z, T)) and op_sel / op_sel_hi
// broadcast one half to both packed lanes -- the compiler's form needs every
// constant duplicated in a pair (7 VGPRs more at the 80-VGPR occupancy limit).
// The four pair chains are interleaved, so dependent ops are 4 apart (no
// wait states, and a lone wave in the queue tail issues back to back). Op
// order per pair is exactly filter2's.
struct RayP {
    f2 r0, r1, r2, r3;
};

__device__ __forceinline__ RayP ray_pack(const RayF& r) {
    RayP p;
    p.r0 = f2{r.dx.x, r.dy.x};
    p.r1 = f2{r.dz.x, r.k1.x};
    p.r2 = f2{r.o2x.x, r.o2y.x};
    p.r3 = f2{r.o2z.x, r.T};
    return p;
}

__device__ __forceinline__ void filter8(const RayP& R, f2 cxa, f2 cxb, f2 cxc, f2 cxd, f2 cya,
                                        f2 cyb, f2 cyc, f2 cyd, f2 cza, f2 czb, f2 czc, f2 czd,
                                        f2 sa, f2 sb, f2 sc, f2 sd, f2& ha, f2& hb, f2& hc,
                                        f2& hd, float& hmax) {
    asm volatile(
        // hb = k1 + (-dnx) cx + (-dny) cy + (-dnz) cz
        "v_pk_fma_f32 %[ha], %[r0], %[cxa], %[r1] op_sel:[0,0,1] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hb], %[r0], %[cxb], %[r1] op_sel:[0,0,1] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hc], %[r0], %[cxc], %[r1] op_sel:[0,0,1] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hd], %[r0], %[cxd], %[r1] op_sel:[0,0,1] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[ha], %[r0], %[cya], %[ha] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[hb], %[r0], %[cyb], %[hb] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[hc], %[r0], %[cyc], %[hc] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[hd], %[r0], %[cyd], %[hd] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[ha], %[r1], %[cza], %[ha] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hb], %[r1], %[czb], %[hb] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hc], %[r1], %[czc], %[hc] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hd], %[r1], %[czd], %[hd] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        // H = hb^2 + S + o2z cz + o2y cy + o2x cx
        "v_pk_fma_f32 %[ha], %[ha], %[ha], %[sa]\n\t"
        "v_pk_fma_f32 %[hb], %[hb], %[hb], %[sb]\n\t"
        "v_pk_fma_f32 %[hc], %[hc], %[hc], %[sc]\n\t"
        "v_pk_fma_f32 %[hd], %[hd], %[hd], %[sd]\n\t"
        "v_pk_fma_f32 %[ha], %[r3], %[cza], %[ha] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hb], %[r3], %[czb], %[hb] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hc], %[r3], %[czc], %[hc] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hd], %[r3], %[czd], %[hd] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[ha], %[r2], %[cya], %[ha] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[hb], %[r2], %[cyb], %[hb] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[hc], %[r2], %[cyc], %[hc] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[hd], %[r2], %[cyd], %[hd] op_sel:[1,0,0] op_sel_hi:[1,1,1]\n\t"
        "v_pk_fma_f32 %[ha], %[r2], %[cxa], %[ha] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hb], %[r2], %[cxb], %[hb] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hc], %[r2], %[cxc], %[hc] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %[hd], %[r2], %[cxd], %[hd] op_sel:[0,0,0] op_sel_hi:[0,1,1]\n\t"
        // group max of the 8 H (v_max3 drops a quiet-NaN operand, as fmaxf)
        "v_max3_f32 %[hm], v40, v41, v42\n\t"
        "v_max3_f32 %[hm], %[hm], v43, v44\n\t"
        "v_max3_f32 %[hm], %[hm], v45, v46\n\t"
        "v_max_f32 %[hm], %[hm], v47"
        : [ha] "={v[40:41]}"(ha), [hb] "={v[42:43]}"(hb), [hc] "={v[44:45]}"(hc),
          [hd] "={v[46:47]}"(hd), [hm] "=&v"(hmax)
        : [r0] "v"(R.r0), [r1] "v"(R.r1), [r2] "v"(R.r2), [r3] "v"(R.r3), [cxa] "s"(cxa),
          [cxb] "s"(cxb), [cxc] "s"(cxc), [cxd] "s"(cxd), [cya] "s"(cya), [cyb] "s"(cyb),
          [cyc] "s"(cyc), [cyd] "s"(cyd), [cza] "s"(cza), [czb] "s"(czb), [czc] "s"(czc),
          [czd] "s"(czd), [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc), [sd] "s"(sd));
}

__device__ __forceinline__ uint32_t ge(float h, float t) { return h >= t ? 1u : 0u; }

#if defined(RT_ASM_FILTER) && defined(__HIP_DEVICE_COMPILE__)
// The lane's 8-bit candidate mask (bit j = H_j >= T, the same compares as
// ge()): the 8 compares go to 8 SGPR lane masks, then m = 2m + c_j shifts
// them in with v_addc (carry-in = the lane's bit of c_j), sphere 7 first --
// 16 VALU instead of 8 compares + 8 v_cndmask + 4 ORs, and every mask is
// read 7+ instructions after its compare wrote it (no VALU-SGPR wait states).
__device__ __forceinline__ uint32_t cand_mask8(f2 g01, f2 g23, f2 g45, f2 g67, float T) {
    uint32_t m;
    uint64_t c0, c1, c2, c3, c4, c5, c6, c7;
    asm("v_cmp_ge_f32_e64 %[c7], %[h7], %[T]\n"
        "v_cmp_ge_f32_e64 %[c6], %[h6], %[T]\n"
        "v_cmp_ge_f32_e64 %[c5], %[h5], %[T]\n"
        "v_cmp_ge_f32_e64 %[c4], %[h4], %[T]\n"
        "v_cmp_ge_f32_e64 %[c3], %[h3], %[T]\n"
        "v_cmp_ge_f32_e64 %[c2], %[h2], %[T]\n"
        "v_cmp_ge_f32_e64 %[c1], %[h1], %[T]\n"
        "v_cmp_ge_f32_e64 %[c0], %[h0], %[T]\n"
        "v_cndmask_b32_e64 %[m], 0, 1, %[c7]\n"
        "v_addc_co_u32_e64 %[m], %[c7], %[m], %[m], %[c6]\n"
        "v_addc_co_u32_e64 %[m], %[c6], %[m], %[m], %[c5]\n"
        "v_addc_co_u32_e64 %[m], %[c5], %[m], %[m], %[c4]\n"
        "v_addc_co_u32_e64 %[m], %[c4], %[m], %[m], %[c3]\n"
        "v_addc_co_u32_e64 %[m], %[c3], %[m], %[m], %[c2]\n"
        "v_addc_co_u32_e64 %[m], %[c2], %[m], %[m], %[c1]\n"
        "v_addc_co_u32_e64 %[m], %[c1], %[m], %[m], %[c0]\n"
        : [m] "=&v"(m), [c0] "=&s"(c0), [c1] "=&s"(c1), [c2] "=&s"(c2), [c3] "=&s"(c3),
          [c4] "=&s"(c4), [c5] "=&s"(c5), [c6] "=&s"(c6), [c7] "=&s"(c7)
        : [h0] "v"(g01.x), [h1] "v"(g01.y), [h2] "v"(g23.x), [h3] "v"(g23.y),
          [h4] "v"(g45.x), [h5] "v"(g45.y), [h6] "v"(g67.x), [h7] "v"(g67.y), [T] "v"(T));
    return m;
}
#endif

template <bool FAST>
__device__ __forceinline__ void drain_list(const uint32_t* cq, uint32_t cnt,
                                           const float4* __restrict__ sph, v3 o, v3 d, float a,
                                           float ya, float& best_t, int& best_i EXACT_ARGS) {
    const uint32_t lane = __lane_id();
    for (uint32_t k = 0; k < cnt; ++k) {
        const uint32_t e = cq[k * 64 + lane];
        uint32_t m = e & 0xFFu;
        const uint32_t base = (e >> 8) * RT_GROUP;
        while (m) {
            const uint32_t j = __builtin_ctz(m);
            m &= m - 1;
            exact_body<FAST>(sph[base + j], (int)(base + j), o, d, a, ya, best_t, best_i EXACT_PASS);
        }
    }
}

// Run the exact test for every queued candidate of this lane, in list order.
// Queue entries are (group << 8 | 8-bit candidate mask), one column per lane.
__device__ __forceinline__ void drain_candidates(const uint32_t* cq, uint32_t cnt,
                                                 const float4* __restrict__ sph, v3 o, v3 d,
                                                 float a, bool fast, float& best_t,
                                                 int& best_i EXACT_ARGS) {
    if (fast)
        drain_list<true>(cq, cnt, sph, o, d, a, rt_recip_rn(a), best_t, best_i EXACT_PASS);
    else
        drain_list<false>(cq, cnt, sph, o, d, a, a, best_t, best_i EXACT_PASS);
}

// Closest hit over the whole list (intersect.wgsl:133-143).
// grp: the sphere list as groups of RT_GROUP=8, SoA (cx[8], cy[8], cz[8], S[8]),
// padded to whole groups with pad records of S = -inf (never candidates).
// Wave-uniform: read with s_load_dwordx16 and fed to the packed ops as SGPR
// pairs. sph: the padded records AoS (cx, cy, cz, r2), gathered per lane by
// the exact tests. Pass 1 filters every sphere and queues candidates per lane
// (LDS, cq); the group test is max(H) >= T over the 8 spheres. Pass 2 (drain)
// runs the exact reference test on the queued candidates in list order, so the
// wave pays for max-over-lanes candidates, not for their union.
// Returns the best index (-1 = miss) and t.
__device__ __forceinline__ int intersect_world(const float4* __restrict__ grp,
                                               const float4* __restrict__ sph, uint32_t ngroups,
                                               uint32_t scene_fast, v3 o, v3 d, float& t_out,
                                               uint32_t* cq
#ifdef RT_PROFILE
                                               , Prof& prof_
#endif
                                               ) {
    const float l = sqrt_x(dot(d, d));
    const float a = l * l;  // sqr(length(r.dir)), intersect.wgsl:98
    const bool fast = ray_fast(scene_fast, o, a);
#if defined(RT_ASM_FILTER) && defined(__HIP_DEVICE_COMPILE__)
    const RayP RP = ray_pack(ray_filter_consts(o, d));
    const float RT_T = RP.r3.y;
#else
    const RayF R = ray_filter_consts(o, d);
    const float RT_T = R.T;
#endif
    const uint32_t lane = __lane_id();
    float best_t = VERY_FAR;
    int best_i = -1;
    uint32_t cnt = 0;
#ifdef RT_PROFILE
    uint32_t ecnt[2] = {0, 0};
#endif
    // constant address space: the groups are read with s_load into SGPRs
    // whatever the alias analysis concludes about other stores
#if defined(__HIP_DEVICE_COMPILE__)
    const cfloat4* gp = (const cfloat4*)(uintptr_t)grp;
#else
    const float4* gp = grp;  // host pass: never executed
#endif
    for (uint32_t g = 0; g < ngroups; ++g) {
        const auto* p = gp + (size_t)g * 8;
        const float4 X0 = p[0], X1 = p[1], Y0 = p[2], Y1 = p[3];
        const float4 Z0 = p[4], Z1 = p[5], S0 = p[6], S1 = p[7];
#if defined(RT_ASM_FILTER) && defined(__HIP_DEVICE_COMPILE__)
        f2 g01, g23, g45, g67;
        float hmax;
        filter8(RP, f2{X0.x, X0.y}, f2{X0.z, X0.w}, f2{X1.x, X1.y}, f2{X1.z, X1.w},
                f2{Y0.x, Y0.y}, f2{Y0.z, Y0.w}, f2{Y1.x, Y1.y}, f2{Y1.z, Y1.w},
                f2{Z0.x, Z0.y}, f2{Z0.z, Z0.w}, f2{Z1.x, Z1.y}, f2{Z1.z, Z1.w},
                f2{S0.x, S0.y}, f2{S0.z, S0.w}, f2{S1.x, S1.y}, f2{S1.z, S1.w}, g01, g23, g45, g67,
                hmax);
#else
        // group test below: max of the 8 H (v_max3 chain; a NaN H is dropped
        // by max -- a NaN H never hits) against the ray's threshold
        const f2 g01 = filter2(f2{X0.x, X0.y}, f2{Y0.x, Y0.y}, f2{Z0.x, Z0.y}, f2{S0.x, S0.y}, R);
        const f2 g23 = filter2(f2{X0.z, X0.w}, f2{Y0.z, Y0.w}, f2{Z0.z, Z0.w}, f2{S0.z, S0.w}, R);
        const f2 g45 = filter2(f2{X1.x, X1.y}, f2{Y1.x, Y1.y}, f2{Z1.x, Z1.y}, f2{S1.x, S1.y}, R);
        const f2 g67 = filter2(f2{X1.z, X1.w}, f2{Y1.z, Y1.w}, f2{Z1.z, Z1.w}, f2{S1.z, S1.w}, R);
        const float hmax = fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(g01.x, g01.y), g23.x), g23.y),
                                                   g45.x), g45.y), g67.x), g67.y);
#endif
        if (rt_ballot(hmax >= RT_T) != 0) {
            PROF_ADD(5, 1);
            if (rt_ballot(cnt >= RT_CQ_CAP) != 0) {  // a lane's queue is full: drain all
                PROF_ADD(11, 1);
                drain_candidates(cq, cnt, sph, o, d, a, fast, best_t, best_i EXACT_PASS);
                cnt = 0;
            }
            const float T = RT_T;
#if defined(RT_ASM_FILTER) && defined(__HIP_DEVICE_COMPILE__)
            const uint32_t m = cand_mask8(g01, g23, g45, g67, T);
#else
            const uint32_t m = ge(g01.x, T) | (ge(g01.y, T) << 1) | (ge(g23.x, T) << 2) |
                               (ge(g23.y, T) << 3) | (ge(g45.x, T) << 4) | (ge(g45.y, T) << 5) |
                               (ge(g67.x, T) << 6) | (ge(g67.y, T) << 7);
#endif
            if (m) {
                cq[cnt * 64 + lane] = (g << 8) | m;
                ++cnt;
            }
        }
    }
    PROF_MARK(1);
#ifdef RT_PROFILE
    PROF_ADD(6, wave_max_u32(cnt));
#endif
    drain_candidates(cq, cnt, sph, o, d, a, fast, best_t, best_i EXACT_PASS);
    PROF_MARK(2);
#ifdef RT_PROFILE
    PROF_ADD(13, wave_max_u32(ecnt[0]));
    PROF_ADD(14, wave_max_u32(ecnt[1]));
    {
        uint32_t sum0 = ecnt[0];
        for (int off = 32; off > 0; off >>= 1) sum0 += __shfl_xor(sum0, off);
        PROF_ADD(15, sum0);
    }
#endif
    t_out = best_t;
    return best_i;
}

// Sphere-parallel closest hit for the few live rays of a nearly empty wave
// (the end of the work queue, where a wave's remaining paths would otherwise
// each pay the whole ray-parallel list walk): one ray at a time, the 64 lanes
// split the list and run the exact reference test (intersect.wgsl:97-115) on
// their spheres in list order with the strict `<`; the wave reduction then
// takes the smallest t, ties to the smallest index -- exactly the answer of
// the sequential strict-`<` scan (intersect.wgsl:133-143).
__device__ __forceinline__ void intersect_wide(const float4* __restrict__ sph, uint32_t n,
                                               uint32_t scene_fast, uint64_t active, v3 o, v3 d,
                                               int& hi, float& t) {
    const uint32_t lane = __lane_id();
    while (active) {
        const int src = (int)__builtin_ctzll(active);
        active &= active - 1;
        const v3 ro = mk(__shfl(o.x, src), __shfl(o.y, src), __shfl(o.z, src));
        const v3 rd = mk(__shfl(d.x, src), __shfl(d.y, src), __shfl(d.z, src));
        const float l = sqrt_x(dot(rd, rd));
        const float a = l * l;  // sqr(length(r.dir)), intersect.wgsl:98
        const bool fast = ray_fast(scene_fast, ro, a);
        const float ya = fast ? rt_recip_rn(a) : a;
        float bt = VERY_FAR;
        int bi = -1;
        for (uint32_t i = lane; i < n; i += 64) {
#ifdef RT_PROFILE
            uint32_t ecnt[2];
            exact_test(sph[i], (int)i, ro, rd, a, ya, fast, bt, bi, ecnt);
#else
            exact_test(sph[i], (int)i, ro, rd, a, ya, fast, bt, bi);
#endif
        }
        for (int off = 32; off > 0; off >>= 1) {
            const float ot = __shfl_xor(bt, off);
            const int oi = __shfl_xor(bi, off);
            if (ot < bt || (ot == bt && (uint32_t)oi < (uint32_t)bi)) {
                bt = ot;
                bi = oi;
            }
        }
        if ((int)lane == src) {
            hi = bi;
            t = bt;
        }
    }
}

__device__ __forceinline__ uint32_t lanemask_lt_count(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

}  // namespace

// Lane state of one in-flight path.
struct PathState {
    v3 o, d;            // current ray
    v3 pd;              // primary direction of this pixel (generate.wgsl: pixel-only)
    v3 color;           // throughput (intersection.color, clear.wgsl:86)
    v3 bsum;            // sum of finished samples of the current block
    v3 nseed;           // normalize(seed)
    float seedx;        // seed.x (dielectric Schlick test)
    uint32_t x, y;      // global pixel
    uint32_t item;      // work item = (block - block_begin) * npix + pixel
    uint32_t s, s_end;  // current sample, end of the block
    uint32_t bounce;
};

// New sample s of the lane's pixel: seed (shade.wgsl:216-218), primary ray
// (generate.wgsl:109-129; origin = camera translation, direction cached per
// item since it depends on the pixel only), throughput 1 (clear.wgsl:86).
__device__ __forceinline__ void start_sample(const KParams& P, PathState& st) {
    const uint32_t frame = P.frame0 + st.s;
    const uint32_t idx = st.x + P.width * st.y + (P.width * P.height) * frame;
    const v3 seed = hash3(idx);
    st.seedx = seed.x;
    st.nseed = normalize_seed(seed);
    // (with the opt-in camera sampling the main loop replaces this primary
    // ray before tracing it: one call site for sampled_primary_ray)
    st.o = mk(0.0f + P.T[12], 0.0f + P.T[13], 0.0f + P.T[14]);
    st.d = st.pd;
    st.color = mk(1.0f, 1.0f, 1.0f);
    st.bounce = 0;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    const uint32_t t = __umulhi(f.m, n);
    return (t + ((n - t) >> f.sh1)) >> f.sh2;
}

// Shard pixel p -> global (x, y): rows are blocks of row_block dealt
// serpentine to the shards (rt_block_owner).
__device__ __forceinline__ void pixel_xy(const KParams& P, uint32_t p, uint32_t& x, uint32_t& y) {
    const uint32_t r = fdiv(p, P.div_width);
    x = p - r * P.width;
    const uint32_t rb = fdiv(r, P.div_row_block);
    y = rt_shard_block(rb, P.shard_count, P.shard_index) * P.row_block + (r - rb * P.row_block);
}

// k-th pixel of a block in processing order -> shard-local pixel index
// (row-major). Order: 8x8 tiles, so the 64 lanes of a wave trace a compact
// patch of the image (coherent rays: fewer sphere groups with a candidate in
// the wave); tile rows run bottom-up so the queue ends on the cheap sky rows.
__device__ __forceinline__ uint32_t order_to_pixel(const KParams& P, uint32_t k) {
    k = P.npix - 1 - k;
    const uint32_t W = P.width;
    const uint32_t tiled = P.tile_full_rows * 8 * W;
    uint32_t x, r;
    if (k < tiled) {
        const uint32_t tr = fdiv(k, P.div_8w);
        const uint32_t rem = k - tr * 8 * W;
        const uint32_t tx = rem >> 6;
        if (tx < P.tile_full_cols) {
            x = tx * 8 + (rem & 7);
            r = tr * 8 + ((rem >> 3) & 7);
        } else {  // the narrow last tile of the tile row
            const uint32_t j = rem - P.tile_full_cols * 64;
            const uint32_t jr = fdiv(j, P.div_wrem);
            x = P.tile_full_cols * 8 + (j - jr * P.tile_wrem);
            r = tr * 8 + jr;
        }
    } else {
        const uint32_t j = k - tiled;
        const uint32_t jr = fdiv(j, P.div_width);
        x = j - jr * W;
        r = P.tile_full_rows * 8 + jr;
    }
    return r * W + x;
}

// Work item -> (sample block, pixel). block_sums is indexed by (block, pixel)
// for the collect pass.
// pixel table entry (rt_primary_kernel): k-th pixel of the processing order
// -> its primary direction and (shard pixel index, x | y << 16).
struct PixelEntry {
    float4 d;       // xyz: primary direction, w: unused
    uint32_t p, xy;
    uint32_t pad0, pad1;
};

__device__ __forceinline__ void start_item(const KParams& P, PathState& st, uint32_t item,
                                           const PixelEntry* __restrict__ tab) {
    uint32_t k, s0, s1;  // pixel in processing order; the item's samples [s0, s1)
    if (item < P.main_all) {  // block item of pair q = (frame f, block b)
        const uint32_t q = fdiv(item, P.div_npix);
        k = item - q * P.npix;
        const uint32_t f = fdiv(q, P.div_nblocks);
        const uint32_t sl = (P.block_begin + (q - f * P.nblocks)) * RT_SAMPLE_BLOCK;
        s0 = P.sample_base + f * P.spp + sl;
        s1 = P.sample_base + f * P.spp + min(P.spp, sl + RT_SAMPLE_BLOCK);
    } else {  // tail item: z = 4, 2 or 1 consecutive samples, each stored on its own
        uint32_t j = item - P.main_all, z, gb, ge;
        if (j < P.ti1) {
            z = 4; gb = P.g0; ge = P.g1;
        } else if (j < P.ti2) {
            j -= P.ti1; z = 2; gb = P.g1; ge = P.g2;
        } else {
            j -= P.ti2; z = 1; gb = P.g2; ge = P.g_end;
        }
        const uint32_t g = fdiv(j, P.div_npix);
        k = j - g * P.npix;
        s0 = P.sample_base + gb + g * z;
        s1 = P.sample_base + min(gb + g * z + z, ge);
    }
    const PixelEntry& e = tab[k];
    const uint4 pxy = *reinterpret_cast<const uint4*>(&e.p);
    const float4 q4 = e.d;
    // block item: its output slot (= queue index); tail item: RT_TAIL_ITEM | k
    st.item = item < P.main_all ? item : (RT_TAIL_ITEM | k);
    st.x = pxy.y & 0xFFFFu;
    st.y = pxy.y >> 16;
    st.s = s0;
    st.s_end = s1;
    st.bsum = mk(0.0f, 0.0f, 0.0f);
    st.pd = mk(q4.x, q4.y, q4.z);
    start_sample(P, st);
}

// One path step after an intersection: shade.wgsl:199-258 for hit `hi` at t.
// Returns true when the path has finished (miss, or hit at bounce D-1).
// Written as converged stages so that each normalize (correctly rounded sqrt
// + 3 divides) is issued once per wave, not once per material branch:
//   record  : hit point + normal (intersect.wgsl:117-127)
//   pre     : normalize(reflect(d,n)) for metal, normalize(d) for dielectric
//   select  : per-material arithmetic producing the vector to normalize
//   post    : normalize(d) for the sky, the new direction otherwise
// Every lane performs exactly the reference's op sequence for its case.
__device__ __forceinline__ bool shade(const KParams& P, PathState& st, int hi, float t,
                                      const float4* __restrict__ sph,
                                      const float2* __restrict__ sph_rm,
                                      const rt_material* __restrict__ mats) {
    const bool miss = hi < 0;
    if (!miss && st.bounce == P.max_depth - 1) {  // shade.wgsl:236-238
        st.color = mk(0.0f, 0.0f, 0.0f);
        return true;
    }
    // ---- record (hit lanes)
    v3 pos = mk(0.0f, 0.0f, 0.0f), nrm = mk(0.0f, 0.0f, 0.0f);
    bool front = true;
    int refl = -1;
    float4 mc = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
    float fuzz = 0.0f, ior = 1.0f;
    if (!miss) {
        const float4 s = sph[hi];
        const float2 rm = sph_rm[hi];
        const float radius = rm.x;
        const uint32_t mi = __float_as_uint(rm.y);
        pos = add(st.o, scale(st.d, t));
        const v3 q = sub(pos, mk(s.x, s.y, s.z));
        nrm = normalize_x(div3_x(q, radius));
        if (dot(st.d, nrm) > 0.0f) {
            nrm = neg(nrm);
            front = false;
        }
        const rt_material& m = mats[mi];
        refl = m.reflectance;
        mc = *reinterpret_cast<const float4*>(m.color);
        fuzz = m.fuzziness;
        ior = m.index_of_refraction;
    }
    // ---- pre-normalize: metal normalize(reflect(d, n)) (shade.wgsl:140),
    //      dielectric unit_dir = normalize(d) (shade.wgsl:169)
    v3 un = mk(0.0f, 0.0f, 0.0f);
    if (refl == RT_METALLIC || refl == RT_DIELECTRIC)
        un = normalize_x(refl == RT_METALLIC ? reflect(st.d, nrm) : st.d);
    // ---- select
    v3 v = st.d;           // vector to normalize (sky: d, shade.wgsl:190)
    bool post = true;      // false: dielectric reflection keeps reflect(d, n) unnormalized
    v3 e_dir_raw = mk(0.0f, 0.0f, 0.0f);
    if (refl == RT_LAMBERTIAN) {  // shade.wgsl:121-124
        const v3 dest = add(add(pos, nrm), st.nseed);
        v = sub(dest, pos);
    } else if (refl == RT_METALLIC) {  // shade.wgsl:141-142
        v = add(un, scale(st.nseed, fuzz));
    } else if (refl == RT_DIELECTRIC) {  // shade.wgsl:164-180
        float ratio = ior;
        if (front) ratio = 1.0f / ior;
        const float cos_theta = fminf(dot(neg(un), nrm), 1.0f);
        const float sin_theta = sqrt_x(1.0f - cos_theta * cos_theta);
        const bool cannot_refract = ratio * sin_theta > 1.0f;
        float r0 = (1.0f - ratio) / (1.0f + ratio);  // reflectance(), shade.wgsl:156-161
        r0 = r0 * r0;
        const float xr = 1.0f - cos_theta;
        const float x2 = xr * xr;
        const float refl_p = r0 + (1.0f - r0) * ((x2 * x2) * xr);
        if (cannot_refract || refl_p > st.seedx) {
            e_dir_raw = reflect(st.d, nrm);
            post = false;
        } else {  // refract(unit_dir, n, ratio), shade.wgsl:148-153
            const v3 perp = scale(add(un, scale(nrm, cos_theta)), ratio);
            const float lp = length_x(perp);
            const float par = -sqrt_x(fabsf(1.0f - (lp * lp)));
            v = add(perp, scale(nrm, par));
        }
    }
    // ---- post-normalize
    v3 vn = mk(0.0f, 0.0f, 0.0f);
    if (post) vn = normalize_x(v);
    if (miss) {  // miss(), shade.wgsl:189-197, color *= sky
        const float tt = 0.5f * vn.y + 1.0f;
        const float omt = (1.0f - tt) * 1.0f;
        st.color = mul(st.color, mk(omt + tt * 0.5f, omt + tt * 0.7f, omt + tt * 1.0f));
        return true;
    }
    if (refl == RT_LAMBERTIAN) {
        st.o = pos;  // no offset (shade.wgsl:123)
        st.d = vn;
        st.color = mul(st.color, mk(mc.x, mc.y, mc.z));
    } else {
        st.o = add(pos, scale(nrm, EPSILON));  // shade.wgsl:139, 182
        st.d = post ? vn : e_dir_raw;
        if (refl == RT_METALLIC) st.color = mul(st.color, mk(mc.x, mc.y, mc.z));
    }
    ++st.bounce;
    return false;
}

#ifdef RT_CHUNK_TRACE
#define RT_CHUNK_TRACE_MAX (1u << 22)
__device__ unsigned long long g_chunk_trace[RT_CHUNK_TRACE_MAX];
__device__ unsigned long long g_chunk_clk[RT_CHUNK_TRACE_MAX];  // shader clock (s_memtime)
#endif
#ifdef RT_WAVE_TRACE
// Diagnostic build only (-DRT_WAVE_TRACE): per wave (start, end, exhausted-at)
// in s_memrealtime ticks (100 MHz) and (iterations, items) -- the schedule's
// tail shape. Read back with rt_debug_wave_trace().
#define RT_TRACE_MAX_WAVES 32768
__device__ unsigned long long g_wave_trace[RT_TRACE_MAX_WAVES * 4];
#endif

#ifndef RT_PARAMS_HOLD
// The launch parameters re-read from the kernarg segment where they are used
// (scalar loads) instead of being held in SGPRs across the whole loop: the
// volatile asm makes the pointer opaque per iteration, so no load of a field
// is hoisted out of the loop. Held, they spilled ~47 SGPRs to VGPR lanes
// (~110 v_readlane/v_writelane in the loop, one VGPR to scratch); re-read:
// no spills, 76 VGPRs, -1.8 % VALU, -1.5 % time (RT_PARAMS_HOLD: the old form).
__device__ __forceinline__ const KParams& fresh_params() {
    typedef __attribute__((address_space(4))) const KParams cKParams;
    cKParams* p = (cKParams*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const KParams*)p;
}
#endif

__global__ __launch_bounds__(RT_BLOCK_THREADS, RT_MIN_WAVES_PER_SIMD) void rt_render_kernel(
    KParams P, const float4* grp, const float4* __restrict__ sph,
    const float2* __restrict__ sph_rm, const rt_material* __restrict__ mats,
    const PixelEntry* __restrict__ tab, float4* __restrict__ block_sums,
    uint32_t* __restrict__ work_counter,
    unsigned long long* __restrict__ seg_counter, unsigned long long* __restrict__ dbg) {
    const uint32_t lane = threadIdx.x & 63u;
    PROF_DECL
    PROF_START();
#ifdef RT_PROFILE
    const unsigned long long t_begin = prof_.last;
#endif
    __shared__ uint32_t s_cq[RT_BLOCK_THREADS * RT_CQ_CAP];  // per-lane candidate queues
    uint32_t* cq = s_cq + (threadIdx.x / 64u) * (64u * RT_CQ_CAP);
#ifdef RT_SPHERES_LDS
    // Experiment variant: the filter reads the sphere groups from LDS (staged
    // once per workgroup) instead of the scalar cache.
    extern __shared__ float4 s_grp[];
    for (uint32_t i = threadIdx.x; i < (P.ngroups + 1) * 8; i += RT_BLOCK_THREADS) s_grp[i] = grp[i];
    __syncthreads();
    grp = s_grp;
#endif
    const uint32_t total = P.main_all + P.tail_items;
#ifdef RT_WAVE_TRACE
#ifdef RT_WAVE_TRACE_LITE
    if (lane == 0) {  // stored at once: nothing stays live across the loop
        const uint32_t wid0 = blockIdx.x * (RT_BLOCK_THREADS / 64) + threadIdx.x / 64;
        if (wid0 < RT_TRACE_MAX_WAVES) g_wave_trace[wid0 * 4 + 0] = __builtin_amdgcn_s_memrealtime();
    }
    const unsigned long long tr_t0 = 0;
#else
    const unsigned long long tr_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    unsigned long long tr_ex = 0;
    uint32_t tr_iters = 0, tr_items = 0, tr_after = 0;
#ifdef RT_WAVE_TRACE_LITE  // start/end only: keeps the product's register budget
#define TR_COUNT(x)
#else
#define TR_COUNT(x) x
#endif
#endif
    // primary-hit reuse: the primary ray is pixel-only unless the opt-in
    // camera sampling varies it per sample
    const bool use_cache =
        (P.flags & (RT_FLAG_NO_PRIMARY_CACHE | RT_FLAG_JITTER | RT_FLAG_THIN_LENS)) == 0;

    PathState st;
    bool has_item = false;
    uint32_t q_next = 0, q_end = 0;  // wave-uniform chunk of work items
    bool exhausted = false;
    uint32_t traced = 0, segs = 0;  // wave totals (wave-uniform: SGPRs, not a VGPR per lane)
    int cache_hi = -1;      // primary hit of this item's pixel (generate.wgsl: pixel-only ray)
    float cache_t = 0.0f;
    // Chunk prefetch: the atomic for the wave's NEXT chunk is issued as soon as
    // the current one is taken, so its round trip to the device-scope counter
    // (one address shared by every wave of the chip) overlaps a whole filter
    // walk instead of stalling the refill. Every prefetched chunk is consumed:
    // a wave only stops after consuming a base >= total, and issues no further
    // prefetch from then on.
    uint32_t iter = 0;            // loop iterations of this wave (wave-uniform)
    // hardware wave slot on its SIMD (HW_ID[3:0]): distinct for co-resident waves
    const uint32_t wave_slot = __builtin_amdgcn_s_getreg((3 << 11) | 4);
    uint32_t pref = 0;            // lane 0: base of the prefetched chunk
    uint32_t pref_chunk = 0;      // its size (0 = none in flight)

    for (;;) {
#ifndef RT_PARAMS_HOLD
        const KParams& P = fresh_params();
#endif
        // ---- refill: lanes without an item take the next ones (wave ballot)
        uint64_t need = rt_ballot(!has_item);
        while (need != 0 && !exhausted) {
            if (q_next >= q_end) {
                // big chunks keep the counter cold; small ones near the end of
                // the queue keep the waves' finishing times together
                uint32_t chunk, base = 0;
                if (pref_chunk) {
                    chunk = pref_chunk;
                    base = pref;
                } else {
                    chunk = q_end >= P.tail_start ? RT_WAVE_CHUNK_TAIL : RT_WAVE_CHUNK;
                    if (lane == 0) base = atomicAdd(work_counter, chunk);
                }
                base = __shfl(base, 0);
                pref_chunk = 0;
                if (base >= total) {
#ifdef RT_WAVE_TRACE
                    TR_COUNT(tr_ex = __builtin_amdgcn_s_memrealtime());
#endif
                    exhausted = true;
                    break;
                }
                q_next = base;
                q_end = min(base + chunk, total);
#ifdef RT_CHUNK_TRACE
                // diagnostic: time at which each 64-item slice of the queue is taken
                if (lane == 0 && (base >> 6) < RT_CHUNK_TRACE_MAX) {
                    g_chunk_trace[base >> 6] = __builtin_amdgcn_s_memrealtime();
                    g_chunk_clk[base >> 6] = __builtin_amdgcn_s_memtime();
                }
#endif
                if (P.prefetch) {
                    pref_chunk = q_end >= P.tail_start ? RT_WAVE_CHUNK_TAIL : RT_WAVE_CHUNK;
                    if (lane == 0) pref = atomicAdd(work_counter, pref_chunk);
                }
            }
            const uint32_t avail = q_end - q_next;
            const uint32_t rank = lanemask_lt_count(need);
            const uint32_t cnt = (uint32_t)__popcll(need);
            if (!has_item && rank < avail) {
                start_item(P, st, q_next + rank, tab);
                has_item = true;
            }
#ifdef RT_WAVE_TRACE
            TR_COUNT(tr_items += min(avail, cnt));
#endif
            q_next += min(avail, cnt);
            need = rt_ballot(!has_item);
        }
        if (rt_ballot(has_item) == 0) break;
        // ---- issue fairness: the SIMD arbiter issues by priority, then age
        // (MI355X_MICROARCH.md "Two waves per SIMD"), so in a persistent
        // launch the waves of a SIMD progress at geometrically falling rates
        // by dispatch order (measured per iteration, 1st..6th wave: 17, 21,
        // 33, 57, 113, 248 us) and the youngest waves' items become the
        // launch's stragglers. Mode 1 (default) rotates the priority level
        // with the wave's iteration count offset by its hardware wave slot
        // (20, 24, 30, 42, 69, 144 us); mode 3 rotates it by wall time
        // (s_memrealtime >> prio_shift), all waves of a SIMD stepping together.
        if (P.prio_mode) {
            const uint32_t lvl =
                P.prio_mode == 1
                    ? (iter + wave_slot) & 3u
                    : ((uint32_t)(__builtin_amdgcn_s_memrealtime() >> P.prio_shift) + wave_slot) & 3u;
            switch (lvl) {
                case 0: __builtin_amdgcn_s_setprio(0); break;
                case 1: __builtin_amdgcn_s_setprio(1); break;
                case 2: __builtin_amdgcn_s_setprio(2); break;
                default: __builtin_amdgcn_s_setprio(3); break;
            }
        }
        ++iter;
#ifdef RT_WAVE_TRACE
        TR_COUNT(++tr_iters);
        TR_COUNT(tr_after += exhausted ? 1u : 0u);
#endif
        PROF_MARK(0);
        PROF_ADD(4, 1);
        PROF_ADD(9, (unsigned long long)__popcll(rt_ballot(has_item)));

        // ---- opt-in camera sampling: a lane at bounce 0 holds a fresh sample
        // whose primary ray varies per sample (no primary-hit reuse then)
        if ((P.flags & (RT_FLAG_JITTER | RT_FLAG_THIN_LENS)) && has_item && st.bounce == 0) {
            const uint32_t idx = st.x + P.width * st.y + (P.width * P.height) * (P.frame0 + st.s);
            sampled_primary_ray(P, st.x, st.y, idx, st.o, st.d);
        }

        // ---- intersect (intersect.wgsl:145-163): every lane with an item holds
        // a ray that needs tracing here.
        int hi = -1;
        float t = VERY_FAR;
        const uint64_t live = rt_ballot(has_item);
        if ((uint32_t)__popcll(live) <= P.wide_max) {  // nearly empty wave: sphere-parallel
            intersect_wide(sph, P.nspheres, P.scene_fast, live, st.o, st.d, hi, t);
        } else if (has_item) {
            hi = intersect_world(grp, sph, P.ngroups, P.scene_fast, st.o, st.d, t, cq
#ifdef RT_PROFILE
                                 , prof_
#endif
                                 );
        }
        traced += (uint32_t)__popcll(live);
        if (has_item) {
            if (st.bounce == 0) {  // first sample of the block: remember the primary hit
                cache_hi = hi;
                cache_t = t;
            }
        }
        // ---- shade; a finished path starts the next sample, whose primary hit
        // is reused (result-identical) so the lane goes on to its bounce-1 ray.
        bool shading = has_item;
        PROF_MARK(12);  // bookkeeping between the drain and the shading loop
        // uniform loop (the segment count is a wave total): one round per
        // path step, lanes without a step to shade idle through the round
        for (;;) {
            const uint64_t sh = rt_ballot(shading);
            if (sh == 0) break;
            segs += (uint32_t)__popcll(sh);
            if (shading) {
                const bool done = shade(P, st, hi, t, sph, sph_rm, mats);
                shading = false;
                if (done) {
                    // path finished: accumulate (collect.wgsl:115-120, blocked);
                    // a tail item stores every sample's colour for the collect
                    if (st.item & RT_TAIL_ITEM) {
                        const v3 c = add(mk(0.0f, 0.0f, 0.0f), st.color);
                        block_sums[P.main_all +
                                   (st.s - P.sample_base - P.g0) * P.npix + (st.item & ~RT_TAIL_ITEM)] =
                            make_float4(c.x, c.y, c.z, 0.0f);
                    } else {
                        st.bsum = add(st.bsum, st.color);
                    }
                    ++st.s;
                    if (st.s < st.s_end) {
                        start_sample(P, st);
                        if (use_cache) {
                            hi = cache_hi;
                            t = cache_t;
                            shading = true;
                        }
                    } else {
                        if (!(st.item & RT_TAIL_ITEM))
                            block_sums[st.item] = make_float4(st.bsum.x, st.bsum.y, st.bsum.z, 0.0f);
                        has_item = false;
                    }
                }
            }
        }
        PROF_MARK(3);
    }

#ifdef RT_PROFILE
    PROF_MARK(7);
    prof_.c[8] = __builtin_amdgcn_s_memtime() - t_begin;
    if (lane == 0)
        for (int i = 0; i < 16; ++i) atomicAdd(dbg + i, prof_.c[i]);
#endif
#ifdef RT_WAVE_TRACE
    {
        const uint32_t wid = blockIdx.x * (RT_BLOCK_THREADS / 64) + threadIdx.x / 64;
        if (lane == 0 && wid < RT_TRACE_MAX_WAVES) {
#ifndef RT_WAVE_TRACE_LITE
            g_wave_trace[wid * 4 + 0] = tr_t0;
#else
            (void)tr_t0;
#endif
            g_wave_trace[wid * 4 + 1] = __builtin_amdgcn_s_memrealtime();
#ifdef RT_PROFILE  // combined diagnostic build: where the wave ran (HW_ID, XCC_ID)
            g_wave_trace[wid * 4 + 2] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                                        ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20)
                                         << 32);
            (void)tr_ex;
#else
            g_wave_trace[wid * 4 + 2] = tr_ex;
#endif
#ifdef RT_PROFILE  // combined diagnostic build: exact tests (wave max, summed) instead of items
            g_wave_trace[wid * 4 + 3] = ((unsigned long long)min(prof_.c[13], 0xFFFFFFFFull) << 32) |
                                        (min(tr_after, 65535u) << 16) | min(tr_iters, 65535u);
#else
            g_wave_trace[wid * 4 + 3] = ((unsigned long long)tr_items << 32) |
                                        (min(tr_after, 65535u) << 16) | min(tr_iters, 65535u);
#endif
        }
    }
#endif
    // ---- segment counts: one atomic per wave
    if (lane == 0) {
        atomicAdd(seg_counter, (unsigned long long)segs);
        atomicAdd(seg_counter + 1, (unsigned long long)traced);
    }
}

// Pixel table, once per frame: for the k-th pixel of the processing order
// its shard pixel index, global (x, y) and primary ray direction
// (generate.wgsl:66-126; the direction depends on the pixel only: lens
// offset 0, no jitter).
__global__ void rt_primary_kernel(KParams P, PixelEntry* __restrict__ tab) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P.npix) return;
    const uint32_t p = order_to_pixel(P, k);
    uint32_t x, y;
    pixel_xy(P, p, x, y);
    v3 o, d;
    primary_ray(P, x, y, o, d);
    PixelEntry e;
    e.d = make_float4(d.x, d.y, d.z, 0.0f);
    e.p = p;
    e.xy = x | (y << 16);
    e.pad0 = e.pad1 = 0;
    tab[k] = e;
}

// Batch closest-hit query (rt_intersect): one ray per lane, same intersect_world.
__global__ __launch_bounds__(RT_BLOCK_THREADS) void rt_intersect_kernel(
    const float4* __restrict__ grp, const float4* __restrict__ sph, uint32_t ngroups,
    uint32_t scene_fast, const float* __restrict__ rays, uint32_t n, int* __restrict__ out_i,
    float* __restrict__ out_t) {
    __shared__ uint32_t s_cq[RT_BLOCK_THREADS * RT_CQ_CAP];
    uint32_t* cq = s_cq + (threadIdx.x / 64u) * (64u * RT_CQ_CAP);
#ifdef RT_PROFILE
    PROF_DECL
    PROF_START();
#endif
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* r = rays + (size_t)i * 6;
    float t;
    const int hi = intersect_world(grp, sph, ngroups, scene_fast, mk(r[0], r[1], r[2]),
                                   mk(r[3], r[4], r[5]),
                                   t, cq
#ifdef RT_PROFILE
                                   , prof_
#endif
                                   );
    out_i[i] = hi;
    out_t[i] = t;
}

// Fold one frame's block sums (launch frame f = blockIdx.y) into acc (block
// order) and, on the frame's last pass, write out = acc / spp with alpha 1
// (collect.wgsl:115-125). One thread per pixel of the processing order k
// (pixel table -> image pixel p). Block b of frame f is pair q = f*nblocks +
// b: a block item's sum at slot q*npix + k if q < qmain, else a tail block
// whose samples' colours sit at main_all + (g - g0)*npix + k (g = f*spp + s)
// and are summed here exactly as a lane sums a block, ((0 + c0) + c1) + ...,
// in sample order, then folded like any other block.
// Progressive mode (rt_render_progressive): on the last pass the frame's sum
// is folded into the running sum, prog = prog + sum (prog_mode 2) or
// prog = sum (1, reset), and out = prog / total_spp.
__global__ void rt_collect_kernel(KParams P, const PixelEntry* __restrict__ tab,
                                  const float4* __restrict__ block_sums,
                                  float4* __restrict__ acc, int first_pass,
                                  int last_pass, float spp, float4* __restrict__ out,
                                  float4* __restrict__ prog, int prog_mode, float prog_total) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P.npix) return;
    const uint32_t f = blockIdx.y;
    out += (size_t)f * P.npix;
    const uint32_t p = tab[k].p;
    float ax = 0.0f, ay = 0.0f, az = 0.0f;
    bool have = !first_pass;
    if (have) {
        const float4 v = acc[p];
        ax = v.x; ay = v.y; az = v.z;
    }
    for (uint32_t b = 0; b < P.nblocks; ++b) {
        const uint32_t q = f * P.nblocks + b;
        float4 v;
        if (q < P.qmain) {
            v = block_sums[(size_t)q * P.npix + k];
        } else {  // a tail block: its samples' colours, summed in sample order
            const uint32_t sl = (P.block_begin + b) * RT_SAMPLE_BLOCK;
            const uint32_t g_end = f * P.spp + min(P.spp, sl + RT_SAMPLE_BLOCK);
            v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            for (uint32_t g = f * P.spp + sl; g < g_end; ++g) {
                const float4 c = block_sums[(size_t)P.main_all + (size_t)(g - P.g0) * P.npix + k];
                v.x = v.x + c.x; v.y = v.y + c.y; v.z = v.z + c.z;
            }
        }
        if (have) {
            ax = ax + v.x; ay = ay + v.y; az = az + v.z;
        } else {
            ax = v.x; ay = v.y; az = v.z;
            have = true;
        }
    }
    if (!last_pass) {
        acc[p] = make_float4(ax, ay, az, 0.0f);
    } else if (prog_mode == 0) {
        out[p] = make_float4(ax / spp, ay / spp, az / spp, 1.0f);
    } else {
        if (prog_mode == 2) {
            const float4 v = prog[p];
            ax = v.x + ax; ay = v.y + ay; az = v.z + az;
        }
        prog[p] = make_float4(ax, ay, az, 0.0f);
        out[p] = make_float4(ax / prog_total, ay / prog_total, az / prog_total, 1.0f);
    }
}

// Display encode: linear RGBA32F -> sRGB RGBA8 (IEC 61966-2-1 transfer curve),
// channels clamped to [0, 1] (NaN -> 0), alpha 255. The reference shows the
// linear texture through Bevy's sprite pass (ray_trace_output.rs:62-77).
__global__ void rt_srgb8_kernel(const float4* __restrict__ in, uchar4* __restrict__ out,
                                uint64_t npix) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const float4 v = in[i];
    const float c[3] = {v.x, v.y, v.z};
    unsigned char q[3];
    for (int k = 0; k < 3; ++k) {
        float x = c[k] > 0.0f ? fminf(c[k], 1.0f) : 0.0f;  // NaN -> 0
        x = x <= 0.0031308f ? 12.92f * x : 1.055f * powf(x, 1.0f / 2.4f) - 0.055f;
        q[k] = (unsigned char)fminf(fmaxf(rintf(x * 255.0f), 0.0f), 255.0f);
    }
    out[i] = make_uchar4(q[0], q[1], q[2], 255);
}

// gathered: shard_count slabs of max_rows*W float4; image: H*W float4.
__global__ void rt_assemble_kernel(const float4* __restrict__ gathered, uint32_t max_rows,
                                   float4* __restrict__ image, uint32_t width, uint32_t height,
                                   uint32_t row_block, uint32_t shard_count) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)width * height) return;
    const uint32_t y = (uint32_t)(i / width);
    const uint32_t x = (uint32_t)(i - (size_t)y * width);
    const uint32_t blk = y / row_block;
    const uint32_t k = rt_block_owner(blk, shard_count);
    const uint32_t r = (blk / shard_count) * row_block + (y % row_block);
    image[i] = gathered[((size_t)k * max_rows + r) * width + x];
}

extern "C" {

hipError_t rt_launch_render(const KParams* P, const float4* grp, const float4* sph,
                            const float2* sph_rm, const rt_material* mats, const float4* pd,
                            float4* block_sums, uint32_t* work_counter,
                            unsigned long long* seg_counter, uint32_t grid, hipStream_t stream) {
#ifdef RT_SPHERES_LDS
    const size_t dyn = (size_t)(P->ngroups + 1) * 8 * sizeof(float4);
#else
    const size_t dyn = 0;
#endif
    hipLaunchKernelGGL(rt_render_kernel, dim3(grid), dim3(RT_BLOCK_THREADS), dyn, stream, *P, grp,
                       sph, sph_rm, mats, reinterpret_cast<const PixelEntry*>(pd), block_sums,
                       work_counter, seg_counter, seg_counter + 2);
    return hipGetLastError();
}

hipError_t rt_launch_primary(const KParams* P, float4* pd, hipStream_t stream) {
    const uint32_t T = 256;
    hipLaunchKernelGGL(rt_primary_kernel, dim3((P->npix + T - 1) / T), dim3(T), 0, stream, *P,
                       reinterpret_cast<PixelEntry*>(pd));
    return hipGetLastError();
}

hipError_t rt_launch_collect(const KParams* P, const float4* pd, const float4* block_sums,
                             float4* acc, int first_pass, int last_pass, float spp, float4* out,
                             float4* prog, int prog_mode, float prog_total, hipStream_t stream) {
    const uint32_t T = 256;
    hipLaunchKernelGGL(rt_collect_kernel, dim3((P->npix + T - 1) / T, P->nframes), dim3(T), 0, stream, *P,
                       reinterpret_cast<const PixelEntry*>(pd), block_sums, acc, first_pass,
                       last_pass, spp, out, prog, prog_mode, prog_total);
    return hipGetLastError();
}

hipError_t rt_launch_srgb8(const float4* in, uchar4* out, uint64_t npix, hipStream_t stream) {
    const uint32_t T = 256;
    hipLaunchKernelGGL(rt_srgb8_kernel, dim3((uint32_t)((npix + T - 1) / T)), dim3(T), 0, stream,
                       in, out, npix);
    return hipGetLastError();
}

hipError_t rt_launch_assemble(const float4* gathered, uint32_t max_rows, float4* image,
                              uint32_t width, uint32_t height, uint32_t row_block,
                              uint32_t shard_count, hipStream_t stream) {
    const uint32_t T = 256;
    const size_t n = (size_t)width * height;
    hipLaunchKernelGGL(rt_assemble_kernel, dim3((uint32_t)((n + T - 1) / T)), dim3(T), 0, stream,
                       gathered, max_rows, image, width, height, row_block, shard_count);
    return hipGetLastError();
}

hipError_t rt_launch_intersect(const float4* grp, const float4* sph, uint32_t ngroups,
                               uint32_t scene_fast, const float* rays, uint32_t n, int* out_i,
                               float* out_t, hipStream_t stream) {
    const uint32_t T = RT_BLOCK_THREADS;
    hipLaunchKernelGGL(rt_intersect_kernel, dim3((n + T - 1) / T), dim3(T), 0, stream, grp, sph,
                       ngroups, scene_fast, rays, n, out_i, out_t);
    return hipGetLastError();
}

#ifdef RT_WAVE_TRACE
int rt_debug_wave_trace(unsigned long long* out, uint32_t max_waves) {
    if (max_waves > RT_TRACE_MAX_WAVES) max_waves = RT_TRACE_MAX_WAVES;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_trace),
                               (size_t)max_waves * 4 * sizeof(unsigned long long)) == hipSuccess
               ? (int)max_waves : -1;
}
#endif

#ifdef RT_CHUNK_TRACE
int rt_debug_chunk_trace(unsigned long long* out, unsigned long long* clk, uint32_t n) {
    if (n > RT_CHUNK_TRACE_MAX) n = RT_CHUNK_TRACE_MAX;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chunk_trace), (size_t)n * 8) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_chunk_clk), (size_t)n * 8) != hipSuccess) return -1;
    return (int)n;
}
#endif

// Diagnostic entry (not part of include/rt_hip.h; tests/test_gpu_math.py):
// the hot path's guarded short forms on caller-given operands, to compare with
// the IEEE operations on zeros, denormals, huge values, inf and NaN.
// mode 0: out[i] = sqrt_x(in[i]); 1: out[3i..3i+2] = normalize_x(in[3i..3i+2]);
// 2: out[3i..3i+2] = div3_x(in[4i..4i+2], in[4i+3]);
// 3: out[i] = div_x(in[2i], in[2i+1], recip_or_nan(in[2i+1])).
__global__ void rt_math_kernel(int mode, const float* __restrict__ in, uint32_t n,
                               float* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mode == 0) {
        out[i] = sqrt_x(in[i]);
    } else if (mode == 1) {
        const v3 r = normalize_x(mk(in[3 * i], in[3 * i + 1], in[3 * i + 2]));
        out[3 * i] = r.x; out[3 * i + 1] = r.y; out[3 * i + 2] = r.z;
    } else if (mode == 2) {
        const v3 r = div3_x(mk(in[4 * i], in[4 * i + 1], in[4 * i + 2]), in[4 * i + 3]);
        out[3 * i] = r.x; out[3 * i + 1] = r.y; out[3 * i + 2] = r.z;
    } else {
        out[i] = div_x(in[2 * i], in[2 * i + 1], recip_or_nan(in[2 * i + 1]));
    }
}

int rt_debug_math(int mode, const float* in_device, uint32_t n, float* out_device) {
    if (mode < 0 || mode > 3 || (n && (!in_device || !out_device))) return -1;
    if (!n) return 0;
    hipLaunchKernelGGL(rt_math_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, mode, in_device, n,
                       out_device);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}

hipError_t rt_render_occupancy(int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, rt_render_kernel,
                                                        RT_BLOCK_THREADS, 0);
}

}  // extern "C"
