// rt_dev_intersect.h -- closest hit: the exact reference test, the packed
// conservative filter (filter8), candidate queues, intersect_world / intersect_wide
// (intersect.wgsl:94-143)
// (included by rt_kernels.hip only: one translation unit, device code)
#pragma once

namespace {

// ---- diagnostic build only (-DRT_PROFILE): per-wave phase clocks (s_memtime)
// and wave-level event counts, summed into a debug buffer. Never compiled into
// the product library.
#ifdef RT_PROFILE
// c[0..3], c[7], c[12], c[16]: phase clocks (rt_kernels.hip PROF_MARK
// sites), c[26] the diagnostic reductions' own time; the rest event counts
// (tools/executed.py names them all).
struct Prof {
    unsigned long long c[RT_DBG_COUNTERS];
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
//
// CULL (the culled list of rt_render_cull_kernel, rt_api.cpp build_cull): the
// list is spatially permuted, so the winner is the lexicographic minimum of
// (t, original index perm[idx]) -- the sequential strict-`<` scan's answer in
// the original order (intersect.wgsl:137) whatever order the candidates come
// in. perm is read only on an exact tie.
// LEX (the matrix-core filter, candidates in any order): the lexicographic
// minimum of (t, index), the sequential scan's answer without a permutation.
// The exact test: calls take(root) with the nearer root in [EPSILON,
// VERY_FAR] (the far one when the near one is out of range; NaN when the
// arithmetic is) and returns without a call when the sphere is missed.
template <bool FAST, typename Take>
__device__ __forceinline__ void exact_core(float4 s, v3 o, v3 d, float a, float ya,
                                           Take&& take EXACT_ARGS) {
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
    take(root);
}

// One exact test against the running best (a NaN root loses every comparison).
template <bool FAST, bool CULL, bool LEX = false>
__device__ __forceinline__ void exact_body(float4 s, int idx, v3 o, v3 d, float a, float ya,
                                           float& best_t, int& best_i,
                                           const uint32_t* perm EXACT_ARGS) {
    exact_core<FAST>(s, o, d, a, ya, [&](float root) {
        if (CULL) {
            if (root <= best_t &&
                (root < best_t || (best_i >= 0 && perm[idx] < perm[best_i]))) {
                best_t = root;
                best_i = idx;
            }
        } else if (LEX) {
            if (root < best_t || (root == best_t && idx < best_i)) {
                best_t = root;
                best_i = idx;
            }
        } else if (root < best_t) {
            best_t = root;
            best_i = idx;
        }
    } EXACT_PASS);
}

template <bool CULL>
__device__ __forceinline__ void exact_test(float4 s, int idx, v3 o, v3 d, float a, float ya,
                                           bool fast, float& best_t, int& best_i,
                                           const uint32_t* perm EXACT_ARGS) {
    if (fast)
        exact_body<true, CULL>(s, idx, o, d, a, ya, best_t, best_i, perm EXACT_PASS);
    else
        exact_body<false, CULL>(s, idx, o, d, a, ya, best_t, best_i, perm EXACT_PASS);
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
// the four pair chains are interleaved, so dependent ops are 4 apart (no
// wait states, and a lone wave in the queue tail issues back to back). Op
// order per pair is exactly filter2's. Every ray constant is held as a
// duplicated VGPR pair: no op_sel / op_sel_hi broadcast of one half of a pair.
// The broadcast form (4 pairs, 7 VGPRs fewer) gave wrong H values, on a few
// waves of some launches only, in a kernel whose other waves ran the
// matrix-core filter on the same SIMDs (tools/isect_diag.py: ~10-100 of
// 400,000 adversarial rays per launch, every one in a VALU-walk wave; the
// same asm without op_sel, or the compiler's filter2, exact over 8 launches;
// DESIGN.md §4.2).
struct RayP {
    f2 dx, dy, dz, k1, ox, oy, oz;  // (-dn, k1, o2) duplicated in both halves
    float T;
};

__device__ __forceinline__ RayP ray_pack(const RayF& r) {
    RayP p;
    p.dx = r.dx; p.dy = r.dy; p.dz = r.dz; p.k1 = r.k1;
    p.ox = r.o2x; p.oy = r.o2y; p.oz = r.o2z;
    p.T = r.T;
    return p;
}

__device__ __forceinline__ void filter8(const RayP& R, f2 cxa, f2 cxb, f2 cxc, f2 cxd, f2 cya,
                                        f2 cyb, f2 cyc, f2 cyd, f2 cza, f2 czb, f2 czc, f2 czd,
                                        f2 sa, f2 sb, f2 sc, f2 sd, f2& ha, f2& hb, f2& hc,
                                        f2& hd, float& hmax) {
    // compiler-allocated registers (early-clobber: every output is written
    // before the last input is read); the dependent packed ops are 4 apart,
    // above the 1 wait state hipcc itself puts after a v_pk_fma_f32 whose
    // result the next VALU reads (tools/hazard_audit.py rule R1)
    asm volatile(
        // hb = k1 + (-dnx) cx + (-dny) cy + (-dnz) cz
        "v_pk_fma_f32 %[ha], %[dx], %[cxa], %[k1]\n\t"
        "v_pk_fma_f32 %[hb], %[dx], %[cxb], %[k1]\n\t"
        "v_pk_fma_f32 %[hc], %[dx], %[cxc], %[k1]\n\t"
        "v_pk_fma_f32 %[hd], %[dx], %[cxd], %[k1]\n\t"
        "v_pk_fma_f32 %[ha], %[dy], %[cya], %[ha]\n\t"
        "v_pk_fma_f32 %[hb], %[dy], %[cyb], %[hb]\n\t"
        "v_pk_fma_f32 %[hc], %[dy], %[cyc], %[hc]\n\t"
        "v_pk_fma_f32 %[hd], %[dy], %[cyd], %[hd]\n\t"
        "v_pk_fma_f32 %[ha], %[dz], %[cza], %[ha]\n\t"
        "v_pk_fma_f32 %[hb], %[dz], %[czb], %[hb]\n\t"
        "v_pk_fma_f32 %[hc], %[dz], %[czc], %[hc]\n\t"
        "v_pk_fma_f32 %[hd], %[dz], %[czd], %[hd]\n\t"
        // H = hb^2 + S + o2z cz + o2y cy + o2x cx
        "v_pk_fma_f32 %[ha], %[ha], %[ha], %[sa]\n\t"
        "v_pk_fma_f32 %[hb], %[hb], %[hb], %[sb]\n\t"
        "v_pk_fma_f32 %[hc], %[hc], %[hc], %[sc]\n\t"
        "v_pk_fma_f32 %[hd], %[hd], %[hd], %[sd]\n\t"
        "v_pk_fma_f32 %[ha], %[oz], %[cza], %[ha]\n\t"
        "v_pk_fma_f32 %[hb], %[oz], %[czb], %[hb]\n\t"
        "v_pk_fma_f32 %[hc], %[oz], %[czc], %[hc]\n\t"
        "v_pk_fma_f32 %[hd], %[oz], %[czd], %[hd]\n\t"
        "v_pk_fma_f32 %[ha], %[oy], %[cya], %[ha]\n\t"
        "v_pk_fma_f32 %[hb], %[oy], %[cyb], %[hb]\n\t"
        "v_pk_fma_f32 %[hc], %[oy], %[cyc], %[hc]\n\t"
        "v_pk_fma_f32 %[hd], %[oy], %[cyd], %[hd]\n\t"
        "v_pk_fma_f32 %[ha], %[ox], %[cxa], %[ha]\n\t"
        "v_pk_fma_f32 %[hb], %[ox], %[cxb], %[hb]\n\t"
        "v_pk_fma_f32 %[hc], %[ox], %[cxc], %[hc]\n\t"
        "v_pk_fma_f32 %[hd], %[ox], %[cxd], %[hd]"
        : [ha] "=&v"(ha), [hb] "=&v"(hb), [hc] "=&v"(hc), [hd] "=&v"(hd)
        : [dx] "v"(R.dx), [dy] "v"(R.dy), [dz] "v"(R.dz), [k1] "v"(R.k1), [ox] "v"(R.ox),
          [oy] "v"(R.oy), [oz] "v"(R.oz), [cxa] "s"(cxa), [cxb] "s"(cxb), [cxc] "s"(cxc),
          [cxd] "s"(cxd), [cya] "s"(cya), [cyb] "s"(cyb), [cyc] "s"(cyc), [cyd] "s"(cyd),
          [cza] "s"(cza), [czb] "s"(czb), [czc] "s"(czc), [czd] "s"(czd), [sa] "s"(sa),
          [sb] "s"(sb), [sc] "s"(sc), [sd] "s"(sd));
    // group max of the 8 H (v_max3 drops a quiet-NaN operand, as fmaxf; in
    // asm so that no canonicalising v_max is put in front of each operand)
    asm volatile(
        "v_max3_f32 %[hm], %[h0], %[h1], %[h2]\n\t"
        "v_max3_f32 %[hm], %[hm], %[h3], %[h4]\n\t"
        "v_max3_f32 %[hm], %[hm], %[h5], %[h6]\n\t"
        "v_max_f32 %[hm], %[hm], %[h7]"
        : [hm] "=&v"(hmax)
        : [h0] "v"(ha.x), [h1] "v"(ha.y), [h2] "v"(hb.x), [h3] "v"(hb.y), [h4] "v"(hc.x),
          [h5] "v"(hc.y), [h6] "v"(hd.x), [h7] "v"(hd.y));
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

template <bool FAST, bool CULL>
__device__ __forceinline__ void drain_list(const uint32_t* cq, uint32_t cnt,
                                           const float4* __restrict__ sph, uint32_t nsph, v3 o,
                                           v3 d, float a,
                                           float ya, float& best_t, int& best_i,
                                           const uint32_t* perm EXACT_ARGS) {
    const uint32_t lane = __lane_id();
    for (uint32_t k = 0; k < cnt; ++k) {
        const uint32_t e = cq[RT_IDX(k, RT_CQ_CAP, RT_SITE_CQ) * 64 + lane];
        uint32_t m = e & 0xFFu;
        const uint32_t base = (e >> 8) * RT_GROUP;
        while (m) {
            const uint32_t j = __builtin_ctz(m);
            m &= m - 1;
            exact_body<FAST, CULL>(sph[RT_IDX(base + j, nsph, RT_SITE_CQ_SPH)], (int)(base + j), o, d,
                                   a, ya, best_t, best_i,
                                   perm EXACT_PASS);
        }
    }
}

// Run the exact test for every queued candidate of this lane, in list order.
// Queue entries are (group << 8 | 8-bit candidate mask), one column per lane.
template <bool CULL>
__device__ __forceinline__ void drain_candidates(const uint32_t* cq, uint32_t cnt,
                                                 const float4* __restrict__ sph, uint32_t nsph,
                                                 v3 o, v3 d,
                                                 float a, bool fast, float& best_t,
                                                 int& best_i, const uint32_t* perm EXACT_ARGS) {
    if (fast)
        drain_list<true, CULL>(cq, cnt, sph, nsph, o, d, a, rt_recip_rn(a), best_t, best_i,
                               perm EXACT_PASS);
    else
        drain_list<false, CULL>(cq, cnt, sph, nsph, o, d, a, a, best_t, best_i, perm EXACT_PASS);
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
//
// CULL (rt_render_cull_kernel; the list permuted into spatial groups,
// clusters of 8 groups and supers of 8 clusters by rt_api.cpp build_cull):
// a super's 8 cluster BOUNDS, then a passing cluster's 8 group bounds --
// spheres (C_j, R_j) stored exactly like a group of spheres, S_j = R_j^2 -
// (1 - m - muB)|C_j|^2 -- go through the same packed filter against the
// threshold TB = (1 - m - muB)|o|^2, and only the groups some lane of the
// wave passes are filtered. Each bound dominates its members'
// filter values (proof in rt_api.cpp build_cull: R_j^2 = (1 + 2^-3) L^2 with
// L = max(|C_j - c_i| + r_i (1 + 2^-18)) over the members -- the spheres of the
// group, or of all 8 groups of the cluster -- and muB = 2^-7): a lane with a
// candidate in group j passes bound j and its cluster's bound, so a skipped
// group held no candidate of any lane
// and the candidate lists -- hence the hits -- are those of the full walk.
// The proof needs finite, moderate operands: a wave with a lane outside
// |o_i| <= 2^30, |d|^2 in [2^-100, 2^100] walks every group (bounds of groups
// with huge or non-finite members are "always pass" on the host side).
template <bool CULL>
__device__ __forceinline__ int intersect_world(const float4* __restrict__ grp,
                                               const float4* __restrict__ sph, uint32_t ngroups,
                                               uint32_t scene_fast, v3 o, v3 d, float& t_out,
                                               uint32_t* cq,
#ifdef RT_PROFILE
                                               Prof& prof_,
#endif
                                               const float4* bnd, const uint32_t* perm,
                                               uint32_t nclusters, bool use_supers = true) {
    const float l = sqrt_x(dot(d, d));
    const float a = l * l;  // sqr(length(r.dir)), intersect.wgsl:98
    const bool fast = ray_fast(scene_fast, o, a);
#if defined(RT_ASM_FILTER) && defined(__HIP_DEVICE_COMPILE__)
    const RayP RP = ray_pack(ray_filter_consts(o, d));
    const float RT_T = RP.T;
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
    const cfloat4* bp = (const cfloat4*)(uintptr_t)bnd;
#else
    const float4* gp = grp;  // host pass: never executed
    const float4* bp = bnd;
#endif
    // The filter of one group of 8 (pass 1 of the walk).
    auto group = [&](uint32_t g) __attribute__((always_inline)) {
        PROF_ADD(10, 1);  // groups filtered
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
                drain_candidates<CULL>(cq, cnt, sph, ngroups * RT_GROUP, o, d, a, fast, best_t, best_i,
                                       perm EXACT_PASS);
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
                cq[RT_IDX(cnt, RT_CQ_CAP, RT_SITE_CQ) * 64 + lane] = (g << 8) | m;
                ++cnt;
            }
        }
    };
    if constexpr (CULL) {
        const float oo = __builtin_fmaf(o.z, o.z, __builtin_fmaf(o.y, o.y, o.x * o.x));
        const float TB = (1.0f - 0x1p-16f - 0x1p-7f) * oo;  // bound threshold, muB = 2^-7
        const float om = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
        const bool cull_ok = (rt_ballot(!(om <= 0x1p30f)) | rt_ballot(!(a >= 0x1p-100f)) |
                              rt_ballot(!(a <= 0x1p100f))) == 0;
        // The wave's 8-bit mask of the bounds in one SoA record that some lane
        // passes (the record layout of a group: the same filter8).
        auto bound_mask = [&](const auto* p) __attribute__((always_inline)) -> uint32_t {
            const float4 X0 = p[0], X1 = p[1], Y0 = p[2], Y1 = p[3];
            const float4 Z0 = p[4], Z1 = p[5], S0 = p[6], S1 = p[7];
#if defined(RT_ASM_FILTER) && defined(__HIP_DEVICE_COMPILE__)
            f2 b01, b23, b45, b67;
            float bmax;
            filter8(RP, f2{X0.x, X0.y}, f2{X0.z, X0.w}, f2{X1.x, X1.y}, f2{X1.z, X1.w},
                    f2{Y0.x, Y0.y}, f2{Y0.z, Y0.w}, f2{Y1.x, Y1.y}, f2{Y1.z, Y1.w},
                    f2{Z0.x, Z0.y}, f2{Z0.z, Z0.w}, f2{Z1.x, Z1.y}, f2{Z1.z, Z1.w},
                    f2{S0.x, S0.y}, f2{S0.z, S0.w}, f2{S1.x, S1.y}, f2{S1.z, S1.w}, b01, b23,
                    b45, b67, bmax);
#else
            const f2 b01 = filter2(f2{X0.x, X0.y}, f2{Y0.x, Y0.y}, f2{Z0.x, Z0.y}, f2{S0.x, S0.y}, R);
            const f2 b23 = filter2(f2{X0.z, X0.w}, f2{Y0.z, Y0.w}, f2{Z0.z, Z0.w}, f2{S0.z, S0.w}, R);
            const f2 b45 = filter2(f2{X1.x, X1.y}, f2{Y1.x, Y1.y}, f2{Z1.x, Z1.y}, f2{S1.x, S1.y}, R);
            const f2 b67 = filter2(f2{X1.z, X1.w}, f2{Y1.z, Y1.w}, f2{Z1.z, Z1.w}, f2{S1.z, S1.w}, R);
            const float bmax = fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(fmaxf(b01.x, b01.y), b23.x),
                                                         b23.y), b45.x), b45.y), b67.x), b67.y);
#endif
            if (rt_ballot(bmax >= TB) == 0) return 0u;
            return (rt_ballot(b01.x >= TB) != 0 ? 0x01u : 0u) |
                   (rt_ballot(b01.y >= TB) != 0 ? 0x02u : 0u) |
                   (rt_ballot(b23.x >= TB) != 0 ? 0x04u : 0u) |
                   (rt_ballot(b23.y >= TB) != 0 ? 0x08u : 0u) |
                   (rt_ballot(b45.x >= TB) != 0 ? 0x10u : 0u) |
                   (rt_ballot(b45.y >= TB) != 0 ? 0x20u : 0u) |
                   (rt_ballot(b67.x >= TB) != 0 ? 0x40u : 0u) |
                   (rt_ballot(b67.y >= TB) != 0 ? 0x80u : 0u);
        };
        // three levels: supers of 8 clusters (bp: nsupers records of cluster
        // bounds, then nclusters records of group bounds), clusters of 8 groups;
        // the super level only pays with many clusters (host: use_supers)
        const uint32_t nsupers = (nclusters + 7u) >> 3;
        const auto* cp = bp + (size_t)nsupers * 8;
        for (uint32_t u = 0; u < nsupers; ++u) {
            const uint32_t valid = nclusters - u * 8u >= 8u ? 0xFFu : (1u << (nclusters - u * 8u)) - 1u;
            uint32_t cm = cull_ok && use_supers ? bound_mask(bp + (size_t)u * 8) : valid;
            while (cm) {
                const uint32_t k = u * 8u + __builtin_ctz(cm);
                cm &= cm - 1u;
                uint32_t gm = cull_ok ? bound_mask(cp + (size_t)k * 8) : 0xFFu;
                while (gm) {
                    const uint32_t j = __builtin_ctz(gm);
                    gm &= gm - 1u;
                    group(k * 8u + j);
                }
            }
        }
    } else {
        (void)bp;
        (void)nclusters;
        for (uint32_t g = 0; g < ngroups; ++g) group(g);
    }
    PROF_MARK(1);
#ifdef RT_PROFILE
    PROF_ADD(24, wave_max_u32(cnt));  // VALU walk: queue depth (wave max)
#ifdef RT_PROF_NESTED  // c[14]: the nested drain's wave iterations, sum_k max_lanes popcount(m_k)
    {
        const uint32_t kmax = wave_max_u32(cnt);
        for (uint32_t k = 0; k < kmax; ++k) {
            const uint32_t pc = k < cnt ? (uint32_t)__popc(cq[k * 64 + lane] & 0xFFu) : 0u;
            PROF_ADD(25, wave_max_u32(pc));
        }
    }
#endif
#endif
    drain_candidates<CULL>(cq, cnt, sph, ngroups * RT_GROUP, o, d, a, fast, best_t, best_i,
                           perm EXACT_PASS);
    PROF_MARK(2);
#ifdef RT_PROFILE
    PROF_ADD(13, wave_max_u32(ecnt[0]));
#if defined(RT_PROF_NESTED)
#elif defined(RT_PROF_SUMFULL)  // c[14]: lanes' full exact tests summed (not the wave max)
    {
        uint32_t sum1 = ecnt[1];
        for (int off = 32; off > 0; off >>= 1) sum1 += __shfl_xor(sum1, off);
        PROF_ADD(25, sum1);
    }
#else
    PROF_ADD(25, wave_max_u32(ecnt[1]));
#endif
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
// CULL: the permuted list; ties go to the smaller original index perm[i].
// x from lane (lane ^ off) -- ds_bpermute with the address computed here from
// a fresh lane id: HIP's __shfl_xor lets the compiler hoist every (lane ^ off)
// address of a loop into its own VGPR for the whole kernel (5 VGPRs for the
// reduction below, at the 80-register occupancy limit).
__device__ __forceinline__ uint32_t xor_shuffle(uint32_t x, uint32_t off) {
    uint32_t l = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    asm volatile("" : "+v"(l));
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((l ^ off) << 2), (int)x);
}

__device__ __forceinline__ float lane_value(float x, int src) {  // src wave-uniform
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), src));
}

template <bool CULL>
__device__ __forceinline__ void intersect_wide(const float4* __restrict__ sph, uint32_t n,
                                               uint32_t scene_fast, uint64_t active, v3 o, v3 d,
                                               int& hi, float& t, const uint32_t* perm) {
    const uint32_t lane = __lane_id();
    while (active) {
        const int src = (int)__builtin_ctzll(active);
        active &= active - 1;
        const v3 ro = mk(lane_value(o.x, src), lane_value(o.y, src), lane_value(o.z, src));
        const v3 rd = mk(lane_value(d.x, src), lane_value(d.y, src), lane_value(d.z, src));
        const float l = sqrt_x(dot(rd, rd));
        const float a = l * l;  // sqr(length(r.dir)), intersect.wgsl:98
        const bool fast = ray_fast(scene_fast, ro, a);
        const float ya = fast ? rt_recip_rn(a) : a;
        float bt = VERY_FAR;
        int bi = -1;
        for (uint32_t i = lane; i < n; i += 64) {
#ifdef RT_PROFILE
            uint32_t ecnt[2];
            exact_test<CULL>(sph[RT_IDX(i, n, RT_SITE_WIDE_SPH)], (int)i, ro, rd, a, ya, fast, bt, bi, perm,
                             ecnt);
#else
            exact_test<CULL>(sph[RT_IDX(i, n, RT_SITE_WIDE_SPH)], (int)i, ro, rd, a, ya, fast, bt, bi, perm);
#endif
        }
        for (int off = 32; off > 0; off >>= 1) {
            const float ot = __uint_as_float(xor_shuffle(__float_as_uint(bt), (uint32_t)off));
            const int oi = (int)xor_shuffle((uint32_t)bi, (uint32_t)off);
            bool take;
            if (CULL)  // key: original index, a miss (-1) last
                take = ot < bt || (ot == bt && (oi < 0 ? 0xFFFFFFFFu : perm[oi]) <
                                                   (bi < 0 ? 0xFFFFFFFFu : perm[bi]));
            else
                take = ot < bt || (ot == bt && (uint32_t)oi < (uint32_t)bi);
            if (take) {
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



#ifdef RT_MFMA_FILTER
// ---- the filter on the matrix cores (RT_MFMA_FILTER builds) ----
// The VALU filter's value H = hb^2 + S + o2.c (hb = k1 + e.c, e = -dn) is a
// quadratic form in the sphere centre, so with the ray's k1^2 moved into its
// threshold it is ONE dot product of a sphere row and a ray column:
//   H - k1^2 = H0 = S' + L.c + sum_ab Q_ab c_a c_b,
//   L_a = 2 k1 e_a + o2_a,  Q_aa = e_a^2,  Q_ab = 2 e_a e_b (a < b),
// candidate iff H0 >= T0 = (1 - m - mu')|o|^2 - k1^2 - abs'. The threshold is
// one more term of the same dot product: the MFMAs give V = T0 - H0 straight
// (the ray column holds the NEGATED features, -1 against S', and T0's own
// hi/lo parts against two exact 1s in the sphere row), and a sphere is a
// candidate iff V < 0. Each of the 10 features and T0 is split into f16
// hi/lo parts (x = hi + lo + err): 3 products (hi.hi + hi.lo + lo.hi) per
// feature, 2 for S' and 2 for T0 against exact 1s -- 31 of K = 32 (rt_api.cpp
// build_mfma: the A rows and their layout). Per 32-sphere block b and 32-ray
// half t of the wave, two chained v_mfma_f32_32x32x16_f16 give V for the
// 32 x 32 (sphere, ray) pairs straight into VGPRs; the VALU only ORs them
// (a tile or group with a candidate has a value with the sign bit set) and
// compares. Output layout (MI355X guide): lane l holds column (ray) l & 31 of
// the half, rows (spheres) (i & 3) + 8 (i >> 2) + 4 (l >> 5) in register i:
// four whole groups of 4 spheres per lane. A lane queues (group index, 4
// candidate flags) per half (RT_MF_FLAGS); the ray's lane drains the entries of its
// column's two lanes, in any order, with the (t, index) tie-break (exact_body
// LEX).
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16x __attribute__((ext_vector_type(16)));
// Margins. Split: |x - hi - lo| <= 2^-22|x| + 2^-25 (lo may be subnormal), so
// a feature product is within 3 * 2^-22|a||b| + 2^-25(|a| + |b|) of a b, and
// sum_f |a_f||b_f| <= 4|o||c| + |c|^2 + |S'| (|L| <= 4|o|, sum |Q c c| =
// (sum |e_a c_a|)^2 <= |c|^2): <= 2^-18.8 (|o|^2 + |c|^2) + 2^-20.4 |S'|; T0's
// split adds <= 2^-22 |o|^2 + 2^-25 (|T0| <= |o|^2). The f32 sums of the 31
// exact products (two chained MFMAs, 33 roundings at most, each <= 2^-24 of
// sum |p| <= 4.1 (|o|^2 + |c|^2) + |S'|) add <= 2^-16.9 (|o|^2 + |c|^2) +
// 2^-19 |S'| (measured: <= 4.9 * 2^-24 sum |p|, profiles/r02_mfma_acc.log).
// ASSUMPTION: that rounding model of the MFMA's f32 accumulation -- at most
// one rounding per added term -- is measured (tools/ubench/mfma_acc.hip), not
// a documented property of the hardware; DESIGN.md 4.2 states it and its
// evidence.
// The ray features' own roundings (one fma for L, two products for Q, the
// fma of T0) add <= 2^-21 (|o|^2 + |c|^2), and the ray constants dn, k1, o2
// are the VALU filter's (<= 25 * 2^-24 (|o|^2 + |c|^2), ray_filter_consts).
// Total <= 2^-16.02 (|o|^2 + |c|^2) < mu' = 2^-16 in |o|^2 + |c|^2, so a
// sphere the exact test can hit has V <= -(slack) < 0 (never a signed zero);
// the |S'| <= r^2 + |c|^2 part goes to the m margin's slack (2^-16 - 35 *
// 2^-24) and mu'; the absolute parts, 2^-25 x (the ray features scaled by
// 2^sq <= 2^(sq+1), the linear ones <= 4|o|, T0's lo), to abs' = 2^(sq - 20)
// (rt_api.cpp: mf_abs). Range: |c_i| <= 2^12, |S'| <= 2^15 (build_mfma) and
// per wave |o_i| <= 2^12, |o|^2 <= 2^15 (mfma_wave_ok: T0 in f16 range).
// tests/test_mfma_filter.py restates this arithmetic and checks it.
//
// Block bounds (mf.B). The list is walked in the culled list's spatial order
// (rt_api.cpp build_mfma), and each 16-sphere half of a 32-sphere block has a
// bounding sphere (a block is walked when either half's passes) (C,
// L = max_i (|C - c_i| + r_i (1 + 2^-18)), R^2 = (1 + 2^-5 + 2^-10) L^2 + 2^-60,
// 1 + 2^-4 through round 5) whose
// bound row is a sphere row with S'_B = R^2 - (1 - m - mu' - muB)|C|^2 (rounded
// up; muB = 2^-12 since round 6, 2^-8 before) and K 31 = 1, tested against the
// walk's own ray column, whose K 31 holds -RN_f16(muB |o|^2) (0 in sphere
// rows): T0_B = T0 - RN_f16(muB |o|^2) = (1 - m - mu' - muB')|o|^2 - k1^2 -
// abs' with muB' within 2^-11 muB of muB (a subnormal f16 errs by <= 2^-25
// absolute, inside abs'). A half-wave skips a block whose bounds no ray of the
// half passes (V_B >= 0 in every lane).
// Why a skipped block holds no hit -- straight from the exact test's f32
// arithmetic (exact_core; u = 2^-24, no FMA, correctly rounded sqrt): member
// i (centre c, w = its f32 r^2) is hit only if the computed dis >= 0. With
// v = fl(o - c) (|v - (o - c)| <= u|o - c|), hb = fl(dot(v, d)) (|hb - v.d| <=
// 3.0001u|v||d|), fl(lo * lo) = |v|^2 (1 + rho) (|rho| <= 6.001u: dot,
// sqrt, square), c~ = |v|^2 - w + e_c (|e_c| <= 7.002u|v|^2 + u w), a = |d|^2
// (1 + eps_a) (|eps_a| <= 6.001u) and the two products and the difference each
// rounded once, dis~ >= 0 means fl(hb^2) >= fl(a c~) (a nonzero difference of
// two f32 never rounds to 0), i.e. (v.d)^2 + 7.001u|v|^2|d|^2 >= |d|^2 (|v|^2 -
// w - 14.005u|v|^2 - 8.003u w), so the line's distance from the point o - v is
// dist_v^2 = |v|^2 - (v.d)^2/|d|^2 <= w (1 + 2^-21) + 2^-19.61 |v|^2, and
// from the centre (1-Lipschitz in the point) dist_i <= sqrt(w)(1 + 2^-22) +
// 2^-9.79 |o - c_i|. (In the walk's domain -- |o_i|, |c_i| <= 2^12, |d|^2 in
// [2^-100, 2^100] -- nothing overflows; subnormal products add <= 2^-148
// absolute to dis, <= 2^-48 to dist^2, inside abs'.) Round 5 reached the same
// step through the packed VALU filter's margins (dist_i^2 <= r_i^2 + 2^-14.3
// (|o|^2 + |c_i|^2)), 24x looser, hence its muB = 2^-8.
// The line distance is 1-Lipschitz again: dist_C <= L + s, s = 2^-9.79 |o -
// c_i| (L >= |C - c_i| + r_i (1 + 2^-18)), and with 2ab <= a^2/32 + 32 b^2,
// s^2 <= 2^-19.58 (2|o|^2 + 2|c_i|^2) and |c_i|^2 <= 2|C|^2 + 2L^2:
//   dist_C^2 <= (1 + 2^-5) L^2 + 33 s^2
//            <= (1 + 2^-5 + 2^-12.54) L^2 + 2^-12.54 (|o|^2 + |C|^2).
// The bound row's exact value is F_B = hb~_C^2 + R^2 - (1 - m)|o - C|^2 +
// (mu' + muB')(|o|^2 + |C|^2) + abs' >= R^2 - dist_C^2 + (mu' + muB' - 2^-18)
// (|o|^2 + |C|^2) (hb~ with the computed unit direction, |eta| <= 2^-21) >=
// (2^-10 - 2^-12.54) L^2 + 2^-60 + (mu' + 2^-12 (1 - 2^-11) - 2^-12.54 -
// 2^-18)(|o|^2 + |C|^2), which exceeds the tile's rounding (<= 2^-16.02
// (|o|^2 + |C|^2) + 2^-20.4 |S'_B|, |S'_B| <= R^2 + |C|^2, the analysis
// above; (2^-10 - 2^-12.54) L^2 covers 2^-20.4 R^2; mu' = 2^-16 covers the
// 2^-16.02, and 2^-12 (1 - 2^-11) - 2^-12.54 -
// 2^-18 - 2^-20.4 > 2^-13.9; |C_i| <= 2^12 as the members', |S'_B| <= 2^15 or
// the bound row always passes): V_B = T0_B - H0_B < 0. The proof's domain:
// |o_i| <= 2^12 (mfma_wave_ok) and |d|^2 in [2^-100, 2^100] for every live
// lane, else the wave walks every block. Bound rows of blocks with an
// out-of-range bound always pass (S'_B hi = +inf), of empty blocks never
// (-inf). Chunk-level rows ("Chunk bounds" below, L ~ 15-35 for the
// 10,000-sphere field, where the (1 + t) L^2 term dominates) split the slack
// the other way: t = 2^-7, so 129 s^2 <= 2^-10.57 (|o|^2 + |C|^2 + L^2),
// R^2 = (1 + 2^-7 + 2^-9) L^2 and K 31 = 4 (4 muB = 2^-10 > 2^-10.57 +
// 2^-18 + 2^-20.4; S'_B with 1 - m - mu' - 4 muB). tests/test_mfma_filter.py
// checks both numerically (exact hits of the
// adversarial ray sets never in a skipped block, five summation orders).
//
// Forward bounds. A bound is also skipped for a ray when it lies wholly behind
// the ray's origin. Any hit of a member sphere i (root >= EPSILON > 0) has
// half_b < 0 or |o - c_i|^2 < r_i^2 (1 + 2^-20) in f32 (else exact_core's
// certain-miss shortcut holds), so in exact arithmetic dn.(c_i - o) >=
// -r_i (1 + 2^-20) - 2^-20 (|o| + |c_i|), and dn.(C - o) >= -L - 2^-20 (|o| +
// |C| + L). The forward row (rt_api.cpp build_mfma; one
// v_mfma_f32_32x32x8_f16 per half) computes U = dn_hi.C_hi + c0_hi + L'_hi,
// c0 = fma(2^-9, |o|_1, -k1) (k1 = dn.o), L' = (1 + 2^-12) L + 2^-8 |C|_1 +
// 2^-14 rounded UP to f16 (+inf, always passing, where the line row does or
// beyond 2^15). The f16 parts cost <= 2^-9.9 |C|_1 (dn_hi C_hi) and
// 2^-10.9 |o|_1 (c0_hi, |c0| <= |o|_1), v_rsq and the f32 sums <= 2^-20
// (|C|_1 + |o|_1 + L'), all inside the 2^-12 L + 2^-8 |C|_1 + 2^-9 |o|_1 +
// 2^-14 slack (round 6; through round 5 2^-3 L + 2^-7 (|C|_1 + |o|_1) + 2^-14,
// the L term pure slack: the hit condition needs L (1 + 2^-20)): a hit's bound
// has U > 0, and the tile passes a (ray, bound) pair iff V_B < 0 and U >= +0
// (tile_or_fwd; tests/test_mfma_filter.py test_forward_bounds_are_conservative
// checks it numerically in five summation orders).
#define RT_MF_MU 0x1p-16f
#define RT_MF_MUB 0x1p-12f  // the block-bound tile's extra margin (see "Block bounds")
#ifndef RT_MF_CAP
#define RT_MF_CAP 12  // queue entries per lane and half (LDS)
#endif
#ifndef RT_MF_CAP_LDS
// ... in the kernel that also holds the walk's records in LDS (SPH_LDS:
// 9 entries, so that 4 workgroups of 256 threads still fit a CU's 160 KB)
#define RT_MF_CAP_LDS 9
#endif
// LDS words per wave of the matrix-core walk: the two halves' queues
#define RT_MF_QW (2u * RT_MF_CAP * 64u)

// Queue entry of a group of 4 spheres: its candidate flags in bits 7, 15, 23,
// 31 (sphere 4g + 0..3; v_perm_b32 sign-replicated bytes, mf_flags) and its
// group index g' = 8b + 2q (block b, group q; the half h is the queuing
// lane's, known to the drain) in the other bits, 7 per byte (mf_spread):
// g' < 2^14, so the matrix-core walk takes lists of up to 2^16 spheres
// (rt_api.cpp build_mfma; larger lists use the VALU filter).
#define RT_MF_FLAGS 0x80808080u
__host__ __device__ __forceinline__ uint32_t mf_spread(uint32_t g) {
    return (g & 0x7Fu) | ((g & 0x3F80u) << 1);
}
__device__ __forceinline__ uint32_t mf_unspread(uint32_t e) {
    return (e & 0x7Fu) | ((e >> 1) & 0x3F80u);
}
// the candidate flags of a group's four values V: bytes 0..3 = 0xFF when
// V[4q + byte] has its sign bit set (v_perm_b32 selectors 9 / 11 replicate
// bit 31 of the low / high source), two perms and an OR
__device__ __forceinline__ uint32_t mf_flags(float v0, float v1, float v2, float v3) {
    const uint32_t lo = __builtin_amdgcn_perm(__float_as_uint(v1), __float_as_uint(v0), 0x0C0C0B09u);
    const uint32_t hi = __builtin_amdgcn_perm(__float_as_uint(v3), __float_as_uint(v2), 0x0B090C0Cu);
    return lo | hi;
}

// The lane id (0..63) as a value the compiler cannot hoist or keep in a
// register across loops: an address built from it is recomputed at its use.
__device__ __forceinline__ uint32_t opaque_lane() {
    uint32_t l = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    asm volatile("" : "+v"(l));
    return l;
}

__device__ __forceinline__ uint32_t bperm(uint32_t src_lane, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

// the wave may use the f16 filter: every live lane's |o| within the split's range
// (and |o|^2 <= 2^15, so the threshold T0 <= |o|^2 splits into f16 parts)
__device__ __forceinline__ bool mfma_wave_ok(v3 o, bool live) {
    const float om = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float oo = __builtin_fmaf(o.z, o.z, __builtin_fmaf(o.y, o.y, o.x * o.x));
    return rt_ballot(live && !(om <= 0x1p12f && oo <= 0x1p15f)) == 0;
}

#ifdef RT_PROFILE
#define MF_ECNT , uint32_t* ecnt_
#define MF_ECNT_PASS , ecnt_
#define MF_ECNT_INC
#else
#define MF_ECNT
#define MF_ECNT_PASS
#define MF_ECNT_INC
#endif
// SP: the drain's record array, global (const float4*) or the workgroup's
// LDS copy (lds_cfloat4*, rt_render_kernel).
typedef __attribute__((address_space(3))) const float4 lds_cfloat4;
__device__ __forceinline__ float4 rec_load(const float4* __restrict__ p, uint32_t i) { return p[i]; }
__device__ __forceinline__ float4 rec_load(lds_cfloat4* p, uint32_t i) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) const f4v lds_f4v;
    const f4v v = ((lds_f4v*)p)[i];  // one ds_read_b128
    return make_float4(v.x, v.y, v.z, v.w);
}
#ifdef RT_DRAIN_DUMP
// Diagnostic build only (-DRT_DRAIN_DUMP): every 61st drain of the launch
// (any wave), per lane (ray) its queued entries (low 16 bits) and candidate
// tests (high 16), RT_DRAIN_DUMP_MAX drains; read back with
// rt_debug_drain_dump() (tools/drain_dump.py: the drain's lane balance).
#define RT_DRAIN_DUMP_MAX 65536
__device__ uint32_t g_drain_dump[RT_DRAIN_DUMP_MAX * 64];
__device__ unsigned int g_drain_seq;
__device__ unsigned int g_drain_rec;
#endif
template <bool FAST, typename SP, uint32_t CAP = RT_MF_CAP>
__device__ __forceinline__ void mfma_drain(const uint32_t* cq, uint32_t cnt0, uint32_t cnt1,
                                           SP sph, uint32_t nsph,
                                           const uint32_t* __restrict__ perm, v3 o,
                                           v3 d, float a,
                                           float ya, float& best_t, int& best_i MF_ECNT) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const uint32_t lane = __lane_id();
    const uint32_t t = lane >> 5, j = lane & 31u;
    // the two lanes holding this ray's column: j (rows 4h, h = 0) and j + 32;
    // v_permlane32_swap(x, x) gives (lane < 32 ? x[l] : x[l - 32], lane < 32 ?
    // x[l + 32] : x[l]) (profiles/r02_permlane32_swap.log)
    const auto c0 = __builtin_amdgcn_permlane32_swap(cnt0, cnt0, false, false);
    const auto c1 = __builtin_amdgcn_permlane32_swap(cnt1, cnt1, false, false);
    const uint32_t na = t ? c1[0] : c0[0], nb = t ? c1[1] : c0[1];
    const uint32_t* q = cq + t * (CAP * 64u);
#ifdef RT_PROFILE
    uint32_t* const ecnt = ecnt_;  // [0] exact tests, [1] past the certain-miss shortcut (this lane)
#endif
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // One loop over the lane's (entry, bit) pairs of both columns, in any
    // order (the LEX tie-break makes the order free): the wave pays the max
    // over lanes of the lane's candidate count. Every queued entry has a bit
    // set, so each pass tests one candidate. The nested form (per column, per
    // entry, per bit) cost the wave 4.79 exact-test slots per iteration against
    // this loop's 4.01 (RT_PROFILE, 20-frame launch) and 2.2 % per launch
    // (profiles/r03/ab_drain/); loading the next candidate's record ahead of
    // the current test (123 VGPRs) cost 2.2 %.
    const uint32_t total = na + nb;
#ifdef RT_DRAIN_DUMP
    {
        uint32_t seq = 0;
        if (lane == 0) seq = atomicAdd(&g_drain_seq, 1u);
        seq = (uint32_t)__builtin_amdgcn_readfirstlane((int)seq);
        if (seq % 61u == 0u) {
            uint32_t rec = 0;
            if (lane == 0) rec = atomicAdd(&g_drain_rec, 1u);
            rec = (uint32_t)__builtin_amdgcn_readfirstlane((int)rec);
            if (rec < RT_DRAIN_DUMP_MAX) {
                uint32_t bits = 0;
                for (uint32_t k = 0; k < total; ++k) {
                    const bool s1 = k >= na;
                    bits += __popc(q[(s1 ? k - na : k) * 64u + (s1 ? j + 32u : j)] & RT_MF_FLAGS);
                }
                g_drain_dump[rec * 64u + lane] = total | (bits << 16);
            }
        }
    }
#endif
    uint32_t i = 0, m = 0, base = 0;
    while (m != 0 || i < total) {
        if (m == 0) {
            const bool s1 = i >= na;
            const uint32_t e =
                q[RT_IDX(s1 ? i - na : i, CAP, RT_SITE_MFQ_READ) * 64u + (s1 ? j + 32u : j)];
            m = e & RT_MF_FLAGS;
            // group index 8b + 2q (mf_unspread), + h: the column's lane
            // j (h = 0) or j + 32 (h = 1) queued it
            base = (mf_unspread(e) + (s1 ? 1u : 0u)) * 4u;
            ++i;
        }
        const uint32_t b = __builtin_ctz(m) >> 3;
        m &= m - 1;
        MF_ECNT_INC;
        // the walk's order is spatial: an exact tie goes to the lower
        // ORIGINAL index (perm, read on ties only)
        exact_body<FAST, true>(rec_load(sph, RT_IDX(base + b, nsph, RT_SITE_MF_SPH)), (int)(base + b), o,
                               d, a, ya, best_t, best_i, perm EXACT_PASS);
    }
}


// The ORs of a tile's 16 values V = T0 - H0 per group of 4 and over the tile
// (10 VALU: v_or3 / v_or). A group or tile with a candidate (V < 0) has the
// sign bit set in its OR. The per-value flags are sign bits too (mf_flags), so a
// -0 or a NaN with the sign bit set is queued as well: harmless, since a -0
// never comes from a sphere the exact test can hit (the margins leave V <=
// -slack) and a NaN only from a ray with a NaN/inf feature, whose exact tests
// never hit; rows past the last sphere (whole 32-sphere blocks) read pad
// records, r^2 = -inf, that always miss (rt_set_scene pads the list).
// Integer ORs of the bits in C++ (no canonicalisation as a float max would
// need), so hipcc itself places the wait states between the MFMA that writes
// V and the first VALU reading it (round 2 had this in inline asm opening
// with a hand-placed s_nop 11).
// The 3-input ORs are v_bitop3_b32 (function 0xFE): gfx950 dual-issues it
// like a 2-input v_or_b32 (0.58 quad-cycles per instruction at 4 waves per
// SIMD), where v_or3_b32 -- which hipcc picks for a | b | c -- holds the SIMD
// a full quad-cycle (tools/ubench/valu_forms, profiles/r04/valu_forms/).
__device__ __forceinline__ uint32_t or3_dual(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xFE);
}
// The bound tile's pass flag with the forward rows: the OR over the lane's 16
// (ray, bound) pairs of V & ~U -- the sign bit set iff some pair has V < 0
// (the line passes near) and U >= +0 (the bound is not behind the origin):
// 16 v_bitop3_b32 ((a & ~b) | c, function 0xBA; dual-issued) in four chains,
// then one 3-input OR and an OR.
__device__ __forceinline__ uint32_t tile_or_fwd(const f16x& V, const f16x& U) {
    uint32_t acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        acc[q] = __builtin_amdgcn_bitop3_b32(__float_as_uint(V[4 * q]), __float_as_uint(U[4 * q]), 0u, 0xBA);
#pragma unroll
        for (int i = 1; i < 4; ++i)
            acc[q] = __builtin_amdgcn_bitop3_b32(__float_as_uint(V[4 * q + i]), __float_as_uint(U[4 * q + i]),
                                                 acc[q], 0xBA);
    }
    return or3_dual(acc[0], acc[1], acc[2]) | acc[3];
}
__device__ __forceinline__ void tile_or(const f16x& H, int* gq, int& g) {
    uint32_t v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = __float_as_uint(H[i]);
#pragma unroll
    for (int q = 0; q < 4; ++q) gq[q] = (int)(or3_dual(v[4 * q], v[4 * q + 1], v[4 * q + 2]) | v[4 * q + 3]);
    g = (int)(or3_dual((uint32_t)gq[0], (uint32_t)gq[1], (uint32_t)gq[2]) | (uint32_t)gq[3]);
}

// Called by the whole wave (the MFMA operands span all 64 lanes): lanes
// without a ray (live false) trace a dummy ray whose threshold is +inf.
// mf_qs = 2^sq, mf_abs = abs' (build_mfma). COUNT (the batch query,
// rt_intersect_mfma_kernel; never the render): tile_cnt[0] += the (block,
// half) tiles the wave walks, tile_cnt[1] += the 2 nblk it would walk without
// block bounds (rt_debug_intersect_tiles).
// SPH_LDS (rt_render_kernel): the drain's exact tests read the records
// from the workgroup's LDS copy sph_lds (render_body copies mf.sph there when
// it fits) instead of global memory.
// MULTI: any list (the chunk loop over ceil(nblk / 16) bound chunks, with the
// chunk-level bounds when mf.top); false: lists of at most 16 blocks (512
// walk positions, e.g. RTIOW's 484 spheres) -- one bound chunk, no loop, no
// chunk-level code (rt_render_kernel; rt_render_multi_kernel takes the rest):
// the loop's code in the single-chunk kernel cost its walk 2.2 % (register
// allocation and placement, profiles/r05/bisect/).
template <bool COUNT = false, bool SPH_LDS = false, bool MULTI = true, uint32_t CAP = RT_MF_CAP,
          bool ORIG = true>
__device__ __forceinline__ int intersect_world_mfma(const MfScene& mf,
                                                    uint32_t scene_fast, v3 o, v3 d, bool live,
                                                    uint64_t live_mask, float& t_out,
                                                    uint32_t* cq
#ifdef RT_PROFILE
                                                    , Prof& prof_
#endif
                                                    , unsigned long long* tile_cnt = nullptr,
                                                    lds_cfloat4* sph_lds = nullptr) {
    const uint4* __restrict__ mfA = mf.A;
    const uint32_t nblk = mf.nblk;
    const float mf_qs = mf.qs, mf_abs = mf.abs;
    const float4* __restrict__ sph = mf.sph;
    (void)sph_lds;
    if (!live) {
        o = mk(0.0f, 0.0f, 0.0f);
        d = mk(0.0f, 0.0f, 1.0f);
    }
    // chunk 0's block-bound fragments, loaded first so that the ray features
    // cover their latency (from block 0's A fragments when there are no
    // bounds, entries [0, 64) of its RT_MF_BLK: the load stays unconditional,
    // so hipcc's vmcnt waits count exactly, and in range)
    // The lane offsets come from an opaque lane id at each use (opaque_lane):
    // hoisted, hipcc kept them as three 64-bit per-lane offsets live across
    // the whole kernel, and spilled them to scratch around the bound tiles.
    // With chunk-level bounds (mf.top) the first bound chunk tested is the
    // chunk-level one, after the ceil(nblk / 16) block-bound chunks.
    const bool has_b = mf.B != nullptr;
    // block-bound chunks: 16 blocks, 2 bounds each (one when !MULTI)
    const uint32_t nbchunk = MULTI ? (nblk + 15u) >> 4 : 1u;
    const uint4* pb0 = has_b ? mf.B + (MULTI && mf.top ? (size_t)nbchunk * RT_MF_BCHUNK : 0) : mfA;
    const uint32_t pb0_n = has_b ? RT_MF_BCHUNK : RT_MF_BLK;  // uint4 entries of chunk / block 0
    (void)pb0_n;  // (read by the checked build's RT_IDX only)
    uint4 bq0, bq1;
    uint2 bq2;
    {
        const uint32_t l = opaque_lane();
        bq0 = pb0[RT_IDX(l, pb0_n, RT_SITE_MF_BOUND)];
        bq1 = pb0[RT_IDX((has_b ? 64u : 0u) + l, pb0_n, RT_SITE_MF_BOUND)];
        bq2 = reinterpret_cast<const uint2*>(pb0)[RT_IDX((has_b ? 256u : 0u) + l, 2u * pb0_n,
                                                         RT_SITE_MF_BOUND)];
    }
    const float dd = dot(d, d);
    const float l = sqrt_x(dd);
    const float a = l * l;  // sqr(length(r.dir)), intersect.wgsl:98
    const bool fast = ray_fast(scene_fast, o, a);
    const float ya = fast ? rt_recip_rn(a) : a;
    const uint32_t lane = __lane_id();
    // ray constants (ray_filter_consts, with the wider mu'), then the features
    const float rs = __builtin_amdgcn_rsqf(dd);
    const float ex = -(d.x * rs), ey = -(d.y * rs), ez = -(d.z * rs);  // e = -dn
    const float m_ = 0x1p-16f;
    const float oo = __builtin_fmaf(o.z, o.z, __builtin_fmaf(o.y, o.y, o.x * o.x));
    const float k1 = __builtin_fmaf(-ez, o.z, __builtin_fmaf(-ey, o.y, -ex * o.x));
    const float two = 2.0f * (1.0f - m_);
    const float T = live ? __builtin_fmaf(-k1, k1, (1.0f - m_ - RT_MF_MU) * oo) - mf_abs : INFINITY;
    const float k2 = 2.0f * k1;
    float f[9];  // L_x, L_y, L_z, Q_xx, Q_yy, Q_zz, Q_xy, Q_xz, Q_yz
    f[0] = __builtin_fmaf(k2, ex, two * o.x);
    f[1] = __builtin_fmaf(k2, ey, two * o.y);
    f[2] = __builtin_fmaf(k2, ez, two * o.z);
    f[3] = (ex * ex) * mf_qs;
    f[4] = (ey * ey) * mf_qs;
    f[5] = (ez * ez) * mf_qs;
    f[6] = ((2.0f * ex) * ey) * mf_qs;
    f[7] = ((2.0f * ex) * ez) * mf_qs;
    f[8] = ((2.0f * ey) * ez) * mf_qs;
    // The ray column, 16 words of two f16 (K 2m, 2m+1 in word m), against the
    // sphere rows of rt_api.cpp build_mfma (x_f = -f[f], the NEGATED features;
    // y_f the sphere's; hi = RN_f16(x), lo = RN_f16(x - hi)):
    //   K group 0  w0..w3   (hi x0, hi x1) .. (hi x6, hi x7)  vs (hi y) pairs
    //              w4..w7   the same hi pairs                  vs (lo y) pairs
    //   K group 1  w8..w11  (lo x0, lo x1) .. (lo x6, lo x7)  vs (hi y) pairs
    //              w12      (hi x8, lo x8)                     vs (hi y8, hi y8)
    //              w13      (hi x8, T0 hi)                     vs (lo y8, 1)
    //              w14      (T0 lo, -1)                        vs (1, S' hi)
    //              w15      (-1, 0)                            vs (S' lo, 0)
    // -- per feature hi.hi + hi.lo + lo.hi, T0 against two exact 1s, -1 against
    // S': the dot product is T0 - H0. The hi / lo pairs come from packed
    // converts (v_cvt_pk_f16_f32, round to nearest even); x - hi is exact in
    // f32. A lane without a ray has T0 = +inf (hi +inf, lo 0): V = +inf,
    // never a candidate.
    typedef _Float16 h2v __attribute__((ext_vector_type(2)));
    auto pk = [](float lo_half, float hi_half) {
        const h2v v = {(_Float16)lo_half, (_Float16)hi_half};
        uint32_t u;
        __builtin_memcpy(&u, &v, 4);
        return u;
    };
    // the f32 value of one half of a packed word: v_cvt_f32_f16 (SDWA for the
    // upper half) of the word itself -- the empty asm keeps the compiler from
    // converting x a second time for it
    auto half_f32 = [](uint32_t u, int half) {
        const uint16_t b = half ? (uint16_t)(u >> 16) : (uint16_t)u;
        _Float16 x;
        __builtin_memcpy(&x, &b, 2);
        return (float)x;
    };
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float xa = -f[2 * q], xb = -f[2 * q + 1];
        uint32_t hi = pk(xa, xb);
        asm volatile("" : "+v"(hi));
        w[q] = w[4 + q] = hi;
        w[8 + q] = pk(xa - half_f32(hi, 0), xb - half_f32(hi, 1));
    }
    {
        const float x8 = -f[8];
        uint32_t h8t = pk(x8, T);  // (hi x8, T0 hi)
        asm volatile("" : "+v"(h8t));
        const float l8 = x8 - half_f32(h8t, 0);
        const float tl = live ? T - half_f32(h8t, 1) : 0.0f;
        w[12] = pk(x8, l8);
        w[13] = h8t;
        w[14] = pk(tl, -1.0f);
        // K 31: -RN_f16(muB |o|^2) against a bound row's 1 (T0_B's margin,
        // "Block bounds") and a sphere row's 0
        w[15] = pk(-1.0f, -(RT_MF_MUB * oo));
    }
    // B fragments of K group g (K 16g..16g+15), half t: lane l holds column
    // l & 31, k = 16g + 8 (l >> 5) .. + 8. v_permlane32_swap(lo, hi) swaps lo's
    // upper 32 lanes with hi's lower 32 (profiles/r02_permlane32_swap.log): from
    // each lane's own words 8g+q (K 16g + 2q ..) and 8g+4+q its first result is
    // half 0's fragment word q, its second half 1's.
    uint32_t b0[2][4], b1[2][4];  // [K group][word] of half 0 / half 1
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const auto r = __builtin_amdgcn_permlane32_swap(w[8 * g + q], w[8 * g + 4 + q], false, false);
            b0[g][q] = r[0];
            b1[g][q] = r[1];
        }
    auto as_h8 = [](const uint32_t* v) {
        const uint4 q = make_uint4(v[0], v[1], v[2], v[3]);
        h8v r;
        __builtin_memcpy(&r, &q, 16);
        return r;
    };
    const h8v B00 = as_h8(b0[0]), B01 = as_h8(b0[1]);  // half 0: K 0..15, K 16..31
    const h8v B10 = as_h8(b1[0]), B11 = as_h8(b1[1]);  // half 1
    const f16x zero = {};

    // ---- block bounds (mf.B): which 32-sphere blocks some ray of each half
    // passes near. The bound tile is the TRANSPOSED product -- the rays'
    // fragments as the A operand (rows), the chunk's 32 block bounds as B
    // (columns; their fragments have the sphere rows' layout, which is B's) --
    // so lane l holds bound l & 31 against 16 of the half's rays, and the
    // AND-NOT / OR tree of the line tile V_B and the forward tile U + one
    // ballot give the half's 32-bit bound mask. The ray column is the walk's
    // own (a bound row's K 31 = 1 picks up its -muB |o|^2: T0_B; "Block
    // bounds" and "Forward bounds" in the header above). A wave with a live
    // ray outside |d|^2 in [2^-100, 2^100] (the proof's domain) walks every
    // block.
    //
    // Chunk bounds (mf.top: 2..32 bound chunks, e.g. 10,000 spheres in 20):
    // row j of the chunk-level chunk is the bound of bound chunk j's 512 walk
    // positions, built like a block bound (C, L over its members, R^2 =
    // (1 + 2^-5 + 2^-10) L^2, muB, forward row), so the "Block bounds" / "Forward
    // bounds" proofs hold for it unchanged: a ray with an exact hit in chunk
    // j passes row j. Its tile (the same three MFMAs per half) runs first; a
    // half that no ray of passes chunk j gets no block of chunk j, and a chunk
    // neither half passes is not tested at all.
    const uint32_t nchunk = MULTI ? (nblk + 31u) >> 5 : 1u;  // of the walk: 32 blocks
    uint32_t mv0 = 0xFFFFFFFFu, mv1 = 0xFFFFFFFFu;  // lane k: walk chunk k's masks, halves 0 / 1
    if (has_b && rt_ballot(live && !(dd >= 0x1p-100f && dd <= 0x1p100f)) == 0) {
        mv0 = mv1 = 0u;
        // the forward column (rt_api.cpp build_mfma; "Forward bounds"), K 0..7
        // of v_mfma_f32_32x32x8_f16: dn = -e hi x3, c0 = fma(2^-9, |o|_1, -k1)
        // hi | 1, 0 x3 -- lanes 32..63 of a half's fragment hold the constant
        // K 4..7
        typedef _Float16 h4v __attribute__((ext_vector_type(4)));
        h4v G0, G1;
        {
            const float c0 = __builtin_fmaf(0x1p-9f, fabsf(o.x) + fabsf(o.y) + fabsf(o.z), -k1);
            const uint32_t u0 = pk(-ex, -ey), u1 = pk(-ez, c0);
            const uint32_t k4 = pk(1.0f, 0.0f), k6 = 0u;
            const auto r0 = __builtin_amdgcn_permlane32_swap(u0, k4, false, false);
            const auto r1 = __builtin_amdgcn_permlane32_swap(u1, k6, false, false);
            const uint2 g0 = make_uint2(r0[0], r1[0]), g1 = make_uint2(r0[1], r1[1]);
            __builtin_memcpy(&G0, &g0, 8);
            __builtin_memcpy(&G1, &g1, 8);
        }
        // one bound chunk's tiles: per half the 32-bit mask of its rows some
        // ray of the half passes
        // (hook: called once the tile's last MFMAs have been issued, so the
        // next chunk's rows can load into bq while this chunk's ORs run)
        auto bound_tiles = [&](uint32_t* mk2, auto&& hook) {
            h8v F0, F1;
            h4v F2;
            __builtin_memcpy(&F0, &bq0, 16);
            __builtin_memcpy(&F1, &bq1, 16);
            __builtin_memcpy(&F2, &bq2, 8);
#pragma unroll
            for (uint32_t t = 0; t < 2; ++t) {
                const f16x V = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                    t ? B11 : B01, F1, __builtin_amdgcn_mfma_f32_32x32x16_f16(t ? B10 : B00, F0, zero, 0, 0, 0),
                    0, 0, 0);
                const f16x U = __builtin_amdgcn_mfma_f32_32x32x8f16(t ? G1 : G0, F2, zero, 0, 0, 0);
                if (t == 1) hook();
                const uint32_t acc = tile_or_fwd(V, U);
                const uint64_t bm = rt_ballot((int)acc < 0);
                mk2[t] = (uint32_t)bm | (uint32_t)(bm >> 32);
            }
        };
        // bound rows 2i, 2i + 1 are block 16 k + i's halves: its bit is
        // their OR, the 16 block bits compressed from the even positions
        auto fold = [](uint32_t m) {
            m = (m | (m >> 1)) & 0x55555555u;
            m = (m | (m >> 1)) & 0x33333333u;
            m = (m | (m >> 2)) & 0x0F0F0F0Fu;
            m = (m | (m >> 4)) & 0x00FF00FFu;
            m = (m | (m >> 8)) & 0x0000FFFFu;
            return m;
        };
        if constexpr (!MULTI) {  // one bound chunk, preloaded: lane 0's masks
            uint32_t mk2[2];
            bound_tiles(mk2, [] {});
            if (lane == 0u) {
                mv0 = fold(mk2[0]);
                mv1 = fold(mk2[1]);
            }
            PROF_ADD(17, 1);
        } else {
        const bool top = mf.top != 0u;
        uint32_t top2[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};  // chunks some ray of each half passes near
        if (top) {
            bound_tiles(top2, [] {});  // the preloaded chunk-level fragments
            PROF_ADD(27, 1);    // chunk-level bound tiles (2 halves x 3 MFMAs)
        }
        // one bound chunk's rows into bq: the chunk's base an opaque SGPR
        // pair, so the loads take the scalar-base form with a 32-bit lane
        // offset, not three per-lane 64-bit pointers stepped through the loop
        auto chunk_load = [&](uint32_t k) {
            const uint4* pb = mf.B + (size_t)RT_IDX(k, nbchunk, RT_SITE_MF_BOUND) * RT_MF_BCHUNK;
#ifndef RT_CHUNK_LSR
            asm volatile("" : "+s"(pb));
            const uint32_t l = opaque_lane();
#else  // (A/B builds only: the loads as hipcc strength-reduces them)
            const uint32_t l = lane;
#endif
            bq0 = pb[l];
            bq1 = pb[64u + l];
            bq2 = reinterpret_cast<const uint2*>(pb)[256u + l];
        };
        // The bound chunks to test, in order: with chunk bounds those some
        // half passes near (at most 32 chunks), else all (chunk 0 preloaded).
        // Software-pipelined: the next chunk's rows load into bq as soon as
        // the current chunk's last MFMAs have read them (bound_tiles' hook;
        // no extra registers, so no spills), and the L2 round trip overlaps
        // this chunk's ORs, ballots and folds; the last chunk reloads itself
        // (an L1 hit), so every load stays unconditional and hipcc's vmcnt
        // waits count exactly.
        uint32_t cm = top ? (top2[0] | top2[1]) : 0u;  // (top) chunks not yet taken
        uint32_t k = 0;
        bool any = nbchunk != 0u;
        if (top) {
            any = cm != 0u;
            k = any ? (uint32_t)__builtin_ctz(cm) : 0u;
            cm &= cm - 1u;
            if (any) chunk_load(k);
        }
        while (any) {
            bool more;
            uint32_t kn;
            if (top) {
                more = cm != 0u;
                kn = more ? (uint32_t)__builtin_ctz(cm) : k;
                cm &= cm - 1u;
            } else {
                more = k + 1u < nbchunk;
                kn = more ? k + 1u : k;
            }
            uint32_t mk2[2];
            bound_tiles(mk2, [&] { chunk_load(kn); });
            if (top) {  // a half that passes no ray near the chunk gets none of its blocks
                mk2[0] = ((top2[0] >> k) & 1u) ? mk2[0] : 0u;
                mk2[1] = ((top2[1] >> k) & 1u) ? mk2[1] : 0u;
            }
            const uint32_t sh = (k & 1u) * 16u;
            const uint32_t f0 = fold(mk2[0]) << sh, f1 = fold(mk2[1]) << sh;
            if (lane == (k >> 1)) {
                mv0 |= f0;
                mv1 |= f1;
            }
            PROF_ADD(17, 1);  // bound chunks: 2 halves x (2 MFMA 32x32x16 + 1 MFMA 32x32x8)
            k = kn;
            any = more;
        }
        }  // MULTI
    }
    PROF_MARK(16);  // ray column + bound tiles

    float best_t = VERY_FAR;
    int best_i = -1;
    // each lane's next queue slot per half (LDS word pointers, never below the
    // queue: a DS address past the LDS window drops the write): an append is
    // one store and one add; the counts are derived when needed
    uint32_t* const q0 = cq + lane;
    uint32_t* const q1 = cq + CAP * 64u + lane;
    uint32_t *qp0 = q0, *qp1 = q1;
    auto qcount = [](const uint32_t* p, const uint32_t* p0) { return (uint32_t)(p - p0) >> 6; };
#ifdef RT_PROFILE
    // this lane's exact tests (c[13]: wave max, c[15]: lane sum) and those
    // past the certain-miss shortcut (c[21]: lane sum)
    uint32_t ecnt_[2] = {0, 0};
#endif
    // wave-uniform upper bounds of every lane's queue length per half (SGPRs):
    // one per group some lane queued from since the last drain
    uint32_t ub0 = 0, ub1 = 0;
    // the exact tests of the queued candidates (the records from global
    // memory, or from the workgroup's LDS copy: SPH_LDS)
    auto drain = [&](uint32_t cnt0, uint32_t cnt1) {
        if constexpr (SPH_LDS) {
            if (__builtin_expect(fast, 1))
                mfma_drain<true, lds_cfloat4*, CAP>(cq, cnt0, cnt1, sph_lds, nblk * 32u, mf.perm, o, d, a, ya, best_t,
                                 best_i MF_ECNT_PASS);
            else
                mfma_drain<false, lds_cfloat4*, CAP>(cq, cnt0, cnt1, sph_lds, nblk * 32u, mf.perm, o, d, a, ya, best_t,
                                  best_i MF_ECNT_PASS);
        } else {
            if (__builtin_expect(fast, 1))  // (the IEEE drain is placed out of the way)
                mfma_drain<true, const float4*, CAP>(cq, cnt0, cnt1, sph, nblk * 32u, mf.perm, o, d, a, ya, best_t,
                                 best_i MF_ECNT_PASS);
            else
                mfma_drain<false, const float4*, CAP>(cq, cnt0, cnt1, sph, nblk * 32u, mf.perm, o, d, a, ya, best_t,
                                  best_i MF_ECNT_PASS);
        }
    };
    // one 32-sphere block: both ray halves against A fragments x0 (K 0..15),
    // x1 (K 16..31)
    auto block = [&](uint32_t b, const uint4 x0, const uint4 x1, uint32_t m0, uint32_t m1) {
        // a block adds at most 4 entries to each half's queue: make room first,
        // while no tile result is live (the lanes' own counts are compared
        // only when the scalar bound says the queue may be full)
        if (__builtin_expect(max(ub0, ub1) + 4u > CAP &&
                             rt_ballot(max(qcount(qp0, q0), qcount(qp1, q1)) + 4u > CAP) != 0,
                             0)) {  // (rare: kept out of the walk's hot blocks)
            const uint32_t cnt0 = qcount(qp0, q0), cnt1 = qcount(qp1, q1);
            PROF_ADD(11, 1);  // queue flushes
            drain(cnt0, cnt1);
            qp0 = q0;
            qp1 = q1;
            ub0 = ub1 = 0;
        }
        h8v A0, A1;
        __builtin_memcpy(&A0, &x0, 16);
        __builtin_memcpy(&A1, &x1, 16);
        const uint32_t sb = mf_spread(b * 8u);  // the block's group entries (wave-uniform, SALU)
        // the appends of half t's tile H
        auto tile = [&](const f16x& H, uint32_t t) {
            // per-group ORs (the lane's 4 groups of 4 spheres), then the tile's
            int gq[4], g;
            tile_or(H, gq, g);
            if (rt_ballot(g < 0) != 0) {
                PROF_ADD(5, 1);  // tiles with a candidate
                uint32_t*& qp = t ? qp1 : qp0;
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    if (rt_ballot(gq[q] < 0) == 0) continue;  // no lane has one in this group
                    ++(t ? ub1 : ub0);
                    PROF_ADD(23, 1);  // group appends (wave-level)
                    const uint32_t m = mf_flags(H[4 * q], H[4 * q + 1], H[4 * q + 2], H[4 * q + 3]);
                    // Branch-free append: every lane writes its next slot
                    // (< CAP: the check above) and keeps it only with a
                    // flag set. A lane whose column has no live ray has no
                    // flags: its T0 = +inf makes every V = +inf (no -inf
                    // term: the pad rows' S' = -inf meets the ray's -1).
                    // b * 8 has its low 3 bits clear: spread(8b + 2q) = spread(8b) + 2q
                    const uint32_t f = m & RT_MF_FLAGS;
#ifdef RT_CHECK_BOUNDS
                    RT_IDX(qcount(qp, t ? q1 : q0), CAP, RT_SITE_MFQ);
                    // a column without a live ray (T0 = +inf) never queues:
                    // this lane holds column lane & 31 of half t, the ray of
                    // lane 32 t + (lane & 31)
                    RT_IDX(f != 0u ? 1u : 0u,
                           ((live_mask >> (32u * t + (lane & 31u))) & 1u) ? 2u : 1u,
                           RT_SITE_DEAD_QUEUE);
                    if (qcount(qp, t ? q1 : q0) >= CAP) qp = t ? q1 : q0;
#endif
                    // the group index as one opaque SGPR: v_or_b32 (dual-
                    // issued) rather than v_or3_b32 with an inline constant
                    uint32_t ge = sb + q * 2u;
                    asm volatile("" : "+s"(ge));
                    *qp = f | ge;
                    // one more entry iff a flag is set: min(f, 1) as one VALU
                    // min (the compiler otherwise emits a compare and a select)
                    uint32_t inc;
                    asm("v_min_u32 %0, 1, %1" : "=v"(inc) : "v"(f));
                    qp += 64u * inc;
                }
            }
        };
        auto mfma2 = [&](const h8v& Bk0, const h8v& Bk1) {
            return __builtin_amdgcn_mfma_f32_32x32x16_f16(
                A1, Bk1, __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, Bk0, zero, 0, 0, 0), 0, 0, 0);
        };
        const bool w0 = ((m0 >> (b & 31u)) & 1u) != 0u, w1 = ((m1 >> (b & 31u)) & 1u) != 0u;
        // the two halves unrolled (no per-tile operand selects) but kept apart
        // (sched_barrier): one tile's 16 result registers live at a time --
        // both halves' four MFMAs back to back (half 1's on the matrix pipe
        // while half 0's results are ORed) spilled 5 VGPRs and cost 5.3 %
        // (profiles/r05/walk_both/)
        if (w0) {
            PROF_ADD(10, 1);  // tiles walked
            tile(mfma2(B00, B01), 0u);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (w1) {
            PROF_ADD(10, 1);
            tile(mfma2(B10, B11), 1u);
        }
    };
    // The blocks some ray of the wave passes near (all blocks without bound
    // tiles), in pairs: the next block's fragments load while this one runs,
    // into the other register set (no fragment copies per block). Block p's
    // fragments at mfA + RT_MF_BLK p (uniform base): A0 (K 0..15) for the 64
    // lanes, then A1 (K 16..31) for lanes 32..63 only -- lanes 0..31 hold K
    // 16..23 of A1, the sphere's hi parts again (= their K 0..7 of A0), so
    // they load their A0 entry a second time (the same cache lines, no new
    // bytes): 1.5 KB per block instead of 2 (rt_api.cpp build_mfma).
    const uint32_t off1 = lane < 32u ? lane : lane + 32u;
    auto load = [&](uint32_t p, uint4& x0, uint4& x1) {
        const uint4* pa = mfA + (size_t)RT_IDX(p, nblk, RT_SITE_MFA) * RT_MF_BLK;
        x0 = pa[lane];
        x1 = pa[off1];
    };
    uint32_t walked = 0;  // COUNT: tiles walked by the wave
    for (uint32_t k = 0; k < nchunk; ++k) {
        const uint32_t m0 = (uint32_t)__builtin_amdgcn_readlane((int)mv0, (int)k);
        const uint32_t m1 = (uint32_t)__builtin_amdgcn_readlane((int)mv1, (int)k);
        const uint32_t rem = nblk - 32u * k;
        const uint32_t valid = rem >= 32u ? 0xFFFFFFFFu : ((1u << rem) - 1u);
        if (COUNT) walked += (uint32_t)(__popc(m0 & valid) + __popc(m1 & valid));
        uint32_t todo = (m0 | m1) & valid;
        if (todo == 0u) continue;
        // the next block to walk (the last one again when none is left: its
        // fragments reload from L1, and every load stays unconditional, so
        // hipcc's vmcnt waits count exactly -- a conditional prefetch made it
        // wait for the prefetch too)
        auto next = [&](uint32_t cur) {
            const uint32_t nb = todo != 0u ? 32u * k + (uint32_t)__builtin_ctz(todo) : cur;
            todo &= todo - 1u;
            return nb;
        };
        uint32_t b = next(0u);
        uint4 a0, a1, n0, n1;
        load(b, a0, a1);
        for (;;) {
            const bool more = todo != 0u;
            const uint32_t bn = next(b);
            load(bn, n0, n1);
            block(b, a0, a1, m0, m1);
            if (!more) break;
            const bool more2 = todo != 0u;
            b = next(bn);
            load(b, a0, a1);
            block(bn, n0, n1, m0, m1);
            if (!more2) break;
        }
    }
    if (COUNT && __lane_id() == 0) {
        atomicAdd(tile_cnt, (unsigned long long)walked);
        atomicAdd(tile_cnt + 1, 2ull * nblk);
    }
    PROF_MARK(1);
    drain(qcount(qp0, q0), qcount(qp1, q1));
    // the walk position of the winner -> its original index (ORIG; the render
    // shades by walk position: the records in the walk's order, MfScene)
    if (ORIG && best_i >= 0) best_i = (int)mf.perm[RT_IDX((uint32_t)best_i, nblk * 32u, RT_SITE_PERM)];
    PROF_MARK(2);
#ifdef RT_PROFILE
    {   // (diagnostic reductions: their time goes to c[26])
        PROF_ADD(13, wave_max_u32(ecnt_[0]));
        uint32_t sum1 = ecnt_[1];
        for (int off = 32; off > 0; off >>= 1) sum1 += __shfl_xor(sum1, off);
        PROF_ADD(21, sum1);
        uint32_t sum0 = ecnt_[0];
        for (int off = 32; off > 0; off >>= 1) sum0 += __shfl_xor(sum0, off);
        PROF_ADD(15, sum0);
        PROF_MARK(26);
    }
#endif
    t_out = best_t;
    return best_i;
}
#endif  // RT_MFMA_FILTER

}  // namespace
