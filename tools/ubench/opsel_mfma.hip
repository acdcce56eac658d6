// Isolates the round-2 finding: v_pk_fma_f32 with
// op_sel / op_sel_hi half-broadcasts of VGPR pairs gave wrong results in
// VALU-walk waves of rt_intersect_mfma_kernel while other waves of the kernel
// ran MFMAs, and never without them (tools/isect_diag.py,
// profiles/r03_isect_diag.log).
//
// Each 256-thread workgroup holds 4 waves. Odd waves run the filter group of
// round 2 (rt_dev_intersect.h filter8) twice per iteration on the same
// operands: once in the op_sel-broadcast form (4 VGPR pairs, halves selected
// per operand) and once in the duplicated-pair form (7 pairs) -- the same
// FMAs on the same values, so the two must agree bit for bit -- and count the
// lanes where they differ. Even waves either run chains of
// v_mfma_f32_32x32x16_f16 (mode "mfma") or sleep (mode "idle"). A third mode
// runs both filter forms in every wave and no MFMA at all ("valu").
//
//   hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -o opsel_mfma opsel_mfma.hip && ./opsel_mfma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16x __attribute__((ext_vector_type(16)));
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(4))) const float4 cfloat4;  // scalar-cache reads
#else
typedef const float4 cfloat4;  // host pass: never executed
#endif

#define ITERS 2048

// op_sel form: r0 = (-dnx, -dny), r1 = (-dnz, k1), r2 = (o2x, o2y), r3 = (o2z, T)
__device__ __forceinline__ void grp_opsel(f2 r0, f2 r1, f2 r2, f2 r3, f2 cxa, f2 cxb, f2 cxc,
                                          f2 cxd, f2 cya, f2 cyb, f2 cyc, f2 cyd, f2 cza, f2 czb,
                                          f2 czc, f2 czd, f2 sa, f2 sb, f2 sc, f2 sd, f2& ha,
                                          f2& hb, f2& hc, f2& hd) {
    asm volatile(
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
        "s_nop 0"
        : [ha] "=&v"(ha), [hb] "=&v"(hb), [hc] "=&v"(hc), [hd] "=&v"(hd)
        : [r0] "v"(r0), [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [cxa] "s"(cxa), [cxb] "s"(cxb),
          [cxc] "s"(cxc), [cxd] "s"(cxd), [cya] "s"(cya), [cyb] "s"(cyb), [cyc] "s"(cyc),
          [cyd] "s"(cyd), [cza] "s"(cza), [czb] "s"(czb), [czc] "s"(czc), [czd] "s"(czd),
          [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc), [sd] "s"(sd));
}

// duplicated-pair form (the shipped filter8's instruction stream)
__device__ __forceinline__ void grp_dup(f2 dx, f2 dy, f2 dz, f2 k1, f2 ox, f2 oy, f2 oz, f2 cxa,
                                        f2 cxb, f2 cxc, f2 cxd, f2 cya, f2 cyb, f2 cyc, f2 cyd,
                                        f2 cza, f2 czb, f2 czc, f2 czd, f2 sa, f2 sb, f2 sc,
                                        f2 sd, f2& ha, f2& hb, f2& hc, f2& hd) {
    asm volatile(
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
        "v_pk_fma_f32 %[hd], %[ox], %[cxd], %[hd]\n\t"
        "s_nop 0"
        : [ha] "=&v"(ha), [hb] "=&v"(hb), [hc] "=&v"(hc), [hd] "=&v"(hd)
        : [dx] "v"(dx), [dy] "v"(dy), [dz] "v"(dz), [k1] "v"(k1), [ox] "v"(ox), [oy] "v"(oy),
          [oz] "v"(oz), [cxa] "s"(cxa), [cxb] "s"(cxb), [cxc] "s"(cxc), [cxd] "s"(cxd),
          [cya] "s"(cya), [cyb] "s"(cyb), [cyc] "s"(cyc), [cyd] "s"(cyd), [cza] "s"(cza),
          [czb] "s"(czb), [czc] "s"(czc), [czd] "s"(czd), [sa] "s"(sa), [sb] "s"(sb),
          [sc] "s"(sc), [sd] "s"(sd));
}

// scalar reference: filter2's op order with one v_fma_f32 per step (compiled
// with -fno-slp-vectorize: no packed ops), for sphere pair (cx, cy, cz, S)
__device__ __forceinline__ f2 grp_scalar2(float ex, float ey, float ez, float k1, float ox,
                                          float oy, float oz, f2 cx, f2 cy, f2 cz, f2 S) {
    f2 h;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const float hb = __builtin_fmaf(ez, cz[e], __builtin_fmaf(ey, cy[e], __builtin_fmaf(ex, cx[e], k1)));
        h[e] = __builtin_fmaf(ox, cx[e], __builtin_fmaf(oy, cy[e], __builtin_fmaf(oz, cz[e],
                              __builtin_fmaf(hb, hb, S[e]))));
    }
    return h;
}

__device__ __forceinline__ unsigned neq(f2 a, f2 b) {
    return (__float_as_uint(a.x) != __float_as_uint(b.x)) + (__float_as_uint(a.y) != __float_as_uint(b.y));
}

// mode 0: even waves MFMA, odd waves both filter forms; 1: even waves idle;
// 2: every wave both filter forms, no MFMA; 3: even waves v_permlane32_swap
// chains; 4: even waves LDS queue traffic (ds_write / ds_read of other lanes'
// words); 5: even waves the matrix-core walk's mix -- MFMA tiles, ORs of the
// results, permlane swaps and LDS queue writes/reads (rt_dev_intersect.h)
__global__ __launch_bounds__(256) void k_opsel(const float4* grp, uint32_t ngroups,
                                               const float* rays, int mode,
                                               unsigned* __restrict__ bad,
                                               unsigned* __restrict__ bad_opsel,
                                               unsigned* __restrict__ bad_dup,
                                               float* __restrict__ sink) {
    __shared__ uint32_t q[4 * 64 * 8];
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    const bool filt = mode == 2 || (wave & 1);
    if (!filt) {
        if (mode == 1) {
            for (int i = 0; i < ITERS / 8; ++i) __builtin_amdgcn_s_sleep(8);
            return;
        }
        uint32_t* wq = q + wave * 64 * 8;
        if (mode == 3) {
            uint32_t x = gid, y = gid * 7u;
            for (int i = 0; i < ITERS * 16; ++i) {
                const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
                x = r[0] + 1u;
                y = r[1] ^ 3u;
            }
            sink[gid] = (float)(x ^ y);
            return;
        }
        if (mode == 4) {
            uint32_t acc = 0;
            for (int i = 0; i < ITERS * 4; ++i) {
                wq[(i & 7) * 64 + lane] = acc + (uint32_t)i;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                acc += wq[(i & 7) * 64 + (lane ^ 32u)];
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            sink[gid] = (float)acc;
            return;
        }
        h8v a, b;
        for (int k = 0; k < 8; ++k) {
            a[k] = (_Float16)(0.001f * (float)((threadIdx.x + k) & 15) - 0.004f);
            b[k] = (_Float16)(0.002f * (float)((threadIdx.x * 3 + k) & 15) - 0.01f);
        }
        f16x acc = {};
        uint32_t cnt = 0, sw = gid;
        for (int i = 0; i < ITERS * 4; ++i) {
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, mode == 5 ? f16x{} : acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(b, a, acc, 0, 0, 0);
            if (mode == 5) {
                int o = 0;
                for (int k = 0; k < 16; ++k) o |= __float_as_int(acc[k]);
                if (__builtin_amdgcn_ballot_w64(o < 0) != 0) {
                    wq[(cnt & 7) * 64 + lane] = (uint32_t)o;
                    ++cnt;
                }
                const auto r = __builtin_amdgcn_permlane32_swap(sw, cnt, false, false);
                sw = r[0] + r[1];
                if ((i & 15) == 15) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    sw += wq[(cnt & 7) * 64 + (lane ^ 32u)];
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
            }
        }
        float s = (float)sw;
        for (int k = 0; k < 16; ++k) s += acc[k];
        sink[gid] = s;
        return;
    }
    const float* r = rays + (size_t)gid * 8;
    const float ex = r[0], ey = r[1], ez = r[2], k1 = r[3], ox = r[4], oy = r[5], oz = r[6], T = r[7];
    const f2 r0 = {ex, ey}, r1 = {ez, k1}, r2 = {ox, oy}, r3 = {oz, T};
    const f2 dx = {ex, ex}, dy = {ey, ey}, dz = {ez, ez}, kk = {k1, k1}, oxx = {ox, ox},
             oyy = {oy, oy}, ozz = {oz, oz};
    const cfloat4* gp = (const cfloat4*)(uintptr_t)grp;
    unsigned nbad = 0, nbad_seen = 0, nb_op = 0, nb_dup = 0;
    float acc = 0.f;
    for (int it = 0; it < ITERS; ++it) {
        const uint32_t g = (uint32_t)it % ngroups;
        const auto* p = gp + (size_t)g * 8;
        const float4 X0 = p[0], X1 = p[1], Y0 = p[2], Y1 = p[3];
        const float4 Z0 = p[4], Z1 = p[5], S0 = p[6], S1 = p[7];
        f2 a0, b0, c0, d0, a1, b1, c1, d1;
        grp_opsel(r0, r1, r2, r3, f2{X0.x, X0.y}, f2{X0.z, X0.w}, f2{X1.x, X1.y}, f2{X1.z, X1.w},
                  f2{Y0.x, Y0.y}, f2{Y0.z, Y0.w}, f2{Y1.x, Y1.y}, f2{Y1.z, Y1.w}, f2{Z0.x, Z0.y},
                  f2{Z0.z, Z0.w}, f2{Z1.x, Z1.y}, f2{Z1.z, Z1.w}, f2{S0.x, S0.y}, f2{S0.z, S0.w},
                  f2{S1.x, S1.y}, f2{S1.z, S1.w}, a0, b0, c0, d0);
        grp_dup(dx, dy, dz, kk, oxx, oyy, ozz, f2{X0.x, X0.y}, f2{X0.z, X0.w}, f2{X1.x, X1.y},
                f2{X1.z, X1.w}, f2{Y0.x, Y0.y}, f2{Y0.z, Y0.w}, f2{Y1.x, Y1.y}, f2{Y1.z, Y1.w},
                f2{Z0.x, Z0.y}, f2{Z0.z, Z0.w}, f2{Z1.x, Z1.y}, f2{Z1.z, Z1.w}, f2{S0.x, S0.y},
                f2{S0.z, S0.w}, f2{S1.x, S1.y}, f2{S1.z, S1.w}, a1, b1, c1, d1);
        nbad += neq(a0, a1) + neq(b0, b1) + neq(c0, c1) + neq(d0, d1);
        if (nbad != nbad_seen) {  // which form is off: both against the scalar reference
            nbad_seen = nbad;
            const f2 ra = grp_scalar2(ex, ey, ez, k1, ox, oy, oz, f2{X0.x, X0.y}, f2{Y0.x, Y0.y},
                                      f2{Z0.x, Z0.y}, f2{S0.x, S0.y});
            const f2 rb = grp_scalar2(ex, ey, ez, k1, ox, oy, oz, f2{X0.z, X0.w}, f2{Y0.z, Y0.w},
                                      f2{Z0.z, Z0.w}, f2{S0.z, S0.w});
            const f2 rc = grp_scalar2(ex, ey, ez, k1, ox, oy, oz, f2{X1.x, X1.y}, f2{Y1.x, Y1.y},
                                      f2{Z1.x, Z1.y}, f2{S1.x, S1.y});
            const f2 rd = grp_scalar2(ex, ey, ez, k1, ox, oy, oz, f2{X1.z, X1.w}, f2{Y1.z, Y1.w},
                                      f2{Z1.z, Z1.w}, f2{S1.z, S1.w});
            nb_op += neq(a0, ra) + neq(b0, rb) + neq(c0, rc) + neq(d0, rd);
            nb_dup += neq(a1, ra) + neq(b1, rb) + neq(c1, rc) + neq(d1, rd);
        }
        acc += a0.x + d1.y;
    }
    bad[gid] = nbad;
    bad_opsel[gid] = nb_op;
    bad_dup[gid] = nb_dup;
    sink[gid] = acc;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    int dev = 0, ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t blocks = (uint32_t)ncu * 4;  // 4 workgroups (16 waves) per CU
    const uint32_t n = blocks * 256;
    // sphere groups (SoA cx[8] cy[8] cz[8] S[8]) and per-lane ray constants,
    // values of the RTIOW scale (|c| ~ 10, |o| ~ 13)
    const uint32_t ngroups = 61;
    std::vector<float> hg(ngroups * 32), hr((size_t)n * 8);
    srand(1234);
    auto U = [] { return (float)rand() / (float)RAND_MAX; };
    for (auto& x : hg) x = 20.f * U() - 10.f;
    for (size_t i = 0; i < (size_t)n; ++i)
        for (int k = 0; k < 8; ++k) hr[i * 8 + k] = (k < 3 ? 2.f * U() - 1.f : 26.f * U() - 13.f);
    float *dg, *dr, *sink;
    unsigned *dbad, *dbo, *dbd;
    hipMalloc(&dg, hg.size() * 4);
    hipMalloc(&dr, hr.size() * 4);
    hipMalloc(&sink, (size_t)n * 4);
    hipMalloc(&dbad, (size_t)n * 4);
    hipMalloc(&dbo, (size_t)n * 4);
    hipMalloc(&dbd, (size_t)n * 4);
    hipMemcpy(dg, hg.data(), hg.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dr, hr.data(), hr.size() * 4, hipMemcpyHostToDevice);
    std::vector<unsigned> hb(n), hbo(n), hbd(n);
    const char* names[6] = {"mfma (even waves MFMA, odd waves filter)",
                            "idle (even waves s_sleep, odd waves filter)",
                            "valu (every wave filter, no MFMA)",
                            "permlane (even waves permlane32_swap)",
                            "lds (even waves LDS queue traffic)",
                            "walk (even waves MFMA + OR + swap + LDS)"};
    int fails = 0;
    for (int mode = 0; mode < 6; ++mode)
        for (int rep = 0; rep < reps; ++rep) {
            hipMemset(dbad, 0, (size_t)n * 4);
            hipMemset(dbo, 0, (size_t)n * 4);
            hipMemset(dbd, 0, (size_t)n * 4);
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_opsel, dim3(blocks), dim3(256), 0, 0, (const float4*)dg, ngroups,
                               dr, mode, dbad, dbo, dbd, sink);
            hipEventRecord(e1);
            if (hipEventSynchronize(e1) != hipSuccess) {
                printf("launch failed\n");
                return 2;
            }
            float ms = 0.f;
            hipEventElapsedTime(&ms, e0, e1);
            hipMemcpy(hb.data(), dbad, (size_t)n * 4, hipMemcpyDeviceToHost);
            hipMemcpy(hbo.data(), dbo, (size_t)n * 4, hipMemcpyDeviceToHost);
            hipMemcpy(hbd.data(), dbd, (size_t)n * 4, hipMemcpyDeviceToHost);
            unsigned long long tot = 0, lanes = 0, to = 0, td = 0;
            for (size_t i = 0; i < hb.size(); ++i) {
                tot += hb[i];
                lanes += hb[i] != 0;
                to += hbo[i];
                td += hbd[i];
            }
            printf("%-46s rep %d: %8.2f ms, %llu differing values in %llu lanes "
                   "(of %llu op_sel filter groups); first differing group per lane vs the "
                   "scalar fma reference: op_sel form %llu values off, duplicated-pair form %llu\n",
                   names[mode], rep, ms, tot, lanes,
                   (unsigned long long)(mode == 2 ? n : n / 2) * ITERS, to, td);
            fflush(stdout);
            fails += tot != 0;
        }
    return 0;
}
