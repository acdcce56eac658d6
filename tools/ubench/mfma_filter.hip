// Micro-benchmark for the next-round design question: the conservative
// sphere filter of rt_render_kernel on the matrix cores vs the packed-fp32
// VALU form, both in isolation (no candidate queue, no exact test), every CU
// busy, W waves per SIMD, the same rays x spheres work:
//   VALU: per group of 8 spheres 28 v_pk_fma_f32 + 3 v_max3 + v_max + v_cmp
//         (rt_dev_intersect.h filter8), sphere data as SGPR pairs (s_load);
//   MFMA: per 32 spheres x 32 rays two v_mfma_f32_32x32x16_f16 (hb and v + S
//         from one shared K = 16 sphere fragment, f16 hi/lo products), then
//         H = hb^2 + (v + S) (8 v_pk_fma_f32), the per-group max over the
//         lane's 4 rows, the other half's 4 rows via v_permlane32_swap, and the
//         compare with the ray's threshold.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1
// (MFMA results in VGPRs: no v_accvgpr_read per output).
// Reported: ms and SIMD cycles per (64 rays x 8 spheres) unit; the values are
// synthetic (the candidate masks are folded into the output so nothing is
// dead code), only the instruction mix and its issue cost matter here.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(4))) const float4 cfloat4;

#define NGROUPS 64  // 512 spheres: 64 groups of 8 = 16 blocks of 32

// ---- VALU form (the product's filter8, reduced to its arithmetic) ----
__global__ __launch_bounds__(256) void k_valu(const float4* __restrict__ grp, float* out,
                                              int iters) {
    const float t = threadIdx.x * 1e-3f;
    f2 r0 = {t, t + 0.1f}, r1 = {t + 0.2f, t + 0.3f}, r2 = {t + 0.4f, t + 0.5f},
       r3 = {t + 0.6f, 1e30f};
    asm volatile("" : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3));
    uint64_t acc = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    const cfloat4* gp = (const cfloat4*)(uintptr_t)grp;  // scalar-cache reads
#else
    const float4* gp = grp;  // host pass: never executed
#endif
    for (int it = 0; it < iters; ++it) {
        for (int g = 0; g < NGROUPS; ++g) {
            const auto* p = gp + (size_t)g * 8;
            const float4 X0 = p[0], X1 = p[1], Y0 = p[2], Y1 = p[3];
            const float4 Z0 = p[4], Z1 = p[5], S0 = p[6], S1 = p[7];
            f2 ha, hb, hc, hd;
            float hm;
            const f2 cxa = {X0.x, X0.y}, cxb = {X0.z, X0.w}, cxc = {X1.x, X1.y}, cxd = {X1.z, X1.w};
            const f2 cya = {Y0.x, Y0.y}, cyb = {Y0.z, Y0.w}, cyc = {Y1.x, Y1.y}, cyd = {Y1.z, Y1.w};
            const f2 cza = {Z0.x, Z0.y}, czb = {Z0.z, Z0.w}, czc = {Z1.x, Z1.y}, czd = {Z1.z, Z1.w};
            const f2 sa = {S0.x, S0.y}, sb = {S0.z, S0.w}, sc = {S1.x, S1.y}, sd = {S1.z, S1.w};
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
                "v_max3_f32 %[hm], v40, v41, v42\n\t"
                "v_max3_f32 %[hm], %[hm], v43, v44\n\t"
                "v_max3_f32 %[hm], %[hm], v45, v46\n\t"
                "v_max_f32 %[hm], %[hm], v47"
                : [ha] "={v[40:41]}"(ha), [hb] "={v[42:43]}"(hb), [hc] "={v[44:45]}"(hc),
                  [hd] "={v[46:47]}"(hd), [hm] "=&v"(hm)
                : [r0] "v"(r0), [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [cxa] "s"(cxa),
                  [cxb] "s"(cxb), [cxc] "s"(cxc), [cxd] "s"(cxd), [cya] "s"(cya), [cyb] "s"(cyb),
                  [cyc] "s"(cyc), [cyd] "s"(cyd), [cza] "s"(cza), [czb] "s"(czb), [czc] "s"(czc),
                  [czd] "s"(czd), [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc), [sd] "s"(sd));
            acc += __builtin_amdgcn_ballot_w64(hm >= r3.y);
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(acc & 0xFFFF) + r0.x;
}

// ---- MFMA form ----
// A: per 32-sphere block b, lane l holds A[row l%32][k 8*(l/32) .. +8) (f16).
__global__ __launch_bounds__(256) void k_mfma(const h8* __restrict__ A, float* out, int iters) {
    const unsigned lane = threadIdx.x & 63u;
    const float t = lane * 1e-3f;
    h8 bu0, bv0, bu1, bv1;  // ray fragments of the two 32-ray halves (built once per iteration)
    for (int i = 0; i < 8; ++i) {
        bu0[i] = (_Float16)(t - i * 1e-2f);
        bv0[i] = (_Float16)(t + i * 1e-2f);
        bu1[i] = (_Float16)(t * 0.5f - i * 1e-2f);
        bv1[i] = (_Float16)(t * 0.5f + i * 1e-2f);
    }
    asm volatile("" : "+v"(bu0), "+v"(bv0), "+v"(bu1), "+v"(bv1));
    float T0 = 1e3f + t, T1 = 1e3f - t;
    asm volatile("" : "+v"(T0), "+v"(T1));
    uint64_t acc = 0;
    const f16v zero = {};
    for (int it = 0; it < iters; ++it) {
        h8 a = A[lane];
        for (int b = 0; b < NGROUPS / 4; ++b) {
            const h8 an = A[((b + 1) & (NGROUPS / 4 - 1)) * 64 + lane];  // next block's fragment
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const h8 bu = half ? bu1 : bu0, bv = half ? bv1 : bv0;
                const float T = half ? T1 : T0;
                const f16v U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bu, zero, 0, 0, 0);
                const f16v V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, bv, zero, 0, 0, 0);
                float H[16];
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    const f2 hb = {U[i], U[i + 1]}, vs = {V[i], V[i + 1]};
                    const f2 h = __builtin_elementwise_fma(hb, hb, vs);
                    H[i] = h.x;
                    H[i + 1] = h.y;
                }
                uint64_t any = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
#ifdef GROUP8  // groups of 8 rows: 4 here, 4 in lane ^ 32 (v_permlane32_swap)
                    const float m = __builtin_fmaxf(__builtin_fmaxf(H[4 * q], H[4 * q + 1]),
                                                    __builtin_fmaxf(H[4 * q + 2], H[4 * q + 3]));
                    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(m),
                                                                     __float_as_uint(m), false, false);
                    const float g = __builtin_fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
#else  // groups of 4 rows, whole in this lane: no cross-half exchange
                    const float g = __builtin_fmaxf(__builtin_fmaxf(H[4 * q], H[4 * q + 1]),
                                                    __builtin_fmaxf(H[4 * q + 2], H[4 * q + 3]));
#endif
                    any |= __builtin_amdgcn_ballot_w64(g >= T);
                }
                acc += any;
            }
            a = an;
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)(acc & 0xFFFF) + t;
}

template <typename F>
float timed(F launch) {
    launch();
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    return best;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    float4* grp;
    h8* A;
    float* out;
    (void)hipMalloc(&grp, NGROUPS * 8 * sizeof(float4));
    (void)hipMalloc(&A, (NGROUPS / 4) * 64 * sizeof(h8));
    (void)hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float));
    (void)hipMemset(grp, 0, NGROUPS * 8 * sizeof(float4));
    (void)hipMemset(A, 0, (NGROUPS / 4) * 64 * sizeof(h8));
    const int iters = 400;
    for (int W : {4, 6}) {
        const int blocks = cus * W;  // W workgroups of 4 waves per CU = W waves per SIMD
        const float v = timed([&] { hipLaunchKernelGGL(k_valu, blocks, 256, 0, 0, grp, out, iters); });
        const float m = timed([&] { hipLaunchKernelGGL(k_mfma, blocks, 256, 0, 0, A, out, iters); });
        // per SIMD: W waves x iters x 64 units of (64 rays x 8 spheres)
        const double units = (double)W * iters * NGROUPS;
        printf("W=%d  VALU filter %.3f ms (%.1f cyc per 64 rays x 8 spheres)  "
               "MFMA filter %.3f ms (%.1f cyc)  ratio %.3f\n",
               W, v, v * 1e-3 * 2.4e9 / units, m, m * 1e-3 * 2.4e9 / units, m / v);
    }
    (void)hipFree(grp);
    (void)hipFree(A);
    (void)hipFree(out);
    return 0;
}
