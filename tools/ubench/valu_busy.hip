// Calibration of the VALU counters on gfx950: kernels whose VALU stream is
// known instruction by instruction (inline asm, independent operands, 6
// waves per SIMD like rt_render_kernel), timed with HIP events. Run under
//   rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES
//             SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- ./valu_busy
// to relate SQ_ACTIVE_INST_VALU (quad-cycles per the counter description) and
// GRBM_GUI_ACTIVE (summed over the 8 XCDs) to the issue cycles each class
// of instruction really takes (tools/valu_calib.py reads the output).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
#define ITERS 8192

// 8 independent v_pk_fma_f32 per iteration (vector operands only)
__global__ __launch_bounds__(256) void k_pk8(float* out, float a) {
    f2 x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    f2 x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    f2 va = {a, a};
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_pk_fma_f32 %0, %0, %8, %8\n\tv_pk_fma_f32 %1, %1, %8, %8\n\t"
            "v_pk_fma_f32 %2, %2, %8, %8\n\tv_pk_fma_f32 %3, %3, %8, %8\n\t"
            "v_pk_fma_f32 %4, %4, %8, %8\n\tv_pk_fma_f32 %5, %5, %8, %8\n\t"
            "v_pk_fma_f32 %6, %6, %8, %8\n\tv_pk_fma_f32 %7, %7, %8, %8"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(va));
    }
    f2 s = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

// 8 independent v_fma_f32 per iteration
__global__ __launch_bounds__(256) void k_fma8(float* out, float a) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
          x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_fma_f32 %0, %0, %8, %8\n\tv_fma_f32 %1, %1, %8, %8\n\t"
            "v_fma_f32 %2, %2, %8, %8\n\tv_fma_f32 %3, %3, %8, %8\n\t"
            "v_fma_f32 %4, %4, %8, %8\n\tv_fma_f32 %5, %5, %8, %8\n\t"
            "v_fma_f32 %6, %6, %8, %8\n\tv_fma_f32 %7, %7, %8, %8"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(a));
    }
    out[blockIdx.x * 256 + threadIdx.x] = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
}

// 8 independent v_add_u32 per iteration (integer ops of the bookkeeping)
__global__ __launch_bounds__(256) void k_add8(float* out, float a) {
    unsigned x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
             x6 = x0 + 6, x7 = x0 + 7, k = __float_as_uint(a);
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\t"
            "v_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
            "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\t"
            "v_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(k));
    }
    out[blockIdx.x * 256 + threadIdx.x] = (float)(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7);
}

// the filter group's shape: 4 v_pk_fma_f32 + 4 v_max3_f32-like scalar ops
__global__ __launch_bounds__(256) void k_mix(float* out, float a) {
    f2 x0 = {(float)threadIdx.x, 1.f}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
    float y0 = threadIdx.x, y1 = y0 + 1, y2 = y0 + 2, y3 = y0 + 3;
    f2 va = {a, a};
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_pk_fma_f32 %0, %0, %8, %8\n\tv_max3_f32 %4, %4, %9, %9\n\t"
            "v_pk_fma_f32 %1, %1, %8, %8\n\tv_max3_f32 %5, %5, %9, %9\n\t"
            "v_pk_fma_f32 %2, %2, %8, %8\n\tv_max3_f32 %6, %6, %9, %9\n\t"
            "v_pk_fma_f32 %3, %3, %8, %8\n\tv_max3_f32 %7, %7, %9, %9"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3)
            : "v"(va), "v"(a));
    }
    f2 s = (x0 + x1) + (x2 + x3);
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y + y0 + y1 + y2 + y3;
}

// One VOP instruction form, 8 independent operands per iteration (x_i = op(x_i, k)).
#define RT_VALU_KERNEL(NAME, INSN, T)                                                        \
    __global__ __launch_bounds__(256) void NAME(float* out, float a) {                      \
        T x0 = (T)threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,           \
          x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                             \
        T k = (T)a;                                                                          \
        for (int i = 0; i < ITERS; ++i) {                                                    \
            asm volatile(INSN " %0, %0, %8\n\t" INSN " %1, %1, %8\n\t" INSN " %2, %2, %8\n\t" \
                         INSN " %3, %3, %8\n\t" INSN " %4, %4, %8\n\t" INSN " %5, %5, %8\n\t" \
                         INSN " %6, %6, %8\n\t" INSN " %7, %7, %8"                           \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5),     \
                           "+v"(x6), "+v"(x7)                                                \
                         : "v"(k));                                                          \
        }                                                                                    \
        out[blockIdx.x * 256 + threadIdx.x] = (float)(x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7); \
    }
RT_VALU_KERNEL(k_addf8, "v_add_f32", float)
RT_VALU_KERNEL(k_mulf8, "v_mul_f32", float)
RT_VALU_KERNEL(k_max8, "v_max_f32", float)
RT_VALU_KERNEL(k_and8, "v_and_b32", unsigned)
RT_VALU_KERNEL(k_mullo8, "v_mul_lo_u32", unsigned)

// 8 independent v_cndmask_b32 on one SGPR-pair mask
__global__ __launch_bounds__(256) void k_cnd8(float* out, float a) {
    float x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
          x6 = x0 + 6, x7 = x0 + 7;
    const bool c = threadIdx.x & 1;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_cndmask_b32_e64 %0, %0, %8, %9\n\tv_cndmask_b32_e64 %1, %1, %8, %9\n\t"
            "v_cndmask_b32_e64 %2, %2, %8, %9\n\tv_cndmask_b32_e64 %3, %3, %8, %9\n\t"
            "v_cndmask_b32_e64 %4, %4, %8, %9\n\tv_cndmask_b32_e64 %5, %5, %8, %9\n\t"
            "v_cndmask_b32_e64 %6, %6, %8, %9\n\tv_cndmask_b32_e64 %7, %7, %8, %9"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(a), "s"(__builtin_amdgcn_ballot_w64(c)));
    }
    out[blockIdx.x * 256 + threadIdx.x] = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
}

// 8 v_cmp_ge_f32 into SGPR pairs (the filter's candidate mask compares)
__global__ __launch_bounds__(256) void k_cmp8(float* out, float a) {
    const float x = threadIdx.x;
    uint64_t m0, m1, m2, m3, m4, m5, m6, m7;
    uint64_t acc = 0;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_cmp_ge_f32_e64 %0, %8, %9\n\tv_cmp_ge_f32_e64 %1, %8, %9\n\t"
            "v_cmp_ge_f32_e64 %2, %8, %9\n\tv_cmp_ge_f32_e64 %3, %8, %9\n\t"
            "v_cmp_ge_f32_e64 %4, %8, %9\n\tv_cmp_ge_f32_e64 %5, %8, %9\n\t"
            "v_cmp_ge_f32_e64 %6, %8, %9\n\tv_cmp_ge_f32_e64 %7, %8, %9"
            : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3), "=s"(m4), "=s"(m5), "=s"(m6), "=s"(m7)
            : "v"(x), "v"(a));
        acc ^= m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7;
    }
    out[blockIdx.x * 256 + threadIdx.x] = (float)(acc & 0xFF);
}

// 8 independent v_sqrt_f32 (transcendental unit)
__global__ __launch_bounds__(256) void k_sqrt8(float* out, float a) {
    float x0 = threadIdx.x + a, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,
          x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_sqrt_f32 %0, %0\n\tv_sqrt_f32 %1, %1\n\tv_sqrt_f32 %2, %2\n\tv_sqrt_f32 %3, %3\n\t"
            "v_sqrt_f32 %4, %4\n\tv_sqrt_f32 %5, %5\n\tv_sqrt_f32 %6, %6\n\tv_sqrt_f32 %7, %7"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));
    }
    out[blockIdx.x * 256 + threadIdx.x] = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
}

// forms considered for the candidate mask (sign bits of H - T instead of 8
// compares into SGPRs): packed add, byte permute, shift-or, add-with-carry
typedef float f2v __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_pkadd8(float* out, float a) {
    f2v x0 = {(float)threadIdx.x, 1.0f}, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,
        x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
    const f2v k = {a, a};
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_pk_add_f32 %0, %0, %8\n\tv_pk_add_f32 %1, %1, %8\n\t"
            "v_pk_add_f32 %2, %2, %8\n\tv_pk_add_f32 %3, %3, %8\n\t"
            "v_pk_add_f32 %4, %4, %8\n\tv_pk_add_f32 %5, %5, %8\n\t"
            "v_pk_add_f32 %6, %6, %8\n\tv_pk_add_f32 %7, %7, %8"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(k));
    }
    const f2v s2 = ((x0 + x1) + (x2 + x3)) + ((x4 + x5) + (x6 + x7));
    out[blockIdx.x * 256 + threadIdx.x] = s2.x + s2.y;
}
#define RT_VOP3_KERNEL(NAME, INSN)                                                          \
    __global__ __launch_bounds__(256) void NAME(float* out, float a) {                      \
        unsigned x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,       \
                 x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                      \
        const unsigned k = (unsigned)(a * 1000.0f), sel = 0x07030602u;                       \
        for (int i = 0; i < ITERS; ++i) {                                                    \
            asm volatile(INSN(0) "\n\t" INSN(1) "\n\t" INSN(2) "\n\t" INSN(3) "\n\t"     \
                         INSN(4) "\n\t" INSN(5) "\n\t" INSN(6) "\n\t" INSN(7)              \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5),     \
                           "+v"(x6), "+v"(x7)                                                \
                         : "v"(k), "v"(sel));                                                \
        }                                                                                    \
        out[blockIdx.x * 256 + threadIdx.x] = (float)(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7); \
    }
#define PERM_I(n) "v_perm_b32 %" #n ", %" #n ", %8, %9"
#define LSHLOR_I(n) "v_lshl_or_b32 %" #n ", %" #n ", 1, %8"
#define MOV_I(n) "v_mov_b32 %" #n ", %8"
#define ANDOR_I(n) "v_and_or_b32 %" #n ", %" #n ", %9, %8"
RT_VOP3_KERNEL(k_perm8, PERM_I)
RT_VOP3_KERNEL(k_lshlor8, LSHLOR_I)
RT_VOP3_KERNEL(k_mov8, MOV_I)
RT_VOP3_KERNEL(k_andor8, ANDOR_I)

// 8 v_addc_co_u32 (carry in/out in SGPR pairs), the current mask build
__global__ __launch_bounds__(256) void k_addc8(float* out, float a) {
    unsigned x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
             x6 = x0 + 6, x7 = x0 + 7;
    const uint64_t c = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);
    uint64_t o0, o1, o2, o3, o4, o5, o6, o7;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_addc_co_u32_e64 %0, %8, %0, %0, %16\n\tv_addc_co_u32_e64 %1, %9, %1, %1, %16\n\t"
            "v_addc_co_u32_e64 %2, %10, %2, %2, %16\n\tv_addc_co_u32_e64 %3, %11, %3, %3, %16\n\t"
            "v_addc_co_u32_e64 %4, %12, %4, %4, %16\n\tv_addc_co_u32_e64 %5, %13, %5, %5, %16\n\t"
            "v_addc_co_u32_e64 %6, %14, %6, %6, %16\n\tv_addc_co_u32_e64 %7, %15, %7, %7, %16"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7),
              "=&s"(o0), "=&s"(o1), "=&s"(o2), "=&s"(o3), "=&s"(o4), "=&s"(o5), "=&s"(o6), "=&s"(o7)
            : "s"(c));
    }
    out[blockIdx.x * 256 + threadIdx.x] = (float)(x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int grid = cus * 6;  // 6 workgroups of 4 waves per CU = 6 waves per SIMD
    float* d;
    hipMalloc(&d, (size_t)grid * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct K { const char* name; void (*fn)(float*, float); } ks[] = {
        {"pk_fma x8", k_pk8}, {"fma x8", k_fma8}, {"add_u32 x8", k_add8},
        {"pk_fma x4 + max3 x4", k_mix}, {"add_f32 x8", k_addf8}, {"mul_f32 x8", k_mulf8},
        {"max_f32 x8", k_max8}, {"and_b32 x8", k_and8}, {"mul_lo_u32 x8", k_mullo8},
        {"cndmask_b32 x8", k_cnd8}, {"cmp_ge_f32 x8", k_cmp8}, {"sqrt_f32 x8", k_sqrt8},
        {"pk_add_f32 x8", k_pkadd8}, {"perm_b32 x8", k_perm8}, {"lshl_or_b32 x8", k_lshlor8},
        {"mov_b32 x8", k_mov8}, {"and_or_b32 x8", k_andor8}, {"addc_co_u32 x8", k_addc8}};
    for (int rep = 0; rep < 2; ++rep)
        for (const K& k : ks) {
            float ms = 0.0f;
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.fn, dim3(grid), dim3(256), 0, 0, d, 0.999f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms, e0, e1);
            const double inst_per_simd = 8.0 * ITERS * 6;  // 6 waves, 8 VALU per iteration
            // cycles per VALU instruction per SIMD at the nominal 2.4 GHz
            printf("%-22s %8.3f ms  %.3f cyc/inst/SIMD @2.4GHz\n", k.name, ms,
                   ms * 1e-3 * 2.4e9 / inst_per_simd);
        }
    hipFree(d);
    return 0;
}
