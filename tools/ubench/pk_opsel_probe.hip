// Probe kernels for tools/hazard_audit.py: each kernel puts one
// producer -> consumer pair of the audit's rules (R1-R5) in hipcc's hands, so
// the wait states the compiler inserts between them (its s_nop) can be read off
// the assembly, and the packed forms it emits for f2{x, x} operands (R6) are
// visible. Compile only -- these kernels are never launched:
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -S --cuda-device-only \
//         tools/ubench/pk_opsel_probe.hip -o tools/ubench/pk_opsel_probe.s
//
// What the committed pk_opsel_probe.s shows:
//   probe_r1_*   v_pk_fma_f32 -> a VALU reading its result: the forwarding
//                wait (s_nop 0) after a packed FMA whose src0 is a whole pair
//                (VGPR or SGPR), none after the src0-broadcast form
//                (op_sel_hi:[0,1,1], probe_r1_src0_broadcast);
//   probe_r6_*   an f2{x, x} operand held in one VGPR becomes op_sel_hi
//                selecting that VGPR's half -- the form rule R6 refuses in a
//                kernel that issues MFMAs; the duplicated pair is the form the
//                render kernel uses instead;
//   probe_r3     8-pass MFMA -> a VALU reading its accumulator (s_nop before it);
//   probe_r4     VALU -> v_permlane32_swap reading its result;
//   probe_r5     VALU -> v_readlane reading its result.
#include <hip/hip_runtime.h>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

extern "C" __global__ void probe_r1_vgpr_pairs(const f2* __restrict__ in, float* __restrict__ out) {
    const int i = threadIdx.x;
    f2 a = in[i], b = in[i + 64], c = in[i + 128];
    f2 r = pk_fma(a, b, c);
    out[i] = r.x + r.y;  // consumer reads the packed result at once
}

extern "C" __global__ void probe_r1_sgpr_pair(const f2* __restrict__ in, f2 k, float* __restrict__ out) {
    const int i = threadIdx.x;
    f2 a = in[i], c = in[i + 64];
    f2 r = pk_fma(a, k, c);  // k: a kernel argument, an SGPR pair
    out[i] = r.x + r.y;
}

extern "C" __global__ void probe_r1_src0_broadcast(const f2* __restrict__ in, const float* __restrict__ s,
                                                   f2 k, float* __restrict__ out) {
    const int i = threadIdx.x;
    const float x = s[i];
    f2 c = in[i];
    f2 r = pk_fma(f2{x, x}, k, c);  // VGPR broadcast against an SGPR pair
    out[i] = r.x + r.y;
}

extern "C" __global__ void probe_r6_broadcast(const f2* __restrict__ in, const float* __restrict__ s,
                                              float* __restrict__ out) {
    const int i = threadIdx.x;
    const float x = s[i];        // one VGPR
    f2 a = in[i], c = in[i + 64];
    f2 r = pk_fma(a, f2{x, x}, c);  // hipcc: op_sel_hi selecting x's VGPR for both halves
    out[i] = r.x * r.y;
}

extern "C" __global__ void probe_r6_duplicated_pair(const f2* __restrict__ in, const f2* __restrict__ s,
                                                    float* __restrict__ out) {
    const int i = threadIdx.x;
    const f2 xx = s[i];          // the pair already holds {x, x} in two VGPRs
    f2 a = in[i], c = in[i + 64];
    f2 r = pk_fma(a, xx, c);
    out[i] = r.x * r.y;
}

extern "C" __global__ void probe_r3(const h8* __restrict__ a, const h8* __restrict__ b, float* __restrict__ out) {
    const int i = threadIdx.x;
    f16v acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i], b[i], acc, 0, 0, 0);
    float m = acc[0];
#pragma unroll
    for (int k = 1; k < 16; ++k) m = fmaxf(m, acc[k]);  // VALU reads the accumulator
    out[i] = m;
}

extern "C" __global__ void probe_r4(const unsigned* __restrict__ in, unsigned* __restrict__ out) {
    const int i = threadIdx.x;
    unsigned x = in[i] ^ in[i + 64];  // VALU producer
    auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    out[i] = r[0] + r[1];
}

extern "C" __global__ void probe_r5(const unsigned* __restrict__ in, unsigned* __restrict__ out) {
    const int i = threadIdx.x;
    unsigned x = in[i] + in[i + 64];  // VALU producer
    out[i] = __builtin_amdgcn_readlane(x, 5);
}
