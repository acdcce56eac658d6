/*
 * rt_oracle.h — CPU oracle for the path-tracer hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * or the timed CPU baseline. The product path (bevy_raytrace_amd/) never links
 * or calls it.
 *
 * A scalar C restatement of the reference's WGSL compute path
 * (assets/shaders/{clear,generate,intersect,shade,collect}.wgsl of
 * brandon-reinhart/bevy_raytrace), with every floating-point operation order
 * fixed; see DESIGN.md "Oracle" for the op-form table.
 * The reference ships no tests, golden images or known-answer vectors and its
 * WGSL has no runtime here. The oracle is pinned by the
 * reference's own six shaders executed by a WGSL interpreter
 * (tests/golden/wgsl_exec.py; fixtures tests/golden/wgsl_*.npz, bit-exact per
 * frame at the reference's depth 3), by the known-answer values of SURVEY
 * Appendix C and by an independent numpy restatement (oracle/rt_oracle_np.py).
 * Unpinned: the precision of the builtins the WGSL leaves to the driver
 * (normalize, length, pow, tan; FMA fusion), fixed below.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>
#include "../include/rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* hash3, shade.wgsl:105-116 */
void rto_hash3(uint32_t n, float out[3]);

/* tan(fov/2) as the renderer uses it (generate.wgsl:67), computed once on the host. */
float rto_tan_half(float fov);

/* rt_sincos of the opt-in thin-lens sampling (rt_hip.h). */
void rto_sincos(float theta, float* s, float* c);

/* Primary ray of pixel (x, y): generate.wgsl:66-129 with lens_offset = 0. */
void rto_primary_ray(const rt_camera* cam, uint32_t width, uint32_t height,
                     uint32_t x, uint32_t y, float origin[3], float dir[3]);

/* Sky colour for a miss along dir: shade.wgsl:189-197. */
void rto_sky(const float dir[3], float out[3]);

/* Closest hit, intersect.wgsl:94-143. Returns the sphere index or -1 (miss);
 * fills t / position / normal / front_face for a hit. */
int rto_intersect(const rt_sphere* spheres, uint32_t n, const float origin[3],
                  const float dir[3], float* t, float pos[3], float normal[3],
                  uint32_t* front_face);

/* Batch of rays (n x 6 floats: origin, direction) -> index (-1 miss) and t. */
void rto_intersect_batch(const rt_sphere* spheres, uint32_t n, const float* rays,
                         uint32_t nrays, int32_t* idx, float* t, int nthreads);

/* One path: colour of sample `frame` of pixel (x, y), and its segment count
 * (reference camera sampling: no jitter, lens offset 0). */
void rto_trace_path(const rt_camera* cam, const rt_sphere* spheres, uint32_t n,
                    const rt_material* materials, uint32_t m, uint32_t width,
                    uint32_t height, uint32_t x, uint32_t y, uint32_t frame,
                    uint32_t max_depth, float color[3], uint32_t* segments);

/* params->flags bit: write the block-folded sample SUMS (alpha 0) instead of
 * sum / spp -- for checking progressive accumulation. */
#define RTO_FLAG_RAW_SUMS 0x80000000u

/* Full render of the rows owned by params' shard (layout as rt_render).
 * nthreads <= 0 -> 1. Returns 0, or -1 on invalid arguments. */
int rto_render(const rt_camera* cam, const rt_sphere* spheres, uint32_t n,
               const rt_material* materials, uint32_t m, const rt_params* params,
               float* out_rgba, uint64_t* segments, int nthreads);

/* Render an explicit list of global rows (for sampled-row parity at large sizes).
 * out_rgba holds nrows*width*4 floats in list order. */
int rto_render_rows(const rt_camera* cam, const rt_sphere* spheres, uint32_t n,
                    const rt_material* materials, uint32_t m, const rt_params* params,
                    const uint32_t* rows, uint32_t nrows, float* out_rgba,
                    uint64_t* segments, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
