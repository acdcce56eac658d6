/*
 * rt_hip.h — C-ABI of the MI355X-native per-pixel path tracer.
 *
 * This is the drop-in boundary that replaces the reference's WGSL dispatch
 * schedule. In brandon-reinhart/bevy_raytrace the per-frame work is recorded by
 *   impl render_graph::Node for RayTraceNode { fn update(..); fn run(..) }
 *   (src/ray_trace_node.rs:173-224)
 * which dispatches clear / generate / 3x(prepass, intersect, shade) / collect
 * (assets/shaders/{clear,generate,intersect,shade,collect}.wgsl) over buffers packed by the `prepare` systems of
 * src/ray_trace_camera.rs:43-68, src/ray_trace_globals.rs:56-68,
 * src/sphere.rs:166-197 and src/ray_trace_materials.rs:129-164.
 *
 * Here the whole chain is ONE persistent HIP kernel on gfx950 behind the entry
 * points below. Plain pointers and sizes only; no torch / HIP types appear in
 * the signatures (streams are passed as `void*` = hipStream_t).
 *
 * Byte layouts mirror the reference's encase/std430/std140 layouts exactly,
 * so a Rust shim can hand over `encase`-packed bytes unchanged:
 *   rt_sphere   = SphereGPU   (src/sphere.rs:12-17; intersect.wgsl:56-60), 32 B
 *   rt_material = MaterialGPU (src/ray_trace_materials.rs:33-43; shade.wgsl:67-73), 32 B
 *   rt_camera   = CameraGPU   (src/ray_trace_camera.rs:14-25; generate.wgsl:5-15), 128 B std140
 *
 * Error convention: every entry point returns an int status (RT_OK = 0,
 * negative = error class) and never throws or aborts across the ABI; the
 * message of the last failing call on a context is rt_last_error(ctx).
 * (The reference panics via unwrap(), src/ray_trace_node.rs:51-53.)
 *
 * Threading: one rt_ctx per device; calls on one ctx must be serialised by the
 * caller; distinct contexts may be used concurrently from different threads.
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 1

/* status codes */
#define RT_OK                 0
#define RT_ERR_INVALID_ARG   -1   /* bad pointer / size / parameter            */
#define RT_ERR_NO_SCENE      -2   /* rt_render before rt_set_scene             */
#define RT_ERR_DEVICE        -3   /* HIP runtime error (message has details)   */
#define RT_ERR_OUT_OF_MEMORY -4   /* device allocation failed                  */
#define RT_ERR_BAD_SCENE     -5   /* material index / reflectance out of range */

/* Reflectance codes, src/ray_trace_materials.rs:144-153 (Lambertian=0,
 * Metallic=1, Dielectric=2), consumed by shade.wgsl:240-252. */
#define RT_LAMBERTIAN 0
#define RT_METALLIC   1
#define RT_DIELECTRIC 2

/* SphereGPU {center: Vec3, radius: f32, material: u32} in a std430 runtime
 * array: 32-byte stride (src/sphere.rs:12-17). */
typedef struct rt_sphere {
    float    center[3];
    float    radius;
    uint32_t material;
    uint32_t _pad[3];
} rt_sphere;

/* MaterialGPU {color: Vec4, reflectance: i32, fuzziness: f32,
 * index_of_refraction: f32, pad2: i32} (src/ray_trace_materials.rs:33-43). */
typedef struct rt_material {
    float   color[4];
    int32_t reflectance;
    float   fuzziness;
    float   index_of_refraction;
    int32_t _pad;
} rt_material;

/* CameraGPU, std140, 128 B (src/ray_trace_camera.rs:14-25).
 * transform is column-major (glam Mat4): transform[col*4 + row]. Only
 * transform, fov, image_plane_distance and lens_focal_length are read by the
 * path (generate.wgsl:67-126); forward/up/right/position/fstop are carried. */
typedef struct rt_camera {
    float transform[16];
    float forward[3];  float fov;
    float up[3];       float image_plane_distance;
    float right[3];    float lens_focal_length;
    float position[3]; float fstop;
} rt_camera;

/* Render parameters (replaces GlobalsGPU, src/ray_trace_globals.rs:11-24, and
 * the compile-time schedule constants of src/lib.rs:25-26 and
 * src/ray_trace_node.rs:213).
 *   width, height : full image size (pixel/seed addressing is always global)
 *   spp           : samples per pixel; sample s uses globals.frame = frame0+s
 *   max_depth     : number of (intersect, shade) iterations D (reference: 3);
 *                   a hit at bounce D-1 is killed black (shade.wgsl:236)
 *   frame0        : frame index of sample 0 (the RNG seed input)
 *   row_block, shard_count, shard_index :
 *                   row tiling for multi-GPU. Rows are grouped in blocks of
 *                   row_block rows, dealt to the K = shard_count shards in
 *                   groups of K, serpentine: in group g = b / K, block b goes
 *                   to shard b % K (g even) or K-1 - b % K (g odd), so a
 *                   top-to-bottom cost trend cancels between shards. The
 *                   output of a call holds only the owned rows, in increasing
 *                   y, packed. shard_count = 1 -> whole image.
 *   flags         : RT_FLAG_* bits.                                          */
typedef struct rt_params {
    uint32_t width;
    uint32_t height;
    uint32_t spp;
    uint32_t max_depth;
    uint32_t frame0;
    uint32_t row_block;
    uint32_t shard_count;
    uint32_t shard_index;
    uint32_t flags;
    uint32_t _reserved[3];
} rt_params;

/* Sample accumulation order (part of the result definition, not a tuning
 * knob): the S per-sample colours of a pixel are summed in f32 sequentially
 * inside blocks of RT_SAMPLE_BLOCK consecutive samples; the block sums are
 * folded in f32 in block order; the pixel is that sum / f32(S)
 * (collect.wgsl:114-122 generalised to S > 1). */
#define RT_SAMPLE_BLOCK 8

/* flags */
#define RT_FLAG_NO_PRIMARY_CACHE 0x1u  /* trace the primary ray for every sample
                                          (off by default: the primary ray is
                                          pixel-only, Appendix B Q1/Q3, so its
                                          hit is reused across the samples of a
                                          sample block; results are identical) */

/* Opt-in camera sampling: the reference's thin_lens_ray
 * (generate.wgsl:85-107) is called with lens_offset = (0, 0) and integer
 * pixel coordinates (generate.wgsl:117-121), so both are latent. These flags
 * turn them on; they change the image, so they are off by default, and they
 * disable the primary-hit reuse (the primary ray then varies per sample).
 * For pixel (x, y) and seed frame f, with idx = x + W*y + W*H*f (u32 wrap,
 * the shade seed's index, shade.wgsl:216-218):
 *   RT_FLAG_JITTER    : j = hash3(idx * RT_JITTER_HASH_MUL);
 *                       pixel = (x + (j.x - 0.5), y + (j.y - 0.5))
 *   RT_FLAG_THIN_LENS : l = hash3(idx * RT_LENS_HASH_MUL);
 *                       lens_offset = (2*PI * l.x, l.y), then thin_lens_ray
 *                       verbatim: theta = lens_offset.x + 2*PI, radius =
 *                       lens_offset.y, (u, v) = (cos, sin)(theta) * sqrt(radius),
 *                       origin = (1,0,0)*(u*coc) + (0,1,0)*(v*coc),
 *                       coc = lens_focal_length / (2 * fstop),
 *                       dir = normalize(focus_point - origin).
 * cos/sin are this library's rt_sincos (Cody-Waite reduction by pi/2, Taylor
 * polynomials of degree 9 / 10, plain f32 ops; |error| < 2e-7), restated
 * identically by the oracle -- the WGSL leaves them to the driver. */
#define RT_FLAG_JITTER    0x2u
#define RT_FLAG_THIN_LENS 0x4u
/* RT_FLAG_CULL: trace against the culled list -- the spheres permuted into
 * spatial groups of 8 with a conservative bounding sphere per group, so a
 * wave filters only the groups near some lane's ray. Hits,
 * segment counts and images are identical to the brute-force walk of
 * intersect.wgsl:133-143 (ties still go to the lower sphere index); only the
 * work differs, so it is opt-in like the other non-reference modes. */
#define RT_FLAG_CULL      0x8u
/* RT_FLAG_VALU_FILTER: run the brute-force walk's conservative sphere filter
 * as packed fp32 FMAs on the vector ALUs instead of the default f16 hi/lo
 * tiles on the matrix cores (the matrix-core filter is used
 * whenever the scene fits its range). Both filters only decide which spheres
 * get the reference's exact test, so hits, segment counts and images are
 * identical; the flag exists for A/B timing and for checking one filter
 * against the other (rt_render*, rt_intersect_ex). */
#define RT_FLAG_VALU_FILTER 0x10u
/* RT_FLAG_IMAGE_OUT (device-output calls: rt_render_device,
 * rt_render_frames_device): the output pointer addresses whole images --
 * frame i at out + i*width*height pixels -- and the call writes the rows it
 * owns at their image rows (y*width + x), leaving the other rows untouched,
 * instead of its rows packed. N row shards of one frame then write one image:
 * e.g. rank 0's buffer mapped into every rank (hipIpcOpenMemHandle), so the
 * row tiling needs no gather. The reference has no
 * counterpart (one device, ray_trace_node.rs:213-224). Visibility: the image
 * rows are written with system-scope write-through stores that every writing
 * wave waits on before it ends (nothing is left in its L2), so once the host has seen the call
 * complete (rt_wait / a stream sync, then e.g. a process barrier) the device
 * that owns the image reads them after rt_acquire(). */
#define RT_FLAG_IMAGE_OUT 0x20u
#define RT_JITTER_HASH_MUL 0x9E3779B1u
#define RT_LENS_HASH_MUL   0x85EBCA77u

/* Per-call statistics. */
typedef struct rt_stats {
    uint64_t segments;         /* algorithmic ray segments = intersect_world calls
                                  on live rays (intersect.wgsl:154-158)          */
    uint64_t traced_segments;  /* segments actually intersected on the GPU       */
    uint64_t sphere_tests;     /* traced_segments * sphere_count                  */
    uint64_t paths;            /* pixels * spp                                    */
    double   kernel_ms;        /* sum of render-kernel durations (HIP events)     */
    double   total_ms;         /* whole call incl. collect / copies               */
    uint32_t kernel_launches;  /* number of render-kernel launches                */
    uint32_t short_math;       /* 1: the scene lies inside the domain of the exact
                                  sphere test's short correctly-rounded sqrt and
                                  divide, which waves whose rays do too then use;
                                  0: IEEE operations only. Same bits either way. */
    double   clock_ghz;        /* shader clock the render kernels ran at, averaged
                                  over their waves' lifetimes: sum of the waves'
                                  s_memtime deltas / sum of their s_memrealtime
                                  deltas x 0.1 GHz (the SIMD-issue roofline's peak
                                  is 1024 SIMDs x this clock)                    */
} rt_stats;

typedef struct rt_ctx rt_ctx;

/* Library / ABI version (RT_ABI_VERSION). */
int rt_version(void);

/* Number of rows owned by a shard (see rt_params). Pure host arithmetic. */
uint32_t rt_shard_rows(uint32_t height, uint32_t row_block,
                       uint32_t shard_count, uint32_t shard_index);

/* Create a context on HIP device `device` (replaces RayTracePlugin::build +
 * RayTracePipeline::from_world, src/plugin.rs:25-47, ray_trace_pipeline.rs:171-211). */
int rt_create(int device, rt_ctx** out_ctx);
void rt_destroy(rt_ctx* ctx);

/* Upload the scene (replaces sphere.rs:180-197 and ray_trace_materials.rs:129-164).
 * Arrays are borrowed and copied during the call. Sphere order = list order =
 * tie-break order of intersect_world (intersect.wgsl:135-139). n may be 0.
 * If it fails after validation (e.g. RT_ERR_OUT_OF_MEMORY), the context has
 * no scene until the next successful call (renders return RT_ERR_NO_SCENE). */
int rt_set_scene(rt_ctx* ctx, const rt_sphere* spheres, uint32_t n,
                 const rt_material* materials, uint32_t m);

/* Incremental scene edits (SURVEY §8f "persistent scene + dirty tracking";
 * the reference re-uploads the whole list every frame, sphere.rs:180-197, and
 * the materials when their count changes, ray_trace_materials.rs:129-164).
 * Replace records [first, first+count) of the current scene; counts N and M
 * are unchanged. Only the touched sphere records and 8-sphere groups are
 * re-packed and uploaded. The matrix-core filter's layout follows at the next
 * call that walks it (a caller that renders only the culled list never pays
 * for it): a moved sphere that keeps its radius and stays near its 32-sphere
 * block's box, with the features' scale unchanged, is moved in place -- its
 * f16 row, its half-block's and chunk's bound rows and its records, O(moved +
 * blocks) on the host (13 us at 10,000 and 60,000 spheres), a few KB uploaded;
 * otherwise the layout is rebuilt (scale, k-d spatial order O(N log N), 64 B
 * per sphere uploaded; buffers sized for the worst-case order, so neither path
 * allocates). The culled list (RT_FLAG_CULL), which depends on every sphere,
 * is rebuilt at the next culled call. rt_update_materials rebuilds the
 * shading records only (both orders, O(N), 32 B per sphere): no geometry. */
int rt_update_spheres(rt_ctx* ctx, uint32_t first, const rt_sphere* spheres, uint32_t count);
int rt_update_materials(rt_ctx* ctx, uint32_t first, const rt_material* materials,
                        uint32_t count);

/* Render one frame (replaces RayTraceNode::run, src/ray_trace_node.rs:195-224).
 * Synchronous. out_rgba: caller-owned HOST buffer of
 * rt_shard_rows(...) * width * 4 floats (Rgba32Float, row-major, alpha 1,
 * linear; collect.wgsl:122). stats may be NULL. */
int rt_render(rt_ctx* ctx, const rt_camera* camera, const rt_params* params,
              float* out_rgba, rt_stats* stats);

/* Frames in flight: up to RT_MAX_PENDING rt_render_device / rt_render_async
 * calls may be pending on one ctx. Each pending frame owns a slot of work
 * buffers and (when no stream is given) its own stream, so the next frame's
 * waves start on CUs the previous frame's last waves have released.
 * rt_wait() completes the OLDEST pending frame. rt_render,
 * rt_render_progressive and rt_intersect require no pending frame. */
#define RT_MAX_PENDING 2

/* Same, but the output is a DEVICE pointer on this ctx's device and the work
 * is enqueued on `stream` (hipStream_t, NULL = the frame slot's own stream).
 * Returns after enqueueing; call rt_wait() before reading stats. */
int rt_render_device(rt_ctx* ctx, const rt_camera* camera, const rt_params* params,
                     float* out_rgba_device, void* stream);

/* Several frames of one camera in ONE persistent launch (an animation's or a
 * progressive viewer's consecutive frames; the reference renders one frame
 * per RayTraceNode::run, src/ray_trace_node.rs:195-224, with globals.frame
 * advancing per frame, src/ray_trace_globals.rs:56-68). Frame i renders
 * samples frame0 + i*spp ... frame0 + i*spp + spp - 1 (bit-identical to
 * rt_render_device with frame0 + i*spp) into the DEVICE buffer
 * out_rgba_device + i * rt_shard_rows(...) * width * 4. The frames' work
 * items share one queue, so only the launch (not every frame) pays the drain
 * of its last waves. Same pending/stream rules as rt_render_device. */
int rt_render_frames_device(rt_ctx* ctx, const rt_camera* camera, const rt_params* params,
                            uint32_t nframes, float* out_rgba_device, void* stream);

/* Allocate, up front, the device work buffers (block sums, pixel table,
 * counters) that rt_render_frames_device(params, nframes) needs, in every
 * frames-in-flight slot, without rendering -- the analogue of the reference
 * sizing its ray / intersection buffers in its prepare systems
 * (src/ray_trace_rays.rs:50-66) rather than inside RayTraceNode::run -- and
 * the one-frame host-output staging of rt_render / rt_render_async. Renders
 * of that size or smaller then allocate nothing. No call may be pending. */
int rt_reserve(rt_ctx* ctx, const rt_params* params, uint32_t nframes);

/* Asynchronous host-output variant: enqueue, return; rt_wait() completes the
 * device->host copy into out_rgba and fills stats. Into pageable memory the
 * HIP runtime stages the copy and this call returns only once the frame has
 * been copied; into a buffer given to rt_host_register it returns at once. */
int rt_render_async(rt_ctx* ctx, const rt_camera* camera, const rt_params* params,
                    float* out_rgba);
int rt_wait(rt_ctx* ctx, rt_stats* stats);

/* Page-lock a host buffer that rt_render_async writes (the Bevy shim's two
 * frame buffers), so the frame's device->host copy is a DMA straight into it
 * and rt_render_async does not wait for the frame (measured: a 1080p frame
 * blocks the pageable call for its whole 1.3 ms, the registered one for
 * 0.03 ms, profiles/r03_bench_reference1080.json). No reference counterpart:
 * the reference's frame stays on the GPU as the wgpu texture
 * (src/ray_trace_output.rs:41-61); the drop-in path hands it to Bevy through
 * the host. The buffer must stay allocated until rt_host_unregister(ptr) or
 * rt_destroy. Registering an already registered pointer is an error;
 * rt_host_unregister waits for pending frames first. */
int rt_host_register(rt_ctx* ctx, void* ptr, size_t bytes);
int rt_host_unregister(rt_ctx* ctx, void* ptr);

/* Closest-hit query for a batch of rays against the current scene: the same
 * intersect_world code path the renderer traces with (intersect.wgsl:133-143).
 * rays: n x 6 floats (origin xyz, direction xyz), HOST memory. Outputs (host):
 * hit_index[i] = sphere index or -1 (miss), hit_t[i] = t (1e20 on a miss).
 * Synchronous. Used for picking and for the intersection parity tests. */
int rt_intersect(rt_ctx* ctx, const float* rays, uint32_t n, int32_t* hit_index, float* hit_t);

/* rt_intersect with flags: RT_FLAG_CULL traces the culled list (same hits). */
int rt_intersect_ex(rt_ctx* ctx, const float* rays, uint32_t n, uint32_t flags,
                    int32_t* hit_index, float* hit_t);

/* Progressive accumulation: the reference shows independent
 * 1-spp frames (collect.wgsl:115-125, no history). Here a running per-pixel sum
 * stays on the device across calls: each call renders params->spp new samples
 * (frames frame0 .. frame0+spp-1; callers advance frame0 by spp per call),
 * folds the call's sum into the running sum (sum_new = sum_old + call_sum, f32)
 * and writes out_rgba (HOST) = running sum / total samples. reset != 0 (or a
 * different image geometry) restarts the sum. Synchronous. *total_spp (may be
 * NULL) receives the samples accumulated so far. */
int rt_render_progressive(rt_ctx* ctx, const rt_camera* camera, const rt_params* params,
                          int reset, float* out_rgba, uint64_t* total_spp);

/* Display encode of an Rgba32Float image: sRGB transfer curve (IEC 61966-2-1),
 * channels clamped to [0,1], NaN -> 0, alpha 255, RGBA8. DEVICE buffers,
 * enqueued on `stream` (NULL = ctx stream, synchronous). */
int rt_encode_srgb8(rt_ctx* ctx, const float* rgba_device, uint8_t* rgba8_device, uint64_t npix,
                    void* stream);

/* Re-assemble gathered shard outputs into the full image on the device:
 * gathered = shard_count consecutive slabs of max_rows*width*4 floats (slab k =
 * shard k's output, padded to max_rows rows); image = height*width*4 floats. */
int rt_assemble_shards(rt_ctx* ctx, const float* gathered_device, uint32_t max_rows,
                       float* image_device, uint32_t width, uint32_t height,
                       uint32_t row_block, uint32_t shard_count, void* stream);

/* The same for `frames` (1..65535) consecutive frames in one launch, in the
 * layout one gather of the shards' multi-frame launches lands: gathered =
 * shard_count slabs of frames*max_rows*width*4 floats (slab k = shard k's
 * frames in order, each padded to max_rows rows); image = frames*height*
 * width*4 floats. rt_assemble_shards is frames = 1. */
int rt_assemble_shard_frames(rt_ctx* ctx, const float* gathered_device, uint32_t max_rows,
                             uint32_t frames, float* image_device, uint32_t width,
                             uint32_t height, uint32_t row_block, uint32_t shard_count,
                             void* stream);

/* System-scope acquire on the ctx's device, enqueued on `stream` (NULL = ctx
 * stream, synchronous): work enqueued after it on that stream reads what OTHER
 * devices wrote into this device's memory (RT_FLAG_IMAGE_OUT rows of other
 * ranks, written through a hipIpcOpenMemHandle mapping) once the host has
 * seen those writers' calls complete. Row-tiled multi-GPU rendering only
 * (DESIGN.md §7); the reference renders on one device. */
int rt_acquire(rt_ctx* ctx, void* stream);

/* Message for the last failing call on ctx (or on the library when ctx is NULL). */
const char* rt_last_error(const rt_ctx* ctx);

#ifdef __cplusplus
}
#endif

#endif /* RT_HIP_H */
