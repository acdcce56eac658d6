// rt_api.cpp — the C-ABI (include/rt_hip.h) over the gfx950 kernels.
//
// Replaces the reference's host-side schedule: RayTracePlugin::build and
// RayTracePipeline::from_world (src/plugin.rs:25-47, src/ray_trace_pipeline.rs
// :171-211) become rt_create; the per-frame `prepare` uploads
// (src/ray_trace_camera.rs:43-68, src/ray_trace_globals.rs:56-68,
// src/sphere.rs:180-197, src/ray_trace_materials.rs:129-164) become
// rt_set_scene + the by-value kernel parameters; RayTraceNode::run
// (src/ray_trace_node.rs:195-224) becomes rt_render*.
//
// Per call: memset the work/segment counters, then per sample-block pass one
// persistent render launch + one collect launch (a single pass unless the
// block-sum scratch would exceed the scratch_bytes budget, 16 GiB), timed with HIP events on
// the stream they run on.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <ctime>
#include <string>
#include <functional>
#include <vector>

#include "rt_internal.h"

namespace {

thread_local std::string g_err;  // errors with no context

struct Pass {
    uint32_t frame_begin, nframes;   // frames of the launch
    uint32_t block_begin, nblocks;   // sample blocks of each frame in the launch
};

}  // namespace

// Per-frame work buffers (one set per frame in flight).
struct Frame {
    hipStream_t stream = nullptr;   // the slot's own stream (used when the caller gives none)
    float4* d_block_sums = nullptr;
    size_t bs_cap = 0;
    float4* d_acc = nullptr;
    size_t acc_cap = 0;
    float4* d_pd = nullptr;         // pixel table (rt_primary_kernel), 32 B per pixel
    size_t pd_cap = 0;
    float4* d_out = nullptr;        // host-output path staging
    size_t out_cap = 0;
    uint32_t* d_counters = nullptr; // [0..3] 2 x u64 segment counters, [4..] per-pass work counters
    size_t counters_cap = 0;        // in u32 words
    unsigned long long* h_segs = nullptr;  // pinned, RT_CNT_U64 counters
    std::vector<hipEvent_t> ev;     // 2 per pass
    hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;
    // the pending call in this slot
    hipStream_t pending_stream = nullptr;
    uint32_t passes = 0;
    uint64_t paths = 0;
    uint32_t short_math = 0;        // KParams.scene_fast of the call
};

// A/B and fault-injection knobs of one context (rt_debug_tune, internal). The
// defaults ARE the product: nothing reads the environment, so a stray
// variable in a host application cannot change the schedule. Every setting
// gives the same bits (tested); they exist for the measurements in DESIGN.md.
struct Tuning {
    size_t scratch_bytes = (size_t)16 << 30;  // block sums per launch (of 288 GB HBM)
    bool split_all = false;       // without primary reuse, every block as single samples
    // 1- / 2-sample tail items at the end of a launch: 1 on, 0 off, -1 by the
    // call (enqueue: off where the whole last pair of every pixel, which the
    // tail region rounds up to, is more than 4x the samples it is meant for)
    int32_t tail_split = -1;
    // tail regions (4-, 2-, 1-sample items) x D x lanes. Round 5: 0, 1, 0.5
    // against 0, 1, 1 (profiles/r05/tail/): headline -0.18 %, 10k spheres
    // -1.9 %, 4K -0.1 %, the N = 4 / 2 row shards -0.75 / -0.2 %
    double tail[3] = {0.0, 1.0, 0.5};
    double block_region = -1.0;   // single-block items before the tail, x D x lanes samples (-1: by spp / D)
    bool block_align = true;      // the pixel region ends at a frame boundary (block_pairs)
    // lead items: every frame past the pixel region starts with one pixel item
    // of its first block_lead blocks (one slot instead of block_lead); 0 = off,
    // -1 = by the call (regions below)
    int32_t block_lead = -1;
    // KParams::item_order: pixel-major block / tail items (bit 0) and pixel
    // items (bit 1): a wave's lanes then share pixels, so its primary rays
    // (and first-bounce origins) coincide -- warm 20-frame launches, one box
    // (profiles/r03/item_order/): full frame 243.7 -> 240.2 ms, N=8 shard
    // 34.9 -> 33.5 ms; 1 alone 242.6 / 33.5, 2 alone 241.0 / 35.4
    // bit 2 (round 5): grouped by pix_group = 4 neighbouring pixels, so
    // a wave's slot and output stores are whole 64-B pieces of lines its own
    // XCD's L2 merges: render-kernel writes per headline launch 2.41 ->
    // 1.74 GB at the same time (groups of 8: 1.73 GB but +0.4 % time, the
    // rays of 8 pixels per wave less coherent), profiles/r05/item_order/
    uint32_t item_order = 7;
    uint32_t pix_group = 4;       // item_order bit 2: pixels per group (4 or 8)
    bool prefetch = true;         // waves prefetch their next work chunk
    int32_t prio_mode = -1;       // s_setprio rotation: 0 off, 1 by iteration, 3 by wall time (-1: by the call)
    int32_t wave_chunk = -1;      // work items per atomic before the launch's tail (-1: RT_WAVE_CHUNK)
    uint32_t prio_shift = 14;     // mode 3 step: 2^prio_shift ticks of 10 ns
    uint32_t wg_per_cu = 0;       // resident workgroups per CU (0 = by the call's size, enqueue)
    int64_t wide_max = -1;        // sphere-parallel threshold (-1 = cost model)
    bool fast_exact = true;       // short correctly-rounded exact test when in domain
    int64_t fail_alloc_after = -1;  // fault injection: device allocations left (-1 = off)
    // positive control of the checked build: the bound of one RT_IDX site
    // (4 sph, 5 shading records, 7 slots, 16 output) given as 0, so its first index is
    // reported (the product build reads no bound: no effect)
    uint32_t chk_shrink = 0;
    // whole items write their output pixel themselves (KParams::dout); off:
    // every frame through the slots and rt_collect_kernel (same bits)
    bool direct_out = true;
    // the matrix-core walk skips the 32-sphere blocks whose bound no ray of
    // the half-wave passes (MfScene::B); off: every block (same bits)
    bool mf_cull = true;
    // lists of 2..32 bound chunks test the chunk-level bounds first
    // (MfScene::top); off: every chunk's block bounds (same bits)
    bool mf_top = true;
    // RT_FLAG_IMAGE_OUT: a system-scope release (buffer_wbl2 sc0 sc1) per
    // collect wave after its write-through stores. Off (the product): every
    // byte of the hand-off is stored sc0 sc1 (write-through, nothing dirty
    // left in this device's L2) and drained by s_waitcnt vmcnt(0), the
    // producer form MI355X_MICROARCH.md lists beside the release when the
    // consumer acquires (rt_acquire). The per-wave write-back of the L2 cost
    // an N = 8 shard's 20-frame call 2.3 ms (2.51 -> 0.18 ms beyond the
    // render, profiles/r05/split/); on: A/B only.
    bool dsys_release = false;
    // fault injection (bench.py --debug-skip-collect-rank): the call writes no
    // output at all -- no direct output, no collect -- so the frame's pixels
    // keep whatever the buffer held, the stale rows a lost hand-off would
    // leave; the N>1 cross-rank check must catch them. Not a same-bits knob.
    bool skip_collect = false;
};

// The matrix-core walk's scene on the host -- exactly what its device buffers
// hold (build_mfma fills it from a spatial order; mf_update keeps it current
// for moved spheres without a new order).
struct MfHost {
    bool ok = false;
    int sq = 0;                    // quadratic features scaled by 2^-sq
    uint32_t nblk = 0, npos = 0, nchunk = 0;
    bool top = false;              // a chunk-level bound chunk follows the block bounds
    std::vector<uint32_t> order;   // walk position -> original index (0xFFFFFFFF: pad), npos
    std::vector<uint16_t> A;       // A fragments, RT_MF_BLK uint4 per 32-sphere block
    std::vector<uint16_t> B;       // bound chunks (+ the chunk-level one), RT_MF_BCHUNK uint4 each
    std::vector<float4> msph;      // (cx, cy, cz, r^2) in walk order (pads r^2 = -inf)
    std::vector<uint32_t> mperm;   // walk position -> original index (pads 0)
    std::vector<uint32_t> iperm;   // original index -> walk position
    std::vector<double> bqmax;     // per block max_i max_a c_a^2 of its members (the scale's input)
};

struct rt_ctx {
    int device = 0;
    std::string err;
    int cu_count = 0;
    int blocks_per_cu = 0;          // resident workgroups per CU, brute-force kernel
    int blocks_per_cu_c = 0;        // ... culled kernel
    Tuning tune;
    uint64_t allocs = 0;            // device allocations made (rt_debug_alloc_count)

    // scene
    bool has_scene = false;
    bool cull_dirty = true;         // the culled list is rebuilt at the next RT_FLAG_CULL call
    bool scene_fast = false;  // scene_fast_ok(): the exact tests may take the short divide/sqrt
    uint32_t n = 0, ngroups = 0, m = 0;
    float4* d_grp = nullptr;        // groups of RT_GROUP=8 spheres, SoA (cx[8], cy[8], cz[8], S[8])
    float4* d_sph = nullptr;        // (cx, cy, cz, r*r)
    // per-sphere shading record, 2 float4: (radius, reflectance bits,
    // fuzziness, index of refraction), (material colour) -- the sphere's
    // radius and its material in one place, so shading issues its loads
    // together (no sphere -> material index -> material chain)
    float4* d_shd = nullptr;
    size_t grp_cap = 0, sph_cap = 0, shd_cap = 0;
    std::vector<float4> h_sph, h_grp;  // host mirrors of the packed scene
    std::vector<float> h_S;
    std::vector<float2> h_rm;
    std::vector<rt_material> h_mats;
    // culled list (RT_FLAG_CULL, build_cull): the records permuted into spatial
    // groups, clusters of 8 groups, the group bounds and the permutation
    uint32_t n_c = 0, ngroups_c = 0, nclusters_c = 0;
    float4* d_grp_c = nullptr;
    float4* d_sph_c = nullptr;
    float4* d_shd_c = nullptr;      // shading records in the culled order
    float4* d_bnd_c = nullptr;
    uint32_t* d_perm_c = nullptr;
    size_t grp_c_cap = 0, sph_c_cap = 0, shd_c_cap = 0, bnd_c_cap = 0, perm_c_cap = 0;
    // (radius, material bits) in the culled order, kept so that a material
    // update rebuilds only d_shd_c (the geometry does not move)
    std::vector<float2> h_rm_c;
    // matrix-core filter (RT_MFMA_FILTER builds, build_mfma): f16 A fragments
    bool mf_ok = false;
    bool mf_dirty = false;          // rt_update_spheres: fragments rebuilt by mfma_ready
    uint32_t mf_nblk = 0;
    bool mf_top = false;  // a chunk-level bound chunk follows the block bounds (build_mfma)
    float mf_qs = 1.0f;   // 2^sq: the ray side's scale of the quadratic features
    float mf_abs = 0.0f;  // absolute margin of the threshold, 2^(sq - 20)
    uint4* d_mfA = nullptr;
    size_t mfA_cap = 0;
    // the walk's spatial order (cull_layout's): block-bound fragments, the
    // records the drain reads, and the walk position -> original index map
    uint4* d_mfB = nullptr;
    float4* d_mf_sph = nullptr;
    uint32_t* d_mf_perm = nullptr;
    size_t mfB_cap = 0, mf_sph_cap = 0, mf_perm_cap = 0;
    // the shading records in the walk's order (2 float4 per walk position;
    // the render shades by walk position, rt_dev_path.h) and original index
    // -> walk position (the VALU and sphere-parallel walks' answers)
    float4* d_mf_shd = nullptr;
    uint32_t* d_mf_iperm = nullptr;
    size_t mf_shd_cap = 0, mf_iperm_cap = 0;
    MfHost mfh;                     // the matrix-core walk's host mirror (build_mfma)
    // spheres rt_update_spheres changed since the layout was built (flags by
    // original index, and the list): mfma_ready moves them into the layout
    // in place when it can (mf_update), else rebuilds it
    std::vector<uint8_t> mf_moved_flag;
    std::vector<uint32_t> mf_moved;
    uint64_t mf_builds = 0, mf_inplace = 0;  // layouts built whole / updated in place

    // frames in flight: RT_MAX_PENDING slots of per-frame work buffers, each
    // with its own stream, so frame i+1 can start while frame i drains
    Frame fr[RT_MAX_PENDING];
    uint32_t head = 0;      // oldest pending slot
    uint32_t npending = 0;  // frames enqueued and not yet waited for
    hipStream_t stream = nullptr;  // = fr[0].stream: scene uploads, intersect, progressive
    unsigned long long dbg[RT_DBG_COUNTERS] = {};  // diagnostic counters of the last waited frame
    // the last rt_intersect's matrix-core walk: (block, half) tiles walked,
    // and tiles without block bounds (rt_debug_intersect_tiles)
    unsigned long long isect_tiles[2] = {};

    struct HostReg {
        void* ptr;
        size_t bytes;
    };
    std::vector<HostReg> host_regs;  // rt_host_register'd buffers

    float4* d_prog = nullptr;       // progressive running sum (rt_render_progressive)
    size_t prog_cap = 0;
    uint64_t prog_total = 0;        // samples accumulated so far
    uint64_t prog_key = 0;          // geometry the running sum belongs to
};

static int fail(rt_ctx* ctx, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
static int fail(rt_ctx* ctx, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (ctx)
        ctx->err = buf;
    else
        g_err = buf;
    return code;
}

#define HIP_TRY(ctx, call)                                                                     \
    do {                                                                                       \
        hipError_t e_ = (call);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail((ctx), e_ == hipErrorOutOfMemory ? RT_ERR_OUT_OF_MEMORY : RT_ERR_DEVICE, \
                        "%s failed: %s", #call, hipGetErrorString(e_));                        \
    } while (0)

template <typename T>
static int ensure(rt_ctx* ctx, T** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap && *p) return RT_OK;
    if (*p) {
        hipFree(*p);
        *p = nullptr;
        *cap = 0;
    }
    if (bytes == 0) return RT_OK;
    if (ctx->tune.fail_alloc_after == 0)
        return fail(ctx, RT_ERR_OUT_OF_MEMORY, "hipMalloc(%zu) failed: injected (rt_debug_tune)",
                    bytes);
    if (ctx->tune.fail_alloc_after > 0) --ctx->tune.fail_alloc_after;
    HIP_TRY(ctx, hipMalloc((void**)p, bytes));
    *cap = bytes;
    ++ctx->allocs;
    return RT_OK;
}

// Granlund-Montgomery constants for FastDiv (rt_internal.h).
static FastDiv make_fastdiv(uint32_t d) {
    FastDiv f{};
    f.d = d;
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) ++l;  // l = ceil(log2 d)
    f.m = (uint32_t)((((1ull << l) - d) << 32) / d + 1);
    f.sh1 = l < 1 ? l : 1;
    f.sh2 = l > 1 ? l - 1 : 0;
    return f;
}

// One knob of rt_debug_tune: name -> field. Returns false for an unknown name
// or a malformed value (the knob is left unchanged).
static bool tune_set(Tuning& t, const char* name, const char* v) {
    char* end = nullptr;
    auto num = [&](double& out) {
        out = strtod(v, &end);
        return end != v && *end == '\0';
    };
    double x = 0.0;
    if (!strcmp(name, "tail")) {
        double w[3];
        if (sscanf(v, "%lf,%lf,%lf", &w[0], &w[1], &w[2]) != 3 || w[0] < 0 || w[1] < 0 || w[2] < 0)
            return false;
        for (int i = 0; i < 3; ++i) t.tail[i] = w[i];
        return true;
    }
    if (!num(x)) return false;
    if (!strcmp(name, "scratch_bytes")) {
        if (x < 16) return false;
        t.scratch_bytes = (size_t)x;
    } else if (!strcmp(name, "split_all")) {
        t.split_all = x != 0;
    } else if (!strcmp(name, "tail_split")) {
        if (x != -1 && x != 0 && x != 1) return false;
        t.tail_split = (int32_t)x;
    } else if (!strcmp(name, "item_order")) {
        if (x < 0 || x > 7) return false;
        t.item_order = (uint32_t)x;
    } else if (!strcmp(name, "pix_group")) {
        if (x != 4 && x != 8) return false;
        t.pix_group = (uint32_t)x;
    } else if (!strcmp(name, "block_align")) {
        t.block_align = x != 0;
    } else if (!strcmp(name, "block_lead")) {
        if (x < -1 || x > 64) return false;
        t.block_lead = (int32_t)x;
    } else if (!strcmp(name, "block_region")) {
        if (x < 0) return false;
        t.block_region = x;
    } else if (!strcmp(name, "prefetch")) {
        t.prefetch = x != 0;
    } else if (!strcmp(name, "wave_chunk")) {
        if (x != -1 && (x < 16 || x > 1024)) return false;
        t.wave_chunk = (int32_t)x;
    } else if (!strcmp(name, "prio_mode")) {
        t.prio_mode = (int32_t)x;
    } else if (!strcmp(name, "prio_shift")) {
        t.prio_shift = (uint32_t)x;
    } else if (!strcmp(name, "wg_per_cu")) {
        t.wg_per_cu = (uint32_t)x;
    } else if (!strcmp(name, "wide_max")) {
        t.wide_max = (int64_t)x;
    } else if (!strcmp(name, "fast_exact")) {
        t.fast_exact = x != 0;
    } else if (!strcmp(name, "fail_alloc_after")) {
        t.fail_alloc_after = (int64_t)x;
    } else if (!strcmp(name, "direct_out")) {
        t.direct_out = x != 0;
    } else if (!strcmp(name, "mf_cull")) {
        t.mf_cull = x != 0;
    } else if (!strcmp(name, "mf_top")) {
        t.mf_top = x != 0;
    } else if (!strcmp(name, "dsys_release")) {
        t.dsys_release = x != 0;
    } else if (!strcmp(name, "skip_collect")) {
        t.skip_collect = x != 0;
    } else if (!strcmp(name, "chk_shrink")) {
        if (x != 0 && x != 4 && x != 5 && x != 7 && x != 16) return false;
        t.chk_shrink = (uint32_t)x;
    } else {
        return false;
    }
    return true;
}

extern "C" {

int rt_version(void) { return RT_ABI_VERSION; }

uint32_t rt_shard_rows(uint32_t height, uint32_t row_block, uint32_t shard_count,
                       uint32_t shard_index) {
    if (row_block == 0) row_block = 1;
    if (shard_count == 0) shard_count = 1;
    if (shard_index >= shard_count) return 0;
    uint32_t rows = 0;
    const uint32_t nblk = (height + row_block - 1) / row_block;
    for (uint32_t b = 0; b < nblk; ++b) {
        if (rt_block_owner(b, shard_count) != shard_index) continue;
        const uint32_t y0 = b * row_block;
        const uint32_t y1 = y0 + row_block < height ? y0 + row_block : height;
        rows += y1 - y0;
    }
    return rows;
}

int rt_create(int device, rt_ctx** out_ctx) {
    if (!out_ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_create: out_ctx is NULL");
    *out_ctx = nullptr;
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0)
        return fail(nullptr, RT_ERR_DEVICE, "rt_create: no HIP device (%s)",
                    e != hipSuccess ? hipGetErrorString(e) : "count 0");
    if (device < 0 || device >= ndev)
        return fail(nullptr, RT_ERR_INVALID_ARG, "rt_create: device %d out of range [0,%d)",
                    device, ndev);
    rt_ctx* ctx = new rt_ctx();
    ctx->device = device;
    int rc = RT_OK;
    do {
        if ((e = hipSetDevice(device)) != hipSuccess) break;
        if ((e = hipDeviceGetAttribute(&ctx->cu_count, hipDeviceAttributeMultiprocessorCount,
                                       device)) != hipSuccess)
            break;
        if ((e = rt_render_occupancy(&ctx->blocks_per_cu, &ctx->blocks_per_cu_c)) != hipSuccess) break;
        for (Frame& f : ctx->fr) {
            if ((e = hipStreamCreateWithFlags(&f.stream, hipStreamNonBlocking)) != hipSuccess) break;
            if ((e = hipHostMalloc((void**)&f.h_segs, RT_CNT_U64 * sizeof(unsigned long long))) != hipSuccess)
                break;
            if ((e = hipEventCreate(&f.ev_t0)) != hipSuccess) break;
            if ((e = hipEventCreate(&f.ev_t1)) != hipSuccess) break;
        }
        ctx->stream = ctx->fr[0].stream;
    } while (0);
    if (e != hipSuccess) {
        rc = fail(nullptr, RT_ERR_DEVICE, "rt_create: %s", hipGetErrorString(e));
        rt_destroy(ctx);
        return rc;
    }
    if (ctx->blocks_per_cu < 1) ctx->blocks_per_cu = 1;
    if (ctx->blocks_per_cu_c < 1) ctx->blocks_per_cu_c = 1;
    *out_ctx = ctx;
    return RT_OK;
}

void rt_destroy(rt_ctx* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    for (Frame& f : ctx->fr) {
        if (f.stream) hipStreamSynchronize(f.stream);
        if (f.pending_stream) hipStreamSynchronize(f.pending_stream);
    }
    for (const auto& r : ctx->host_regs) hipHostUnregister(r.ptr);
    hipFree(ctx->d_grp);
    hipFree(ctx->d_sph);
    hipFree(ctx->d_shd);

    hipFree(ctx->d_prog);
    hipFree(ctx->d_grp_c);
    hipFree(ctx->d_sph_c);
    hipFree(ctx->d_shd_c);
    hipFree(ctx->d_bnd_c);
    hipFree(ctx->d_perm_c);
    hipFree(ctx->d_mfA);
    hipFree(ctx->d_mfB);
    hipFree(ctx->d_mf_sph);
    hipFree(ctx->d_mf_perm);
    hipFree(ctx->d_mf_shd);
    hipFree(ctx->d_mf_iperm);
    for (Frame& f : ctx->fr) {
        hipFree(f.d_block_sums);
        hipFree(f.d_acc);
        hipFree(f.d_out);
        hipFree(f.d_pd);
        hipFree(f.d_counters);
        if (f.h_segs) hipHostFree(f.h_segs);
        for (hipEvent_t e : f.ev) hipEventDestroy(e);
        if (f.ev_t0) hipEventDestroy(f.ev_t0);
        if (f.ev_t1) hipEventDestroy(f.ev_t1);
        if (f.stream) hipStreamDestroy(f.stream);
    }
    delete ctx;
}

// ---- scene packing --------------------------------------------------------
// Sphere records for the kernel. AoS (cx, cy, cz, r*r) for the exact tests and
// shading; SoA groups of RT_GROUP (cx[8], cy[8], cz[8], S[8]) for the
// wave-uniform filter loop, S = r^2 - (1 - m - mu) |c|^2 rounded once from
// double (DESIGN.md "Exact filter"). Padded to whole groups plus one; pad
// records have r^2 = S = -inf, which the filter never passes. Host mirrors
// are kept so rt_update_* re-packs and uploads only the touched groups.
static void pack_record_to(const rt_sphere& s, float4& q, float& S, float2& rm) {
    const float r = s.radius;
    const float r2 = r * r;  // sqr(s.radius): the f32 value the exact test uses
    q = make_float4(s.center[0], s.center[1], s.center[2], r2);
    const double kS = 1.0 - 0x1p-16 - 0x1p-17;
    const double cx = s.center[0], cy = s.center[1], cz = s.center[2];
    S = (float)((double)r2 - kS * (cx * cx + cy * cy + cz * cz));
    float mbits;
    std::memcpy(&mbits, &s.material, 4);
    rm = make_float2(r, mbits);
}

static void pack_record(rt_ctx* ctx, uint32_t i, const rt_sphere& s) {
    pack_record_to(s, ctx->h_sph[i], ctx->h_S[i], ctx->h_rm[i]);
}

// Shading records of n spheres from their (radius, material bits) and the
// materials (validated: every sphere's index is below mats.size(); a pad
// record's index 0 with no materials gives zeros -- pads are never shaded).
static void shade_records(const float2* rm, size_t n, const std::vector<rt_material>& mats,
                          float4* out) {
    for (size_t i = 0; i < n; ++i) {
        uint32_t mi;
        std::memcpy(&mi, &rm[i].y, 4);
        rt_material m{};
        if (mi < mats.size()) m = mats[mi];
        float refl;
        std::memcpy(&refl, &m.reflectance, 4);
        out[2 * i] = make_float4(rm[i].x, refl, m.fuzziness, m.index_of_refraction);
        out[2 * i + 1] = make_float4(m.color[0], m.color[1], m.color[2], m.color[3]);
    }
}

// Upload the shading records of spheres [first, first + count) (quiesced).
static int upload_shd(rt_ctx* ctx, size_t first, size_t count) {
    if (!count) return RT_OK;
    std::vector<float4> rec(2 * count);
    shade_records(&ctx->h_rm[first], count, ctx->h_mats, rec.data());
    HIP_TRY(ctx, hipMemcpy(ctx->d_shd + 2 * first, rec.data(), sizeof(float4) * rec.size(),
                           hipMemcpyHostToDevice));
    return RT_OK;
}

#ifdef RT_MFMA_FILTER
// The shading records in the matrix-core walk's order (build_mfma; pads zero,
// never shaded), from the host mirrors (quiesced).
static int upload_shd_mf(rt_ctx* ctx) {
    const std::vector<uint32_t>& perm = ctx->mfh.order;
    std::vector<float4> rec(2 * perm.size(), make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (size_t p = 0; p < perm.size(); ++p)
        if (perm[p] != 0xFFFFFFFFu) shade_records(&ctx->h_rm[perm[p]], 1, ctx->h_mats, &rec[2 * p]);
    HIP_TRY(ctx, hipMemcpy(ctx->d_mf_shd, rec.data(), sizeof(float4) * rec.size(), hipMemcpyHostToDevice));
    return RT_OK;
}
#endif

// The exact sphere test's short correctly-rounded sqrt/divide forms (rt_math.h)
// need their operands inside [2^-100, 2^100] / [2^-60, 2^60]. The kernel checks
// the ray side per segment (|origin_i| <= 2^32, |d|^2 in [2^-20, 2^20]); the
// sphere side is checked here once per scene: |centre_i| <= 2^30 and
// r^2 in [2^-40, 2^60]. Then |oc|^2 <= 2^68, |half_b| < 2^46, dis < 2^92 and
// both root numerators < 2^47; and the lower ends need no guard (rt_dev_intersect.h
// exact_body). Any other scene keeps the IEEE operations everywhere.
static bool scene_fast_ok(const rt_ctx* ctx) {
    for (uint32_t i = 0; i < ctx->n; ++i) {
        const float4 q = ctx->h_sph[i];
        if (!(std::fabs(q.x) <= 0x1p30f && std::fabs(q.y) <= 0x1p30f && std::fabs(q.z) <= 0x1p30f))
            return false;
        if (!(q.w >= 0x1p-40f && q.w <= 0x1p60f)) return false;
    }
    return true;
}

static void pack_group_soa(const float4* q, const float* sg, float4* o);
static void pack_group(rt_ctx* ctx, size_t g) {
    pack_group_soa(&ctx->h_sph[RT_GROUP * g], &ctx->h_S[RT_GROUP * g], &ctx->h_grp[RT_GROUP * g]);
}

// ---- culled list (RT_FLAG_CULL) ---------------------------------------------
// The spheres permuted into spatial groups of RT_GROUP (large spheres first, in
// groups of their own; the rest in k-d order of their centres), clusters of
// 8 consecutive groups, supers of 8 clusters, and per group and per cluster a
// bounding sphere (C, R) stored in the group layout -- SoA (Cx[8], Cy[8],
// Cz[8], S_B[8]) per super (its clusters) and per cluster (its groups) -- so
// the kernel runs the same packed filter over the bounds (rt_dev_intersect.h
// intersect_world<true>) and walks only the clusters and groups some lane
// passes, against TB = (1 - m - muB)|o|^2, m = 2^-16, muB = 2^-7. The proof
// below holds for any member set, so for cluster bounds too.
//
// Why a skipped group holds no candidate (all quantities of one lane; exact
// arithmetic unless marked ~). Filter of sphere (c, r): F = hb~^2 + r^2 -
// (1-m)|o-c|^2 + mu(|o|^2+|c|^2), hb~ = dn~.(o-c), dn~ = (1+eta) d/|d| with
// |eta| <= 2^-21 (rsq + products); the computed H~ - T~ is F within
// E = 2^-17 (|o|^2 + |c|^2 + r^2) (the expanded form's rounding, generous;
// operands finite with |o|, |c|, r <= 2^30, so no overflow). A candidate has
// H~ >= T~, so with dist = the true distance of c from the ray's line:
//   dist_i^2 <= r_i^2 (1 + 2^-17) + delta_i,
//   delta_i = 2^-15 (|o - c_i|^2 + |o|^2 + |c_i|^2)      (m + 2^-19, mu + 2^-17 <= 2^-15)
// so dist_i <= r_i (1 + 2^-18) + sqrt(delta_i). The line distance is
// 1-Lipschitz in the point: dist_C <= dist_i + |C - c_i| <= L + sqrt(delta_i)
// with L = max_i (|C - c_i| + r_i (1 + 2^-18)). Then, with 2ab <= a^2/16 + 16 b^2
// and |o - c_i|^2 + |o|^2 + |c_i|^2 <= 6 (|o|^2 + |C|^2) + 4 L^2:
//   dist_C^2 <= (1 + 2^-4) L^2 + 17 delta_i <= (1 + 2^-4 + 2^-8) L^2 + 2^-8 (|o|^2 + |C|^2).
// The bound's filter with R^2 = (1 + 2^-3) L^2 + 2^-60 and S_B = R^2 - (1 - m - muB)|C|^2:
//   F_B = hb~_C^2 + R^2 - (1-m)|o-C|^2 + muB (|o|^2 + |C|^2)
//      >= R^2 - dist_C^2 + (muB - 2^-18)(|o|^2 + |C|^2)
//      >= (2^-4 - 2^-8) L^2 + 2^-60 + (2^-7 - 2^-8 - 2^-18)(|o|^2 + |C|^2),
// which exceeds the bound's own rounding 2^-17 (|o|^2 + |C|^2 + R^2): H~_B >= TB~.
// S_B is rounded up to f32 (a larger S_B only passes more). Groups with a
// non-finite member, a centre component or radius above 2^30 get C = 0,
// S_B = +inf (always pass); empty groups S_B = -inf (never); the kernel walks
// every group for a wave with a lane outside |o_i| <= 2^30, |d|^2 in
// [2^-100, 2^100].
struct CullLayout {
    uint32_t ngroups = 0, nclusters = 0, nsupers = 0, nrec = 0;
    std::vector<uint32_t> perm;  // position -> original index (0xFFFFFFFF = pad)
    std::vector<float4> sph, grp, bnd;
    std::vector<float2> rm;
};

static void pack_group_soa(const float4* q, const float* sg, float4* o) {
    o[0] = make_float4(q[0].x, q[1].x, q[2].x, q[3].x);
    o[1] = make_float4(q[4].x, q[5].x, q[6].x, q[7].x);
    o[2] = make_float4(q[0].y, q[1].y, q[2].y, q[3].y);
    o[3] = make_float4(q[4].y, q[5].y, q[6].y, q[7].y);
    o[4] = make_float4(q[0].z, q[1].z, q[2].z, q[3].z);
    o[5] = make_float4(q[4].z, q[5].z, q[6].z, q[7].z);
    o[6] = make_float4(sg[0], sg[1], sg[2], sg[3]);
    o[7] = make_float4(sg[4], sg[5], sg[6], sg[7]);
}

static float round_up_f32(double v) {
    if (std::isnan(v)) return INFINITY;
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, INFINITY);
    return f;
}

// The spatial order of the list, shared by the culled list (cull_layout) and
// the matrix-core walk (build_mfma): original indices, 0xFFFFFFFF for a pad
// position; its length is a multiple of RT_GROUP. sph: (cx, cy, cz, r*r) f32
// records and S their filter constants, in the original order, n records.
// O(N log N): per k-d level a selection (std::nth_element) of the cut along
// the axis in the total order (centre coordinate, original index), leaves
// sorted in the same order -- deterministic whatever the ties. (Round 4's
// stable sort per level, O(N log^2 N): 36 ms for 10,000 spheres, 168 ms for
// 65,536, on every rt_set_scene / rt_update_spheres.)
static std::vector<uint32_t> spatial_order(const float4* sph, const float* S, uint32_t n) {
    auto finite_rec = [&](uint32_t i) {
        const float4 q = sph[i];
        return std::isfinite(q.x) && std::isfinite(q.y) && std::isfinite(q.z) && std::isfinite(q.w) &&
               std::isfinite(S[i]);
    };
    // large (or non-finite) spheres go first, in groups of their own
    std::vector<double> radii;
    for (uint32_t i = 0; i < n; ++i)
        if (finite_rec(i)) radii.push_back(std::sqrt((double)sph[i].w));
    double thr = INFINITY;
    if (!radii.empty()) {
        std::nth_element(radii.begin(), radii.begin() + radii.size() / 2, radii.end());
        thr = 4.0 * radii[radii.size() / 2];
    }
    std::vector<uint32_t> big, rest;
    for (uint32_t i = 0; i < n; ++i) {
        if (!finite_rec(i) || std::sqrt((double)sph[i].w) > thr) big.push_back(i);
        else rest.push_back(i);
    }
    // the rest in k-d order: split the box's longest axis at a multiple of
    // 64 / 32 / 8 positions near the median (clusters, matrix-core blocks and
    // groups stay whole subtrees), leaves of <= 8 sorted along their longest
    // axis -- compact groups, blocks and clusters (the matrix-core walk's block
    // bounds: radius ~3.8 vs 4-11 in Morton order for RTIOW's small spheres)
    std::vector<uint32_t> kd(rest);
    auto centre = [&](uint32_t i, int a) { return (double)(a == 0 ? sph[i].x : a == 1 ? sph[i].y : sph[i].z); };
    std::function<void(size_t, size_t)> split = [&](size_t b, size_t e) {
        const size_t n2 = e - b;
        if (n2 <= 1) return;
        double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t p = b; p < e; ++p)
            for (int a = 0; a < 3; ++a) {
                blo[a] = std::min(blo[a], centre(kd[p], a));
                bhi[a] = std::max(bhi[a], centre(kd[p], a));
            }
        int ax = 0;
        for (int a = 1; a < 3; ++a)
            if (bhi[a] - blo[a] > bhi[ax] - blo[ax]) ax = a;
        auto less = [&](uint32_t x, uint32_t y) {
            const double cx = centre(x, ax), cy = centre(y, ax);
            return cx < cy || (cx == cy && x < y);
        };
        if (n2 <= RT_GROUP) {  // a leaf: sorted along its longest axis
            std::sort(kd.begin() + b, kd.begin() + e, less);
            return;
        }
        const size_t unit = n2 > 64 ? 64 : (n2 > 32 ? 32 : RT_GROUP);
        size_t cut = std::max(unit, (size_t)std::llround((double)n2 / 2.0 / (double)unit) * unit);
        if (cut >= n2) cut = (n2 / 2 + RT_GROUP - 1) / RT_GROUP * RT_GROUP;
        std::nth_element(kd.begin() + b, kd.begin() + b + cut, kd.begin() + e, less);
        split(b, b + cut);
        split(b + cut, e);
    };
    split(0, kd.size());
    // the large spheres padded to a whole 32-sphere block, so that the k-d
    // subtrees of 32 that follow are exactly the matrix-core walk's blocks
    // (padded to a group only, the blocks straddled subtrees: RTIOW bound
    // radii 4.3-11.4 instead of 3.5-4.8)
    std::vector<uint32_t> order = big;
    if (!big.empty())
        while (order.size() % 32) order.push_back(0xFFFFFFFFu);
    for (uint32_t i : kd) order.push_back(i);
    while (order.size() % RT_GROUP) order.push_back(0xFFFFFFFFu);
    return order;
}

// Walk positions of spatial_order's list for n spheres, at most: the large
// spheres padded to a whole 32-sphere block (<= 31 pads), the rest to a group
// (<= 7) -- the matrix-core buffers are sized for it, so rebuilding them after
// rt_update_spheres (which can move spheres between the large and the rest)
// never reallocates.
static uint32_t spatial_order_max(uint32_t n) { return n + 31u + RT_GROUP - 1u; }

// The culled list: spatial_order's list in groups, clusters of 8 groups and
// supers of 8 clusters with their bounds. rm: (radius, material bits) in the
// original order.
static void cull_layout(const float4* sph, const float* S, const float2* rm, uint32_t n,
                        CullLayout& L) {
    auto finite_rec = [&](uint32_t i) {
        const float4 q = sph[i];
        return std::isfinite(q.x) && std::isfinite(q.y) && std::isfinite(q.z) && std::isfinite(q.w) &&
               std::isfinite(S[i]);
    };
    const std::vector<uint32_t> order = spatial_order(sph, S, n);
    L.ngroups = (uint32_t)(order.size() / RT_GROUP);
    L.nclusters = (L.ngroups + 7) / 8;
    const uint32_t slots = L.nclusters * 8;  // groups the walk may visit
    L.nrec = (slots + 1) * RT_GROUP;         // + one pad group, as the plain list
    L.perm.assign(L.nrec, 0xFFFFFFFFu);
    L.sph.assign(L.nrec, make_float4(0.0f, 0.0f, 0.0f, -INFINITY));
    L.rm.assign(L.nrec, make_float2(0.0f, 0.0f));
    std::vector<float> Sp(L.nrec, -INFINITY);
    for (size_t p = 0; p < order.size(); ++p) {
        const uint32_t i = order[p];
        if (i == 0xFFFFFFFFu) continue;
        L.perm[p] = i;
        L.sph[p] = sph[i];
        L.rm[p] = rm[i];
        Sp[p] = S[i];
    }
    L.grp.assign(L.nrec, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (uint32_t g = 0; g < L.nrec / RT_GROUP; ++g)
        pack_group_soa(&L.sph[RT_GROUP * g], &Sp[RT_GROUP * g], &L.grp[RT_GROUP * g]);
    // bounds: per cluster the SoA record of its 8 group bounds, per super (8
    // clusters) the record of its 8 cluster bounds; bnd = supers, then clusters
    const double kB = 1.0 - 0x1p-16 - 0x1p-7;
    auto bound_of = [&](uint32_t p0, uint32_t p1, float4& C, float& SB) {
        double blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        bool any = false, wild = false;
        for (uint32_t p = p0; p < p1; ++p) {
            const uint32_t i = L.perm[p];
            if (i == 0xFFFFFFFFu) continue;
            any = true;
            const float4 q = sph[i];
            if (!finite_rec(i) || std::fabs(q.x) > 0x1p30f || std::fabs(q.y) > 0x1p30f ||
                std::fabs(q.z) > 0x1p30f || q.w > 0x1p60f) {
                wild = true;
                continue;
            }
            const double c[3] = {q.x, q.y, q.z};
            for (int k = 0; k < 3; ++k) {
                blo[k] = std::min(blo[k], c[k]);
                bhi[k] = std::max(bhi[k], c[k]);
            }
        }
        C = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        SB = -INFINITY;  // empty: never passes
        if (any && wild) {
            SB = INFINITY;  // always passes
        } else if (any) {
            C = make_float4((float)((blo[0] + bhi[0]) * 0.5), (float)((blo[1] + bhi[1]) * 0.5),
                            (float)((blo[2] + bhi[2]) * 0.5), 0.0f);
            double Lm = 0.0;
            for (uint32_t p = p0; p < p1; ++p) {
                const uint32_t i = L.perm[p];
                if (i == 0xFFFFFFFFu) continue;
                const float4 q = sph[i];
                const double dx = (double)q.x - C.x, dy = (double)q.y - C.y, dz = (double)q.z - C.z;
                const double rho = std::sqrt(dx * dx + dy * dy + dz * dz) * (1.0 + 0x1p-40);
                Lm = std::max(Lm, rho + std::sqrt((double)q.w) * (1.0 + 0x1p-18));
            }
            const double R2 = (1.0 + 0x1p-3) * Lm * Lm * (1.0 + 0x1p-40) + 0x1p-60;
            const double CC = (double)C.x * C.x + (double)C.y * C.y + (double)C.z * C.z;
            SB = round_up_f32((R2 - kB * CC) * (1.0 + 0x1p-40) + 0x1p-60);
        }
    };
    L.nsupers = (L.nclusters + 7) / 8;
    L.bnd.assign((size_t)(L.nsupers + L.nclusters) * 8, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    float4 q[8];
    float sb[8];
    for (uint32_t u = 0; u < L.nsupers; ++u) {
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t k = u * 8 + j;  // cluster
            if (k < L.nclusters)
                bound_of(k * 8 * RT_GROUP, (k + 1) * 8 * RT_GROUP, q[j], sb[j]);
            else
                q[j] = make_float4(0.0f, 0.0f, 0.0f, 0.0f), sb[j] = -INFINITY;
        }
        pack_group_soa(q, sb, &L.bnd[(size_t)u * 8]);
    }
    for (uint32_t k = 0; k < L.nclusters; ++k) {
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t g = k * 8 + j;
            bound_of(g * RT_GROUP, (g + 1) * RT_GROUP, q[j], sb[j]);
        }
        pack_group_soa(q, sb, &L.bnd[(size_t)(L.nsupers + k) * 8]);
    }
}

// The culled list's shading records from h_rm_c and the current materials.
static int upload_shd_c(rt_ctx* ctx) {
    std::vector<float4> rec(2 * ctx->h_rm_c.size());
    shade_records(ctx->h_rm_c.data(), ctx->h_rm_c.size(), ctx->h_mats, rec.data());
    HIP_TRY(ctx, hipMemcpy(ctx->d_shd_c, rec.data(), sizeof(float4) * rec.size(), hipMemcpyHostToDevice));
    return RT_OK;
}

// Rebuild and upload the culled list from the host mirrors (set_scene / update).
static int build_cull(rt_ctx* ctx) {
    CullLayout L;
    cull_layout(ctx->h_sph.data(), ctx->h_S.data(), ctx->h_rm.data(), ctx->n, L);
    int rc = ensure(ctx, &ctx->d_grp_c, &ctx->grp_c_cap, sizeof(float4) * L.nrec);
    if (!rc) rc = ensure(ctx, &ctx->d_sph_c, &ctx->sph_c_cap, sizeof(float4) * L.nrec);
    if (!rc) rc = ensure(ctx, &ctx->d_shd_c, &ctx->shd_c_cap, 2 * sizeof(float4) * L.nrec);
    if (!rc) rc = ensure(ctx, &ctx->d_bnd_c, &ctx->bnd_c_cap, sizeof(float4) * L.bnd.size());
    if (!rc) rc = ensure(ctx, &ctx->d_perm_c, &ctx->perm_c_cap, sizeof(uint32_t) * L.nrec);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(ctx->d_grp_c, L.grp.data(), sizeof(float4) * L.nrec, hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(ctx->d_sph_c, L.sph.data(), sizeof(float4) * L.nrec, hipMemcpyHostToDevice));
    ctx->h_rm_c = L.rm;
    {
        int rc2 = upload_shd_c(ctx);
        if (rc2) return rc2;
    }
    if (!L.bnd.empty())
        HIP_TRY(ctx, hipMemcpy(ctx->d_bnd_c, L.bnd.data(), sizeof(float4) * L.bnd.size(),
                               hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(ctx->d_perm_c, L.perm.data(), sizeof(uint32_t) * L.nrec,
                           hipMemcpyHostToDevice));
    ctx->n_c = L.ngroups * RT_GROUP;
    ctx->ngroups_c = L.ngroups;
    ctx->nclusters_c = L.nclusters;
    return RT_OK;
}

static int check_materials(rt_ctx* ctx, const rt_material* mats, uint32_t first, uint32_t count) {
    for (uint32_t j = 0; j < count; ++j) {
        const int r = mats[j].reflectance;
        if (r < RT_LAMBERTIAN || r > RT_DIELECTRIC)
            return fail(ctx, RT_ERR_BAD_SCENE, "material %u: reflectance %d not in {0,1,2}",
                        first + j, r);
    }
    return RT_OK;
}

static int check_spheres(rt_ctx* ctx, const rt_sphere* sp, uint32_t first, uint32_t count,
                         uint32_t m) {
    for (uint32_t i = 0; i < count; ++i)
        if (sp[i].material >= m)
            return fail(ctx, RT_ERR_BAD_SCENE, "sphere %u: material %u >= material count %u",
                        first + i, sp[i].material, m);
    return RT_OK;
}

static int quiesce(rt_ctx* ctx) {  // no kernel may be reading the scene while it changes
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    for (Frame& f : ctx->fr) {
        HIP_TRY(ctx, hipStreamSynchronize(f.stream));
        if (f.pending_stream) HIP_TRY(ctx, hipStreamSynchronize(f.pending_stream));
    }
    return RT_OK;
}

#ifdef RT_MFMA_FILTER
// ---- matrix-core filter fragments (rt_dev_intersect.h intersect_world_mfma) ----
// The filter value less the ray's k1^2, H0 = S' + L.c + sum_ab Q_ab c_a c_b, is
// one 32-term dot product of a sphere row and a ray column (K = 32: two
// chained v_mfma_f32_32x32x16_f16). The sphere's features y_0..y_8 = c_x, c_y,
// c_z, then c_a c_b 2^-sq for ab = xx, yy, zz, xy, xz, yz, each as f16 hi/lo;
// row j in words of two halves (K 2m, 2m+1 in word m):
//   K group 0  w0..w3   (hi y0, hi y1) .. (hi y6, hi y7)
//              w4..w7   (lo y0, lo y1) .. (lo y6, lo y7)
//   K group 1  w8..w11  (hi y0, hi y1) .. (hi y6, hi y7)
//              w12      (hi y8, hi y8)
//              w13      (lo y8, 1)          1 against the ray's T0 hi
//              w14      (1, S' hi)          S' = r^2 - (1 - m - mu')|c|^2
//              w15      (S' lo, 0)
// against the ray column's hi x / hi x / lo x pairs, (hi x8, lo x8), (hi x8,
// T0 hi), (T0 lo, -1), (-1, 0) (x = the NEGATED ray features): the MFMAs give
// T0 - H0 (rt_dev_intersect.h). hi = RN_f16(x), lo = RN_f16(x - hi), all from
// double. sq scales the quadratic features into f16 range (max |c_a c_b|
// 2^-sq <= 2^14); the ray side carries 2^sq. Block b (spheres 32b..32b+31):
// two uint4 per lane, A0 (K 0..15) then A1 (K 16..31), 64 lanes each; lane l:
// row l & 31, elements k = 8 (l >> 5) .. + 8 of that half. Pad rows: 0, the
// two 1s, S' hi = -inf (T0 - H0 = +inf or NaN: never a candidate). Only scenes
// with |c_i| <= 2^12 and |S'| <= 2^15 take it (mf_ok); the rest keep the VALU
// filter.
static uint16_t f16_bits(double x) {
    const _Float16 h = (_Float16)x;
    uint16_t u;
    std::memcpy(&u, &h, 2);
    return u;
}

static void f16_split(double x, uint16_t& hi, uint16_t& lo) {
    hi = f16_bits(x);
    _Float16 hv;
    std::memcpy(&hv, &hi, 2);
    lo = f16_bits(x - (double)hv);
}

static const int MF_QA[6] = {0, 1, 2, 0, 0, 1}, MF_QB[6] = {0, 1, 2, 1, 2, 2};
static const double MF_KS = 1.0 - 0x1p-16 - 0x1p-16;           // 1 - m - mu' (RT_MF_MU)
static const double MF_KB = 1.0 - 0x1p-16 - 0x1p-16 - 0x1p-12;  // 1 - m - mu' - muB (RT_MF_MUB)

// A record inside the f16 split's range (|c_i| <= 2^12, r^2 in [0, 2^24]),
// and its largest quadratic feature max_ab |c_a c_b| = max_a c_a^2.
static bool mf_in_range(const float4 q) {
    return std::fabs(q.x) <= 0x1p12f && std::fabs(q.y) <= 0x1p12f && std::fabs(q.z) <= 0x1p12f &&
           q.w >= 0.0f && q.w <= 0x1p24f;
}
static double mf_qmax(const float4 q) {
    const double x = q.x, y = q.y, z = q.z;
    return std::max(x * x, std::max(y * y, z * z));
}
// sq for the largest quadratic feature: max |c_a c_b| 2^-sq <= 2^14 (<= 10
// for |c| <= 2^12)
static int mf_sq_of(double qmax) {
    int sq = 0;
    while (std::max(qmax, 1.0) * std::ldexp(1.0, -sq) > 0x1p14) ++sq;
    return sq;
}
// sq of n records, or -1 when a record is outside the split's range
static int mf_scale(const float4* sph, uint32_t n) {
    double qmax = 1.0;
    for (uint32_t j = 0; j < n; ++j) {
        if (!mf_in_range(sph[j])) return -1;
        qmax = std::max(qmax, mf_qmax(sph[j]));
    }
    return mf_sq_of(qmax);
}

// S' of a record (the row's constant; the walk takes |S'| <= 2^15)
static double mf_S(const float4 q) {
    const double c[3] = {q.x, q.y, q.z};
    return (double)q.w - MF_KS * (c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
}

// the row of a sphere or bound (c, S'): K 0..31 (f16 bits); pad: S' = -inf
static void mf_make_row(const double c[3], double S, int sq, uint16_t row[32]) {
    std::memset(row, 0, 64);
    uint16_t hi[9], lo[9];
    for (int a = 0; a < 3; ++a) f16_split(c[a], hi[a], lo[a]);
    for (int f = 0; f < 6; ++f) f16_split(std::ldexp(c[MF_QA[f]] * c[MF_QB[f]], -sq), hi[3 + f], lo[3 + f]);
    for (int f = 0; f < 8; ++f) {
        row[f] = hi[f];       // w0..w3
        row[8 + f] = lo[f];   // w4..w7
        row[16 + f] = hi[f];  // w8..w11
    }
    row[24] = row[25] = hi[8];  // w12
    row[26] = lo[8];            // w13
    row[27] = row[28] = f16_bits(1.0);  // against the ray's T0 hi, lo
    if (std::isinf(S)) row[29] = f16_bits(S);
    else f16_split(S, row[29], row[30]);  // w14 hi half, w15 lo half
}

// walk position p's record and sphere row (its original index H.order[p],
// or a pad); false when |S'| leaves the split's range
static bool mf_set_pos(MfHost& H, uint32_t p, const float4* sph) {
    const uint32_t b = p / 32, l0 = p & 31;
    uint16_t row[32];
    const uint32_t i = H.order[p];
    if (i != 0xFFFFFFFFu) {
        const float4 q = sph[i];
        H.msph[p] = q;
        H.mperm[p] = i;
        H.iperm[i] = p;
        const double c[3] = {q.x, q.y, q.z};
        const double S = mf_S(q);
        if (!(std::fabs(S) <= 0x1p15)) return false;
        mf_make_row(c, S, H.sq, row);
    } else {
        const double c[3] = {0.0, 0.0, 0.0};
        mf_make_row(c, -INFINITY, H.sq, row);
    }
    // A0 (K 0..15) of every lane at entry l; A1 (K 16..31) of lanes 32..63 at
    // entry 64 + (l - 32). Lanes 0..31 of A1 hold K 16..23 = the hi parts
    // again, equal to their A0 (K 0..7): the kernel reads A0's entry for them
    // (rt_dev_intersect.h intersect_world_mfma)
    uint16_t* blk = &H.A[(size_t)b * RT_MF_BLK * 8];
    std::memcpy(&blk[(size_t)l0 * 8], &row[0], 16);           // lane l0 (hh = 0)
    std::memcpy(&blk[(size_t)(l0 + 32) * 8], &row[8], 16);    // lane l0 + 32 (hh = 1)
    std::memcpy(&blk[(size_t)(64 + l0) * 8], &row[24], 16);   // A1 of lane l0 + 32
    return true;
}

// The bound of walk positions [p0, p1) as row j of bound chunk blk: line row
// K 0..31 and forward row K 0..7 (rt_dev_intersect.h "Block bounds",
// "Forward bounds"); no member: never passes. A bound row has K 31 = 1,
// against the ray column's -RN_f16(muB |o|^2); the forward row is C hi x3, 1 |
// L' (rounded up), 0 x3 against the ray's dn hi x3, c0 hi | 1, 0 x3
// (v_mfma_f32_32x32x8_f16 B fragments, 8 bytes per lane at uint2 256 + lane).
// chunk: the row is a chunk-level bound (512 walk positions, L ~ 15-35 for
// the 10,000-sphere field) -- its own split of the proof's slack (rt_dev_
// intersect.h "Chunk bounds"): R^2 = (1 + 2^-7 + 2^-9) L^2 and 4 muB (K 31 =
// 4), where a half-block's (L ~ 3) is R^2 = (1 + 2^-5 + 2^-10) L^2 and muB.
static void mf_bound_row(const MfHost& H, uint32_t p0, uint32_t p1, uint16_t* blk, uint32_t j,
                         bool chunk = false) {
    double lo3[3] = {INFINITY, INFINITY, INFINITY}, hi3[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool any = false;
    for (uint32_t p = p0; p < p1; ++p) {
        if (H.order[p] == 0xFFFFFFFFu) continue;
        any = true;
        const float4 q = H.msph[p];
        const double c[3] = {q.x, q.y, q.z};
        for (int a = 0; a < 3; ++a) {
            lo3[a] = std::min(lo3[a], c[a]);
            hi3[a] = std::max(hi3[a], c[a]);
        }
    }
    double C[3] = {0.0, 0.0, 0.0}, SB = -INFINITY;  // empty: never passes
    double Lf = 0.0;  // the forward row's L' (empty: 0, never reached)
    if (any) {
        for (int a = 0; a < 3; ++a) C[a] = (double)(float)((lo3[a] + hi3[a]) * 0.5);
        double Lm = 0.0;
        for (uint32_t p = p0; p < p1; ++p) {
            if (H.order[p] == 0xFFFFFFFFu) continue;
            const float4 q = H.msph[p];
            const double dx = q.x - C[0], dy = q.y - C[1], dz = q.z - C[2];
            Lm = std::max(Lm, std::sqrt(dx * dx + dy * dy + dz * dz) * (1.0 + 0x1p-40) +
                                  std::sqrt((double)q.w) * (1.0 + 0x1p-18));
        }
        // (1 + 2^-5 + 2^-10) (round 6; 1 + 2^-4 before, the culled list's
        // 1 + 2^-3): rt_dev_intersect.h "Block bounds"
        const double R2 = (chunk ? 1.0 + 0x1p-7 + 0x1p-9 : 1.0 + 0x1p-5 + 0x1p-10) * Lm * Lm *
                              (1.0 + 0x1p-40) + 0x1p-60;
        const double CC = C[0] * C[0] + C[1] * C[1] + C[2] * C[2];
        const double kB = chunk ? MF_KB - 3.0 * 0x1p-12 : MF_KB;  // 1 - m - mu' - (4) muB
        SB = (double)round_up_f32((R2 - kB * CC) * (1.0 + 0x1p-40) + 0x1p-60);
        if (!(std::fabs(SB) <= 0x1p15)) SB = INFINITY;  // out of the split's range: always passes
        // L' = (1 + 2^-12) L + 2^-8 |C|_1 + 2^-14, rounded up; +inf (the
        // forward row always passes) with the line row's or beyond f16
        const double C1 = std::fabs(C[0]) + std::fabs(C[1]) + std::fabs(C[2]);
        Lf = (1.0 + 0x1p-12) * Lm + 0x1p-8 * C1 + 0x1p-14;
        if (std::isinf(SB) || !(Lf <= 0x1p15)) Lf = INFINITY;
    }
    uint16_t row[32];
    mf_make_row(C, SB, H.sq, row);
    row[31] = f16_bits(chunk ? 4.0 : 1.0);  // against the ray's -RN_f16(muB |o|^2)
    for (int hh = 0; hh < 2; ++hh)
        for (int half = 0; half < 2; ++half)  // B0: K 0..15, B1: K 16..31
            std::memcpy(&blk[((size_t)half * 64 + 32 * hh + j) * 8], &row[16 * half + 8 * hh], 16);
    uint16_t fw[8] = {};
    for (int a = 0; a < 3; ++a) fw[a] = f16_bits(C[a]);
    fw[3] = f16_bits(1.0);  // against the ray's c0
    fw[4] = f16_bits(Lf);   // against the ray's 1; rounded up below
    {
        _Float16 hv;
        std::memcpy(&hv, &fw[4], 2);
        if ((double)hv < Lf) ++fw[4];  // the next f16 up (Lf > 0)
    }
    for (int hh = 0; hh < 2; ++hh) std::memcpy(&blk[(size_t)128 * 8 + (32 * hh + j) * 4], &fw[4 * hh], 8);
}

// Block bounds: per chunk of 32 bound rows, two bounds per 32-sphere block,
// one per 16-sphere half (a block is walked for a half-wave when either
// passes): bound row r of chunk k = half r & 1 of block 16 k + (r >> 1).
static void mf_half_block_bound(MfHost& H, uint32_t r) {
    const uint32_t k = r / 32, j = r & 31, p0 = 16 * r;
    mf_bound_row(H, p0, r < 2 * H.nblk ? p0 + 16 : p0, &H.B[(size_t)k * RT_MF_BCHUNK * 8], j);
}

// Chunk-level bounds (lists of 2..32 bound chunks, 513..16,384 walk
// positions): one more chunk after the others, row j = the bound of chunk j's
// 512 walk positions, tested first, so a half-wave only tests the block
// bounds of the chunks it passes near (rt_dev_intersect.h "Chunk bounds";
// 10,000 spheres: 20 chunks).
static void mf_chunk_bound(MfHost& H, uint32_t j) {
    const uint32_t p0 = 512 * j, p1 = j < H.nchunk ? std::min(p0 + 512, H.npos) : p0;
    mf_bound_row(H, p0, p1, &H.B[(size_t)H.nchunk * RT_MF_BCHUNK * 8], j, true);
}

// The whole layout of n records in walk order `order` (spatial_order's) at
// scale sq; false when the list does not fit the walk (more than 2,048
// blocks: the queue entries' 14-bit group index, rt_dev_intersect.h
// mf_spread) or a row leaves the split's range.
static bool mf_fill(const float4* sph, uint32_t n, std::vector<uint32_t> order, int sq, MfHost& H) {
    H = MfHost{};
    H.sq = sq;
    H.nblk = (uint32_t)((order.size() + 31) / 32);
    if (H.nblk > 2048u) return false;
    H.npos = H.nblk * 32;
    order.resize(H.npos, 0xFFFFFFFFu);
    H.order = std::move(order);
    H.A.assign((size_t)H.nblk * RT_MF_BLK * 8, 0);
    H.msph.assign(H.npos, make_float4(0.0f, 0.0f, 0.0f, -INFINITY));
    H.mperm.assign(H.npos, 0u);
    H.iperm.assign(n, 0u);
    for (uint32_t p = 0; p < H.npos; ++p)
        if (!mf_set_pos(H, p, sph)) return false;
    H.bqmax.assign(H.nblk, 0.0);
    for (uint32_t p = 0; p < H.npos; ++p)
        if (H.order[p] != 0xFFFFFFFFu) H.bqmax[p / 32] = std::max(H.bqmax[p / 32], mf_qmax(H.msph[p]));
    H.nchunk = (H.nblk + 15) / 16;
    H.top = H.nchunk >= 2 && H.nchunk <= 32;
    H.B.assign((size_t)(H.nchunk + (H.top ? 1 : 0)) * RT_MF_BCHUNK * 8, 0);
    for (uint32_t r = 0; r < H.nchunk * 32; ++r) mf_half_block_bound(H, r);
    if (H.top)
        for (uint32_t j = 0; j < 32; ++j) mf_chunk_bound(H, j);
    H.ok = true;
    return true;
}

// The layout from scratch: scale, spatial order (the culled list's: large
// spheres first, padded to a whole block, the rest in k-d order; only the
// order, no groups or bounds of the culled list), rows, bounds.
static bool mf_build(const float4* sph, const float* S, uint32_t n, MfHost& H) {
    H = MfHost{};
    if (!n) return false;
    const int sq = mf_scale(sph, n);
    if (sq < 0) return false;
    return mf_fill(sph, n, spatial_order(sph, S, n), sq, H);
}

// Moved spheres into the layout in place, keeping the walk order: every moved
// sphere must keep its radius (the large / small split, whose threshold is a
// median radius, is unchanged then) and stay within its block's box of
// centres grown by a quarter of the box's largest extent on each side (so
// the order stays a spatial one and the block's bound grows little), and the
// scale sq must not change. Then its position's record and row, its
// half-block's bound row and (with chunk-level bounds) its chunk's row are
// rebuilt: O(moved) plus one O(N) pass for sq. The result is byte for byte
// mf_fill of the same order (tests/test_scene_update.py). false: H is
// untouched and the caller rebuilds everything. touched_*: what to upload.
static bool mf_update(MfHost& H, const float4* sph, uint32_t n, const std::vector<uint32_t>& moved,
                      std::vector<uint32_t>& touched_blocks, std::vector<uint32_t>& touched_chunks,
                      std::vector<uint32_t>& touched_pos) {
    if (!H.ok || H.iperm.size() != n) return false;
    for (uint32_t i : moved) {
        if (i >= n) return false;
        const uint32_t p = H.iperm[i];
        const float4 o = H.msph[p], q = sph[i];
        if (std::memcmp(&o.w, &q.w, 4) != 0) return false;
        if (!(std::fabs(mf_S(q)) <= 0x1p15)) return false;
        double lo3[3] = {INFINITY, INFINITY, INFINITY}, hi3[3] = {-INFINITY, -INFINITY, -INFINITY};
        const uint32_t b = p / 32;
        for (uint32_t pp = 32 * b; pp < 32 * b + 32; ++pp) {
            if (H.order[pp] == 0xFFFFFFFFu) continue;
            const double c[3] = {H.msph[pp].x, H.msph[pp].y, H.msph[pp].z};
            for (int a = 0; a < 3; ++a) {
                lo3[a] = std::min(lo3[a], c[a]);
                hi3[a] = std::max(hi3[a], c[a]);
            }
        }
        const double ext = std::max(hi3[0] - lo3[0], std::max(hi3[1] - lo3[1], hi3[2] - lo3[2])) * 0.25;
        const double c[3] = {q.x, q.y, q.z};
        for (int a = 0; a < 3; ++a)
            if (!(c[a] >= lo3[a] - ext && c[a] <= hi3[a] + ext)) return false;
    }
    // the scale from the per-block maxima, the moved spheres' blocks
    // recomputed with their new records: O(32 moved + blocks), not O(N)
    std::vector<uint32_t> blocks;
    for (uint32_t i : moved) {
        if (!mf_in_range(sph[i])) return false;
        blocks.push_back(H.iperm[i] / 32);
    }
    std::sort(blocks.begin(), blocks.end());
    blocks.erase(std::unique(blocks.begin(), blocks.end()), blocks.end());
    std::vector<double> bq(blocks.size(), 0.0);
    for (size_t k = 0; k < blocks.size(); ++k)
        for (uint32_t p = 32 * blocks[k]; p < 32 * blocks[k] + 32; ++p)
            if (H.order[p] != 0xFFFFFFFFu) bq[k] = std::max(bq[k], mf_qmax(sph[H.order[p]]));
    double qmax = 1.0;
    for (uint32_t b = 0, k = 0; b < H.nblk; ++b) {
        const bool t = k < blocks.size() && blocks[k] == b;
        qmax = std::max(qmax, t ? bq[k] : H.bqmax[b]);
        k += t ? 1 : 0;
    }
    if (mf_sq_of(qmax) != H.sq) return false;
    for (size_t k = 0; k < blocks.size(); ++k) H.bqmax[blocks[k]] = bq[k];
    touched_blocks.clear();
    touched_chunks.clear();
    touched_pos.clear();
    std::vector<uint32_t> halves;
    for (uint32_t i : moved) {
        const uint32_t p = H.iperm[i];
        mf_set_pos(H, p, sph);  // (in range: checked above)
        touched_pos.push_back(p);
        touched_blocks.push_back(p / 32);
        halves.push_back(p / 16);
        touched_chunks.push_back(p / 512);
    }
    auto uniq = [](std::vector<uint32_t>& v) {
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
    };
    uniq(touched_blocks);
    uniq(halves);
    uniq(touched_chunks);
    uniq(touched_pos);
    for (uint32_t r : halves) mf_half_block_bound(H, r);
    if (H.top) {
        for (uint32_t k : touched_chunks) mf_chunk_bound(H, k);
        touched_chunks.push_back(H.nchunk);  // the chunk-level chunk changed too
    }
    return true;
}

// Upload the whole layout (build_mfma).
static int mf_upload_all(rt_ctx* ctx) {
    const MfHost& H = ctx->mfh;
    // buffers sized for the largest order n spheres can have: a rebuild after
    // rt_update_spheres never reallocates (a reserved render allocates nothing)
    const uint32_t nblk_max = (spatial_order_max(ctx->n) + 31) / 32;
    const size_t nchunk_max = (nblk_max + 15) / 16 + 1;  // + the chunk-level bounds
    int rc = ensure(ctx, &ctx->d_mfA, &ctx->mfA_cap, (size_t)nblk_max * RT_MF_BLK * 16);
    if (!rc) rc = ensure(ctx, &ctx->d_mfB, &ctx->mfB_cap, nchunk_max * RT_MF_BCHUNK * 16);
    if (!rc) rc = ensure(ctx, &ctx->d_mf_sph, &ctx->mf_sph_cap, (size_t)nblk_max * 32 * sizeof(float4));
    if (!rc) rc = ensure(ctx, &ctx->d_mf_perm, &ctx->mf_perm_cap, (size_t)nblk_max * 32 * sizeof(uint32_t));
    if (!rc) rc = ensure(ctx, &ctx->d_mf_shd, &ctx->mf_shd_cap, (size_t)nblk_max * 32 * 2 * sizeof(float4));
    if (!rc) rc = ensure(ctx, &ctx->d_mf_iperm, &ctx->mf_iperm_cap, (size_t)ctx->n * sizeof(uint32_t));
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(ctx->d_mfA, H.A.data(), H.A.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(ctx->d_mfB, H.B.data(), H.B.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(ctx->d_mf_sph, H.msph.data(), H.msph.size() * sizeof(float4), hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(ctx->d_mf_perm, H.mperm.data(), H.mperm.size() * sizeof(uint32_t),
                           hipMemcpyHostToDevice));
    // original index -> walk position, and the walk-order shading records
    HIP_TRY(ctx, hipMemcpy(ctx->d_mf_iperm, H.iperm.data(), H.iperm.size() * sizeof(uint32_t),
                           hipMemcpyHostToDevice));
    return upload_shd_mf(ctx);
}

static int build_mfma(rt_ctx* ctx) {
    ctx->mf_ok = false;
    ctx->mf_moved.clear();
    ctx->mf_moved_flag.assign(ctx->n, 0);
    if (!mf_build(ctx->h_sph.data(), ctx->h_S.data(), ctx->n, ctx->mfh)) {
        ctx->mfh = MfHost{};
        return RT_OK;  // outside the walk's range: the VALU filter
    }
    const int rc = mf_upload_all(ctx);
    if (rc) return rc;
    ++ctx->mf_builds;
    ctx->mf_nblk = ctx->mfh.nblk;
    ctx->mf_top = ctx->mfh.top;
    ctx->mf_qs = (float)std::ldexp(1.0, ctx->mfh.sq);
    ctx->mf_abs = (float)std::ldexp(1.0, ctx->mfh.sq - 20);
    ctx->mf_ok = true;
    return RT_OK;
}

// The spheres rt_update_spheres moved since the layout was built, in place
// (mf_update) when they allow it: only the touched A blocks (1.5 KB each),
// bound chunks (2.5 KB each) and walk positions' records and shading records
// go to the device. Else the whole layout is rebuilt.
static int mf_apply_moves(rt_ctx* ctx) {
    std::vector<uint32_t> tb, tc, tp;
    const bool inplace = ctx->mf_ok &&
                         mf_update(ctx->mfh, ctx->h_sph.data(), ctx->n, ctx->mf_moved, tb, tc, tp);
    if (!inplace) return build_mfma(ctx);
    const MfHost& H = ctx->mfh;
    for (uint32_t b : tb)
        HIP_TRY(ctx, hipMemcpy(reinterpret_cast<uint16_t*>(ctx->d_mfA) + (size_t)b * RT_MF_BLK * 8,
                               &H.A[(size_t)b * RT_MF_BLK * 8], RT_MF_BLK * 16, hipMemcpyHostToDevice));
    for (uint32_t k : tc)
        HIP_TRY(ctx, hipMemcpy(reinterpret_cast<uint16_t*>(ctx->d_mfB) + (size_t)k * RT_MF_BCHUNK * 8,
                               &H.B[(size_t)k * RT_MF_BCHUNK * 8], RT_MF_BCHUNK * 16, hipMemcpyHostToDevice));
    for (uint32_t p : tp) {
        HIP_TRY(ctx, hipMemcpy(ctx->d_mf_sph + p, &H.msph[p], sizeof(float4), hipMemcpyHostToDevice));
        float4 rec[2];
        shade_records(&ctx->h_rm[H.order[p]], 1, ctx->h_mats, rec);
        HIP_TRY(ctx, hipMemcpy(ctx->d_mf_shd + 2 * (size_t)p, rec, sizeof(rec), hipMemcpyHostToDevice));
    }
    for (uint32_t i : ctx->mf_moved) ctx->mf_moved_flag[i] = 0;
    ctx->mf_moved.clear();
    ++ctx->mf_inplace;
    return RT_OK;
}
#endif

int rt_set_scene(rt_ctx* ctx, const rt_sphere* spheres, uint32_t n, const rt_material* materials,
                 uint32_t m) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_set_scene: ctx is NULL");
    if (n && !spheres) return fail(ctx, RT_ERR_INVALID_ARG, "rt_set_scene: spheres is NULL, n=%u", n);
    if (m && !materials)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_set_scene: materials is NULL, m=%u", m);
    int rc = check_materials(ctx, materials, 0, m);
    if (rc) return rc;
    rc = check_spheres(ctx, spheres, 0, n, m);
    if (rc) return rc;
    const uint32_t ngroups = (n + RT_GROUP - 1) / RT_GROUP;
    // + one pad group (the VALU walk's), and whole 32-sphere blocks: the
    // matrix-core walk may queue a pad row of its last block (a NaN ray),
    // whose record always misses
    const size_t nrec = std::max((size_t)(ngroups + 1) * RT_GROUP, (size_t)(n + 31) / 32 * 32);
    rc = quiesce(ctx);
    if (rc) return rc;  // nothing touched yet: the previous scene stays whole
    // From here on the host mirrors and the device buffers change: until every
    // upload succeeded there is no scene (a failed call leaves
    // RT_ERR_NO_SCENE, never a half-written or freed list behind stale counts
    // that a later update or culled build would index with).
    ctx->has_scene = false;
    ctx->cull_dirty = true;
    ctx->mf_ok = false;
    ctx->mf_dirty = false;
    ctx->n = ctx->ngroups = ctx->m = 0;
    ctx->h_sph.assign(nrec, make_float4(0.0f, 0.0f, 0.0f, -INFINITY));
    ctx->h_S.assign(nrec, -INFINITY);
    ctx->h_rm.assign(n ? n : 1, make_float2(0.0f, 0.0f));
    ctx->h_grp.assign(nrec, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (uint32_t i = 0; i < n; ++i) pack_record(ctx, i, spheres[i]);
    for (size_t g = 0; g < nrec / RT_GROUP; ++g) pack_group(ctx, g);
    ctx->h_mats.assign(materials, materials + m);
    rc = ensure(ctx, &ctx->d_sph, &ctx->sph_cap, sizeof(float4) * nrec);
    if (rc) return rc;
    rc = ensure(ctx, &ctx->d_grp, &ctx->grp_cap, sizeof(float4) * nrec);
    if (rc) return rc;
    rc = ensure(ctx, &ctx->d_shd, &ctx->shd_cap, 2 * sizeof(float4) * ctx->h_rm.size());
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(ctx->d_sph, ctx->h_sph.data(), sizeof(float4) * nrec, hipMemcpyHostToDevice));
    HIP_TRY(ctx, hipMemcpy(ctx->d_grp, ctx->h_grp.data(), sizeof(float4) * nrec, hipMemcpyHostToDevice));
    rc = upload_shd(ctx, 0, ctx->h_rm.size());
    if (rc) return rc;
    ctx->n = n;
    ctx->ngroups = ngroups;
    ctx->m = m;
    ctx->scene_fast = scene_fast_ok(ctx);
#ifdef RT_MFMA_FILTER
    rc = build_mfma(ctx);  // with the scene, so a reserved render allocates nothing
    if (rc) {
        ctx->n = ctx->ngroups = ctx->m = 0;
        return rc;
    }
#endif
    ctx->has_scene = true;  // the culled list follows lazily (cull_ready)
    return RT_OK;
}

#ifdef RT_MFMA_FILTER
// The matrix-core walk's scene as the kernels take it (mf_ok).
static MfScene mf_scene(const rt_ctx* ctx) {
    MfScene mf = {};
    mf.A = ctx->d_mfA;
    mf.B = ctx->tune.mf_cull ? ctx->d_mfB : nullptr;
    mf.sph = ctx->d_mf_sph;
    mf.perm = ctx->d_mf_perm;
    mf.shd = ctx->d_mf_shd;
    mf.iperm = ctx->d_mf_iperm;
    mf.nblk = ctx->mf_nblk;
    mf.top = ctx->mf_top && ctx->tune.mf_top ? 1u : 0u;
    mf.qs = ctx->mf_qs;
    mf.abs = ctx->mf_abs;
    return mf;
}
#endif

// The culled list of the current scene, (re)built on the first RT_FLAG_CULL
// call after rt_set_scene / rt_update_spheres. No kernel can be reading the
// old one: those calls quiesce, and the first culled call after them builds
// before it enqueues. A failed build leaves it dirty (the next call retries).
static int cull_ready(rt_ctx* ctx) {
    if (!ctx->cull_dirty) return RT_OK;
    ctx->n_c = ctx->ngroups_c = ctx->nclusters_c = 0;
    int rc = build_cull(ctx);
    if (rc) return rc;
    ctx->cull_dirty = false;
    return RT_OK;
}

// The matrix-core fragments of the current scene, rebuilt on the first
// brute-force call after rt_update_spheres (same size: no allocation). The
// update quiesced, so no kernel reads the old fragments.
static int mfma_ready(rt_ctx* ctx) {
#ifdef RT_MFMA_FILTER
    if (!ctx->mf_dirty) return RT_OK;
    int rc = mf_apply_moves(ctx);
    if (rc) return rc;
    ctx->mf_dirty = false;
#else
    (void)ctx;
#endif
    return RT_OK;
}

// Everything a call with these flags walks: built before its first enqueue,
// or by rt_reserve so a reserved render allocates and uploads nothing.
static int scene_ready(rt_ctx* ctx, uint32_t flags) {
    return (flags & RT_FLAG_CULL) ? cull_ready(ctx) : mfma_ready(ctx);
}


int rt_update_spheres(rt_ctx* ctx, uint32_t first, const rt_sphere* spheres, uint32_t count) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_update_spheres: ctx is NULL");
    if (!ctx->has_scene) return fail(ctx, RT_ERR_NO_SCENE, "rt_update_spheres before rt_set_scene");
    if (count == 0) return RT_OK;
    if (!spheres) return fail(ctx, RT_ERR_INVALID_ARG, "rt_update_spheres: spheres is NULL");
    if ((uint64_t)first + count > ctx->n)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_update_spheres: [%u, %u) outside the %u spheres",
                    first, first + count, ctx->n);
    int rc = check_spheres(ctx, spheres, first, count, ctx->m);
    if (rc) return rc;
    for (uint32_t i = 0; i < count; ++i) pack_record(ctx, first + i, spheres[i]);
#ifdef RT_MFMA_FILTER
    if (ctx->mf_moved_flag.size() == ctx->n)
        for (uint32_t i = first; i < first + count; ++i)
            if (!ctx->mf_moved_flag[i]) {
                ctx->mf_moved_flag[i] = 1;
                ctx->mf_moved.push_back(i);
            }
#endif
    const size_t g0 = first / RT_GROUP, g1 = (first + count - 1) / RT_GROUP + 1;
    for (size_t g = g0; g < g1; ++g) pack_group(ctx, g);
    rc = quiesce(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(ctx->d_sph + first, &ctx->h_sph[first], sizeof(float4) * count,
                           hipMemcpyHostToDevice));
    rc = upload_shd(ctx, first, count);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(ctx->d_grp + RT_GROUP * g0, &ctx->h_grp[RT_GROUP * g0],
                           sizeof(float4) * RT_GROUP * (g1 - g0), hipMemcpyHostToDevice));
    ctx->scene_fast = scene_fast_ok(ctx);
    ctx->cull_dirty = true;  // the permutation and bounds follow at the next culled call
#ifdef RT_MFMA_FILTER
    // and the matrix-core fragments at the next call that walks them
    // (mfma_ready): a caller rendering only the culled list never pays for them
    ctx->mf_dirty = true;
#endif
    return RT_OK;
}

int rt_update_materials(rt_ctx* ctx, uint32_t first, const rt_material* materials,
                        uint32_t count) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_update_materials: ctx is NULL");
    if (!ctx->has_scene) return fail(ctx, RT_ERR_NO_SCENE, "rt_update_materials before rt_set_scene");
    if (count == 0) return RT_OK;
    if (!materials) return fail(ctx, RT_ERR_INVALID_ARG, "rt_update_materials: materials is NULL");
    if ((uint64_t)first + count > ctx->m)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_update_materials: [%u, %u) outside the %u materials",
                    first, first + count, ctx->m);
    int rc = check_materials(ctx, materials, first, count);
    if (rc) return rc;
    std::copy(materials, materials + count, ctx->h_mats.begin() + first);
    rc = quiesce(ctx);
    if (rc) return rc;
    // every sphere's shading record carries its material: all are rebuilt
    // (O(N) on the host, 32 B per sphere), in the original order and -- when
    // the culled list exists -- in its order (its geometry, permutation and
    // bounds do not change)
    rc = upload_shd(ctx, 0, ctx->h_rm.size());
    if (rc) return rc;
#ifdef RT_MFMA_FILTER
    if (ctx->mf_ok && !ctx->mf_dirty) {  // (a pending rebuild uploads them anyway)
        rc = upload_shd_mf(ctx);
        if (rc) return rc;
    }
#endif
    if (!ctx->cull_dirty) {
        rc = upload_shd_c(ctx);
        if (rc) {
            ctx->cull_dirty = true;  // rebuilt whole at the next culled call
            return rc;
        }
    }
    return RT_OK;
}

// Validate and enqueue `nframes` frames of one camera on `stream`: frame i
// covers samples frame0 + i*spp ... (its seeds, shade.wgsl:216-218) and writes
// rows*width float4 pixels at d_out + i*rows*width.
//
// Work plan. The render kernel deals items from ONE queue per launch; a
// launch may hold several frames (their items back to back), so a frame's
// last waves overlap the next frame's first ones and only the launch pays a
// drain tail. Items are (pixel, block of RT_SAMPLE_BLOCK samples); the launch's
// tail (the last `ksplit` blocks of every frame, dealt after all block items)
// is traced as single-sample items, so no wave is left holding an 8-sample
// item of long paths when the queue runs dry. Frames go in one launch while
// their block sums fit the scratch budget; a single frame larger than that runs
// in several passes over its blocks (acc carries the partial sum).
// reserve_only (rt_reserve): size and allocate the slot's buffers exactly as
// the launch would, then return without enqueueing any work.
static int enqueue(rt_ctx* ctx, Frame& f, const rt_camera* cam, const rt_params* prm,
                   uint32_t nframes, float4* d_out, hipStream_t stream, int prog_mode = 0,
                   float prog_total = 0.0f, bool reserve_only = false) {
    if ((!cam && !reserve_only) || !prm)
        return fail(ctx, RT_ERR_INVALID_ARG, "camera or params is NULL");
    if (!ctx->has_scene) return fail(ctx, RT_ERR_NO_SCENE, "rt_render before rt_set_scene");
    const rt_params p = *prm;
    if (p.width == 0 || p.height == 0 || p.spp == 0 || p.max_depth == 0)
        return fail(ctx, RT_ERR_INVALID_ARG, "width/height/spp/max_depth must be > 0 (%u,%u,%u,%u)",
                    p.width, p.height, p.spp, p.max_depth);
    if (nframes == 0) return fail(ctx, RT_ERR_INVALID_ARG, "nframes must be > 0");
    const uint32_t K = p.shard_count ? p.shard_count : 1;
    const uint32_t B = p.row_block ? p.row_block : 1;
    if (p.shard_index >= K)
        return fail(ctx, RT_ERR_INVALID_ARG, "shard_index %u >= shard_count %u", p.shard_index, K);
    if (p.width > 65535 || p.height > 65535)
        return fail(ctx, RT_ERR_INVALID_ARG, "width/height %u x %u above 65535", p.width, p.height);
    if ((uint64_t)p.width * p.height > 0xFFFFFFFFull)
        return fail(ctx, RT_ERR_INVALID_ARG, "image of %u x %u pixels exceeds 2^32", p.width, p.height);
    if ((uint64_t)nframes * p.spp > 0xFFFFFFFFull)
        return fail(ctx, RT_ERR_INVALID_ARG, "nframes * spp exceeds 2^32");
    const uint32_t rows = rt_shard_rows(p.height, B, K, p.shard_index);
    const uint32_t npix = rows * p.width;
    if (npix >= RT_INDEX_LIMIT)
        return fail(ctx, RT_ERR_INVALID_ARG, "%u x %u rows of pixels in one call exceed 2^30",
                    p.width, rows);
    const uint32_t blocks_total = (p.spp + RT_SAMPLE_BLOCK - 1) / RT_SAMPLE_BLOCK;
    if (!d_out && !reserve_only) return fail(ctx, RT_ERR_INVALID_ARG, "output pointer is NULL");

    HIP_TRY(ctx, hipSetDevice(ctx->device));
    std::vector<Pass> passes;
    const size_t per_block = (size_t)npix * sizeof(float4);  // one slot per pixel
    // Tail: per lane ~a1*D single samples, and before them optionally a2*D
    // samples in 2-sample items and a4*D in 4-sample items (knob tail="a4,a2,a1";
    // default 0,1,0.5 since round 5 -- 0,1,1 from the pixel-major item order
    // on, the measured best on the N=8 shards then (31.4 vs 33.0 ms per
    // 20-frame launch for 0,0,6) at the same full frame,
    // profiles/r03/item_order/sweep_tail*.log; 0,0,6 with the pair-major
    // order, 0,0,12 before the matrix-core kernel; and by the call below): a
    // block item (<= 8*D iterations) taken before the tail has finished when
    // the queue runs dry, and an item taken in the tail leaves at most one
    // short path per lane to drain. In samples per pixel:
    const Tuning& tn = ctx->tune;
    const int bpc = (p.flags & RT_FLAG_CULL) ? ctx->blocks_per_cu_c : ctx->blocks_per_cu;
    // Resident workgroups per CU. A small call does better on fewer: with
    // few samples per lane the launch's ramp and drain dominate, and the
    // clock runs higher. Measured (tools/grid_probe.py, profiles/r04/grid/,
    // render-kernel ms at 4 / 3 / 2 / 1 workgroups per CU): 1080p 1 spp
    // depth 3 0.768 / 0.672 / 0.574 / 0.512; 1080p 1 spp depth 16 1.053 /
    // 0.953 / 0.867 / 0.981; 4 spp 2.139 / 2.031 / 1.973 / 2.802; 16 spp
    // 5.51 / 5.36 / 5.67 / 10.2; 64 spp 14.2 / 15.3 / 20.3 / 38.9. By the
    // call's samples per lane at full occupancy x depth (x): x < 64 -> 1,
    // < 1024 -> 2, < 4096 -> 3, else the occupancy limit. Knob wg_per_cu
    // overrides (A/B).
    uint32_t wg_run = (uint32_t)bpc;
    {
        const double x = (double)npix * p.spp * nframes /
                         ((double)std::max(ctx->cu_count, 1) * std::max(bpc, 1) * RT_BLOCK_THREADS) *
                         p.max_depth;
        const uint32_t want = x < 64.0 ? 1u : x < 1024.0 ? 2u : x < 4096.0 ? 3u : (uint32_t)bpc;
        wg_run = std::max<uint32_t>(1u, std::min<uint32_t>(want, (uint32_t)bpc));
        if (ctx->tune.wg_per_cu) wg_run = std::min<uint32_t>(ctx->tune.wg_per_cu, (uint32_t)bpc);
    }
    const uint64_t lanes = (uint64_t)ctx->cu_count * wg_run * RT_BLOCK_THREADS;
    // The tail is meant for ~(a4 + a2 + a1) D samples per lane, but it is
    // made of whole sample pairs of every pixel: one pair is 8 samples per
    // pixel however few the tail needs. Where that pair is more than 4x the
    // tail's samples (large frames: 4K one frame per launch 5.3x, the 8K
    // frame 42x; the headline 2.6x, 10k spheres 2.6x, row shards less) the
    // tail's 1- and 2-sample items, a slot per sample, cost more than they
    // balance -- measured, same box (profiles/r06/c5/): off, 4K -0.8 % time
    // and render writes 3.68 -> 2.55 GB per frame, the 8K frame -0.25 % and
    // 6.70 -> 2.21 GB; the headline +-0 either way, 10k spheres +1.8 % off.
    bool tail_on = tn.tail_split != 0;
    if (tn.tail_split < 0) {
        const double want = (tn.tail[0] + tn.tail[1] + tn.tail[2]) * p.max_depth * (double)lanes;
        tail_on = 8.0 * (double)npix <= 4.0 * want;
    }
    // One tail for every launch. (Launches with about one pixel per lane, the
    // N = 8 row shard of the headline, took 1, 1, 0.25 from the first tail
    // sweep of round 5 -- 26.09 -> 25.43 ms against 0, 1, 1; profiles/r05/tail/
    // -- until the lead items and end-of-launch chunks of 32 items: then
    // 0, 1, 0.5 measured 24.80 ms against 24.98, profiles/r05/tail/call52/.)
    const double* ta = tn.tail;
    auto per_px = [&](double a, uint64_t mult) -> uint64_t {
        if (!npix || a <= 0.0) return 0;
        const uint64_t v = (uint64_t)std::ceil(a * p.max_depth * (double)lanes / (double)npix);
        return (v + mult - 1) / mult * mult;
    };
    const bool all_single = tn.split_all && (p.flags & RT_FLAG_NO_PRIMARY_CACHE);
    const uint64_t A4 = all_single ? 0 : per_px(ta[0], 4), A2 = all_single ? 0 : per_px(ta[1], 2);
    const uint64_t A1 = all_single ? ~0ull / 4 : per_px(ta[2], 1);
    auto tail_pairs = [&](uint64_t pairs) -> uint64_t {
        if (!tail_on || !npix) return 0;
        const uint64_t L = (A4 + A2 + A1 + RT_SAMPLE_BLOCK - 1) / RT_SAMPLE_BLOCK;
        return L < 1 ? 1 : (L > pairs ? pairs : L);
    };
    // Block-item region: the last ~a8*D samples per lane of the main part are
    // dealt as single-block items (knob block_region = a8, default by the call), so the
    // lanes still holding a pixel item (up to spp*D iterations) when the main
    // part runs out finish inside the block items and the tail. It has to be
    // long: the SIMD arbiter issues by age, and the youngest waves of a SIMD
    // iterate several times slower than the oldest, so their
    // last pixel items end late. Measured at 1080p/64, 24-frame launches
    // (kernel ms, one box): a8 = 12: 521, 24: 524, 48: 517, 96: 511.5 -- the
    // round-1 all-block-items kernel 511.7. Round 5, grouped item order,
    // 20-frame launches (profiles/r05/block_region): 96: 191.8 ms, 64: 191.3,
    // 56: 190.6, 48: 194.0; render-kernel writes 1.74 / 1.50 / - / 1.40 GB
    // (fewer block items, fewer slots). The region has to outlast the last
    // pixel item, whose length is the frame's samples (spp x the path's
    // iterations): the 10,000-sphere frame (128 spp, two-frame launches,
    // profiles/r05/block_region/call11, call12) took 405 ms at 64, 160-175 at
    // 96, 154.8 at 128 and 157.2 at 160. So by the call: a8 = 16 spp / D, at
    // least 64 and at most 128 (headline 64; 10k, 4K and the 8K frame 128:
    // 4K 182.3 vs 181.6 ms, 8K 2,292 vs 2,288 ms at 96 -- within their runs'
    // spread).
    const double a8 = tn.block_region >= 0.0
                          ? tn.block_region
                          : std::min(128.0, std::max(64.0, 16.0 * p.spp / std::max(p.max_depth, 1u)));
    const uint64_t A8 = per_px(a8, 1);
    // nb: sample blocks per frame of the pass. The pixel region ends at a
    // frame boundary when that keeps >= 3/4 of the region (knob block_align):
    // its frames are then whole pixel items -- direct output, no short pixel
    // item of a partial frame, fewer slots. Headline: 17 -> 15 block pairs per
    // pixel (18 whole frames in the pixel region), -0.35 % time and render
    // writes 1.50 -> 1.43 GB; the N = 4 row shard (65 -> 62) -1.5 %, N = 8
    // unchanged (its region already ends on a frame), N = 2 (33 -> 30) +0.8 %
    // (profiles/r05/block_align/; 14 pairs, unaligned, +1.7 % at the headline).
    auto block_pairs = [&](uint64_t qmain, uint64_t nb) -> uint64_t {
        uint64_t Q = (A8 + RT_SAMPLE_BLOCK - 1) / RT_SAMPLE_BLOCK;
        if (Q >= qmain) return qmain;
        if (tn.block_align && nb > 1) {
            const uint64_t qa = (qmain - Q + nb - 1) / nb * nb;  // qpix rounded up to a frame
            if (qa < qmain && 4 * (qmain - qa) >= 3 * Q) Q = qmain - qa;
        }
        return Q;
    };
    // first launch-relative sample g = f*spp + s of pair q (block b of frame f)
    auto pair_g = [&](uint64_t q, uint64_t nb, uint64_t bb) -> uint64_t {
        const uint64_t fr = q / nb;
        return fr * p.spp + (bb + (q - fr * nb)) * RT_SAMPLE_BLOCK;
    };
    // slots per pixel of a launch of F frames x blocks [bb, bb + nb): one per
    // frame with pixel-item blocks (its lane-folded sum), one per block item,
    // one per tail sample
    // The main part's item regions: pixel items for the frames with pairs
    // below qpix (fp of them) and, with lead items (knob block_lead, m < nb),
    // one more pixel item per frame past them that has main pairs (fl - fp
    // frames), covering its first min(m, its main pairs) blocks, dealt after
    // the pixel items; block items for the other pairs in [qpix, qmain) --
    // nreg per pixel. Lead items cut the slots the block region writes and the
    // collect reads; by the call m = 2 where a pixel region exists (fp > 0).
    // Measured, same box, against no lead items (profiles/r05/block_lead/):
    // headline render-kernel writes 1.43 -> 1.36 GB per 20-frame launch at
    // +0.1 % cycles (m = 3: 1.29 GB, +0.2 %; 4: 1.22, +0.2-0.6 %; 5: 1.15,
    // +2.4 %); the N = 8 row shard -1.5 % render; 4K unchanged (one frame per
    // launch: no frame past the pixel region). Without a pixel region (10k
    // spheres' two-frame launches: block items only) every frame would get
    // one, +0.5-2.5 %: off there.
    struct Regions {
        uint64_t fp, fl, lead, nreg;
    };
    auto regions = [&](uint64_t qmain, uint64_t qpix, uint64_t nb) -> Regions {
        Regions r{(qpix + nb - 1) / nb, 0, 0, qmain - qpix};
        r.fl = r.fp;
        const uint64_t m = tn.block_lead >= 0 ? (uint64_t)tn.block_lead : (r.fp ? 2u : 0u);
        if (m && m < nb) {
            r.lead = m;
            for (uint64_t f = r.fp; f * nb < qmain; ++f, ++r.fl)
                r.nreg -= std::min<uint64_t>(r.lead, qmain - f * nb);
        }
        return r;
    };
    auto launch_slots = [&](uint64_t F, uint64_t nb, uint64_t bb) -> uint64_t {
        const uint64_t pairs = F * nb, L = tail_pairs(pairs);
        const uint64_t qmain = pairs - L, qpix = qmain - block_pairs(qmain, nb);
        const uint64_t g_end = (F - 1) * p.spp +
                               std::min<uint64_t>(p.spp, (bb + nb) * RT_SAMPLE_BLOCK);
        const uint64_t g0 = L ? pair_g(pairs - L, nb, bb) : g_end;
        const Regions rg = regions(qmain, qpix, nb);
        return rg.fl + rg.nreg + (g_end - g0);
    };
    if (npix) {
        uint64_t slots_cap = tn.scratch_bytes / per_block;
        // slot indices (and work items) stay below RT_INDEX_LIMIT: a slot
        // entry's bit 30 marks a direct output (RT_DIRECT_ITEM)
        const uint64_t by_index = (RT_INDEX_LIMIT - 1ull) / npix;
        if (slots_cap > by_index) slots_cap = by_index;
        if (slots_cap < 1) slots_cap = 1;
        uint64_t bs_slots = 0;
        uint64_t fpl = nframes;  // frames per launch: as many whole frames as fit
        while (fpl > 1 && launch_slots(fpl, blocks_total, 0) > slots_cap) --fpl;
        if (launch_slots(fpl, blocks_total, 0) <= slots_cap) {
            for (uint32_t i = 0; i < nframes; i += (uint32_t)fpl) {
                const uint32_t nf = (uint32_t)std::min<uint64_t>(fpl, nframes - i);
                passes.push_back(Pass{i, nf, 0, blocks_total});
                bs_slots = std::max(bs_slots, launch_slots(nf, blocks_total, 0));
            }
        } else {  // one frame per launch, several passes over its blocks
            if (launch_slots(1, 1, 0) > slots_cap) tail_on = false;  // no room for a tail
            uint64_t pb = blocks_total;
            while (pb > 1 && launch_slots(1, pb, 0) > slots_cap) --pb;
            for (uint32_t fi = 0; fi < nframes; ++fi)
                for (uint32_t b = 0; b < blocks_total; b += (uint32_t)pb) {
                    const uint32_t nb =
                        (uint32_t)((blocks_total - b) < pb ? (blocks_total - b) : pb);
                    passes.push_back(Pass{fi, 1, b, nb});
                    bs_slots = std::max(bs_slots, launch_slots(1, nb, b));
                }
            int rc = ensure(ctx, &f.d_acc, &f.acc_cap, per_block);
            if (rc) return rc;
        }
        int rc = ensure(ctx, &f.d_block_sums, &f.bs_cap, per_block * (size_t)bs_slots);
        if (rc) return rc;
        rc = ensure(ctx, &f.d_pd, &f.pd_cap, per_block);  // 16-B pixel table entries
        if (rc) return rc;
    }
    const size_t words = RT_CNT_WORK_OFFSET + passes.size();
    const size_t words_pad = (words + 3) & ~(size_t)3;  // 16-B multiple
    {
        int rc = ensure(ctx, &f.d_counters, &f.counters_cap, words_pad * sizeof(uint32_t));
        if (rc) return rc;
    }
    while (f.ev.size() < 2 * passes.size()) {
        hipEvent_t e;
        HIP_TRY(ctx, hipEventCreate(&e));
        f.ev.push_back(e);
    }
    {
        int rc = scene_ready(ctx, p.flags);
        if (rc) return rc;
    }
    if (reserve_only) return RT_OK;
    const bool cull = (p.flags & RT_FLAG_CULL) != 0;
    // output frame stride: the call's rows packed, or whole images (RT_FLAG_IMAGE_OUT)
    const size_t fstride = (p.flags & RT_FLAG_IMAGE_OUT) ? (size_t)p.width * p.height : (size_t)npix;
    if ((p.flags & RT_FLAG_IMAGE_OUT) && prog_mode != 0)
        return fail(ctx, RT_ERR_INVALID_ARG, "RT_FLAG_IMAGE_OUT is for device-output calls");

    KParams K_{};
    K_.width = p.width;
    K_.height = p.height;
    K_.spp = p.spp;
    K_.max_depth = p.max_depth;
    K_.frame0 = p.frame0;
    K_.row_block = B;
    K_.shard_count = K;
    K_.shard_index = p.shard_index;
    K_.npix = npix;
    K_.acc_in = f.d_acc;
    K_.nspheres = cull ? ctx->n_c : ctx->n;
    K_.ngroups = cull ? ctx->ngroups_c : ctx->ngroups;
    if (cull) {
        K_.bnd = ctx->d_bnd_c;
        K_.perm = ctx->d_perm_c;
        K_.nclusters = ctx->nclusters_c;
        // measured: with the RTIOW scene's 8 clusters the super level costs
        // more than it saves (18,582 vs 18,919 Mrays/s); with 157 clusters
        // (10 000 spheres) it saves 14 % (3,115 vs 2,685)
        K_.cull_supers = ctx->nclusters_c > 16 ? 1u : 0u;
    }
    K_.scene_fast = ctx->scene_fast && tn.fast_exact ? 1u : 0u;
    K_.flags = p.flags;
    // direct output (KParams::dout): one whole-frame pass per launch, plain
    // frames (not progressive), an output pixel index the item knows (the
    // image layout: one shard, or RT_FLAG_IMAGE_OUT); the launch's output
    // indices below RT_INDEX_LIMIT
    // another device's image (RT_FLAG_IMAGE_OUT): system-scope write-through
    // stores, acknowledged before each wave retires (collect; the per-wave
    // release only with knob dsys_release) -- and no direct output from the
    // render kernel: a store that crosses xGMI or PCIe is acknowledged so late
    // that the wave's next load wait stalls on it (measured: the reference's
    // 1-spp frame written into a registered host buffer by the render kernel
    // took 2.8 ms of kernel instead of 0.77, profiles/r04/direct/)
    K_.dsys = (p.flags & RT_FLAG_IMAGE_OUT) ? 1u : 0u;
    K_.dsys_release = tn.dsys_release ? 1u : 0u;
    const bool direct = tn.direct_out && !tn.skip_collect && prog_mode == 0 && !passes.empty() && !K_.dsys &&
                        passes[0].block_begin == 0 && passes[0].nblocks == blocks_total &&
                        (K == 1 || (p.flags & RT_FLAG_IMAGE_OUT));
    K_.dstride = (uint32_t)fstride;
    K_.dwhole_blk = blocks_total == 1 ? 1u : 0u;
    K_.dwhole_tail = p.spp == 1 ? 1u : 0u;
    // the buffers' sizes (RT_CHECK_BOUNDS builds check every index against them)
    K_.chk_nsph = (uint32_t)((cull ? ctx->sph_c_cap : ctx->sph_cap) / sizeof(float4));
    K_.chk_nrm = (uint32_t)((cull ? ctx->shd_c_cap : ctx->shd_cap) / (2 * sizeof(float4)));
    K_.chk_slots = f.bs_cap / sizeof(float4);
    if (tn.chk_shrink == 4) K_.chk_nsph = 0;
    if (tn.chk_shrink == 5) K_.chk_nrm = 0;
    if (tn.chk_shrink == 7) K_.chk_slots = 0;
#ifdef RT_MFMA_FILTER
    if (!cull && ctx->mf_ok && !(p.flags & RT_FLAG_VALU_FILTER)) {
        K_.mf = mf_scene(ctx);
        K_.chk_wsph = (uint32_t)(ctx->mf_sph_cap / sizeof(float4));
        K_.chk_wrm = (uint32_t)(ctx->mf_shd_cap / (2 * sizeof(float4)));
        if (tn.chk_shrink == 4) K_.chk_wsph = 0;
        if (tn.chk_shrink == 5) K_.chk_wrm = 0;
    }
#endif
    std::memcpy(K_.T, cam->transform, sizeof(K_.T));
    K_.tan_half = (float)std::tan((double)(cam->fov / 2.0f));                 // generate.wgsl:67
    K_.focus_plane = (cam->image_plane_distance * cam->lens_focal_length) /  // generate.wgsl:94-95
                     (cam->image_plane_distance - cam->lens_focal_length);
    K_.coc = cam->lens_focal_length / (2.0f * cam->fstop);  // generate.wgsl:97
    K_.aspect = (float)p.width;
    K_.half_w = (float)p.width / 2.0f;
    K_.half_h = (float)p.height / 2.0f;
    K_.div_npix = make_fastdiv(npix ? npix : 1);
    K_.div_width = make_fastdiv(p.width);
    K_.div_row_block = make_fastdiv(B);
    // processing order: tiles of tile_h x tile_w pixels (8 x 8 for a whole
    // image; a shard's tiles are one row block high, so a tile's pixels stay
    // neighbours in the image -- 8 packed shard rows would span two blocks
    // shard_count x row_block rows apart; 9-row blocks, the N = 8 split of
    // 1080 rows, give 9 x 8 tiles). Only the work order changes: every pixel's
    // result is its own.
    const uint32_t th = (K > 1 && B != 8 && B <= 12) ? B : 8, tw = (64 + th - 1) / th;
    K_.tile_h = th;
    K_.tile_w = tw;
    K_.tile_full_rows = rows / th;
    K_.tile_full_cols = p.width / tw;
    K_.tile_wrem = p.width % tw;
    K_.div_thw = make_fastdiv(th * p.width);
    K_.div_tp = make_fastdiv(th * tw);
    K_.div_tw = make_fastdiv(tw);
    K_.div_wrem = make_fastdiv(K_.tile_wrem ? K_.tile_wrem : 1);
    K_.prefetch = tn.prefetch ? 1u : 0u;
    // The rotation evens out the SIMD's age-ordered issue where the launch's
    // drain is a large share, or its items long (DESIGN.md 4.1 issue
    // fairness); elsewhere it costs more than it returns. Round 5, one box
    // (profiles/r05/prio/): off vs on -- headline (10,125 samples per lane,
    // 64-sample pixel items) -0.33 %, 4K (8,100; 256) -0.5 %; the N = 8
    // shard (1,266) +0.7 %, 10k spheres (2,025) +0.8 %, the 8K frame
    // (129,600; 1,024-sample items) +1.4 %. By the call: on below 4,096
    // samples per lane or where a frame's paths are long -- spp x depth
    // above 4,096 sample-bounces (round 6; round 5 had spp > 256, the same at
    // depth 16). The one-frame 4K launch (256 spp, depth 32: 8,192) ran about
    // half its runs 3-11 % slow with the rotation off -- waves starved by age
    // holding long pixel items -- and every run at the fast time with it on:
    // 6 + 6 runs, 416-462 vs 418.9-419.0 Mcycles (profiles/r06/c16/ab4k/).
    {
        const double spl = (double)npix * p.spp * nframes / (double)std::max<uint64_t>(lanes, 1);
        const double sd = (double)p.spp * p.max_depth;
        K_.prio_mode = tn.prio_mode >= 0 ? (uint32_t)tn.prio_mode : (spl < 4096.0 || sd > 4096.0 ? 1u : 0u);
    }
    const uint32_t prio_call = K_.prio_mode;  // (+ the passes with 128-item chunks, below)
    K_.prio_shift = tn.prio_shift;
    // wide (sphere-parallel) tracing pays ~32 VALU per 64 spheres per ray plus
    // a reduction; the ray-parallel walk ~34 per 8-sphere group per wave plus
    // the drain: switch while k rays cost less sphere-parallel. The wide_max
    // knob overrides (0 = never).
    {
        const uint64_t per_ray = (uint64_t)((K_.nspheres + 63) / 64) * 32 + 48;
        // culled walk: the cluster bounds plus, measured on the RTIOW scene,
        // about a quarter of the groups
        uint64_t k = ((cull ? (uint64_t)K_.nclusters * 40 + (uint64_t)K_.ngroups * 34 / 4
                            : (uint64_t)K_.ngroups * 34) + 300) / per_ray;
        if (k > 16) k = 16;
        if (tn.wide_max >= 0) k = (uint64_t)tn.wide_max;
        K_.wide_max = (uint32_t)k;
    }

    // From the first enqueued operation on, a failure must not leave work
    // running that the slot does not know about (the next enqueue could free
    // buffers under it): HIP_TRY_Q waits for what was enqueued, then reports.
#define HIP_TRY_Q(call)                                                   \
    do {                                                                  \
        hipError_t eq_ = (call);                                          \
        if (eq_ != hipSuccess) {                                          \
            hipStreamSynchronize(stream);                                 \
            return fail(ctx, RT_ERR_DEVICE, "%s failed: %s", #call,       \
                        hipGetErrorString(eq_));                          \
        }                                                                 \
    } while (0)
    HIP_TRY_Q(hipEventRecord(f.ev_t0, stream));
    HIP_TRY_Q(hipMemsetAsync(f.d_counters, 0, words_pad * sizeof(uint32_t), stream));
    const uint32_t grid_full = (uint32_t)(ctx->cu_count * wg_run);
    if (npix) HIP_TRY_Q(rt_launch_primary(&K_, f.d_pd, stream));
    for (size_t i = 0; i < passes.size(); ++i) {
        const Pass& ps = passes[i];
        K_.block_begin = ps.block_begin;
        K_.nblocks = ps.nblocks;
        K_.div_nblocks = make_fastdiv(ps.nblocks);
        K_.nframes = ps.nframes;
        K_.sample_base = ps.frame_begin * p.spp;
        const uint64_t pairs = (uint64_t)ps.nframes * ps.nblocks, L = tail_pairs(pairs);
        const uint64_t g_end = (uint64_t)(ps.nframes - 1) * p.spp +
                               std::min<uint64_t>(p.spp, (uint64_t)(ps.block_begin + ps.nblocks) *
                                                             RT_SAMPLE_BLOCK);
        const uint64_t g0 = L ? pair_g(pairs - L, ps.nblocks, ps.block_begin) : g_end;
        K_.qmain = (uint32_t)(pairs - L);
        K_.qpix = K_.qmain - (uint32_t)block_pairs(K_.qmain, ps.nblocks);
        const Regions rg = regions(K_.qmain, K_.qpix, ps.nblocks);
        K_.fp = (uint32_t)rg.fp;
        K_.lead = (uint32_t)rg.lead;
        K_.c0 = (uint32_t)(rg.fp * ps.nblocks - K_.qpix);
        K_.div_nbl = make_fastdiv(ps.nblocks - K_.lead);
        K_.main_pix = (uint32_t)rg.fl * npix;                     // (frame, pixel) items
        K_.main_fp = (uint32_t)rg.fp * npix;  // lead items after them
        K_.div_nlead = make_fastdiv(rg.fl > rg.fp ? (uint32_t)(rg.fl - rg.fp) : 1u);
        K_.main_all = K_.main_pix + (uint32_t)rg.nreg * npix;     // + (pair, pixel) items
        // tail regions from the end: single samples, 2-sample, 4-sample items
        const uint64_t g2 = g_end - std::min<uint64_t>(A1, g_end - g0);
        const uint64_t g1 = g2 - std::min<uint64_t>(A2, g2 - g0);
        K_.g0 = (uint32_t)g0;
        K_.g1 = (uint32_t)g1;
        K_.g2 = (uint32_t)g2;
        K_.g_end = (uint32_t)g_end;
        K_.ti1 = (uint32_t)((g1 - g0 + 3) / 4 * npix);
        K_.ti2 = K_.ti1 + (uint32_t)((g2 - g1 + 1) / 2 * npix);
        K_.tail_items = K_.ti2 + (uint32_t)((g_end - g2) * npix);
        // grouped order (bit 2) needs whole groups of 8 pixels; else pixel-major
        K_.pix_group_shift = tn.pix_group == 4 ? 2u : 3u;
        K_.lead_group_shift = (tn.item_order & 4u) && npix % tn.pix_group == 0 ? K_.pix_group_shift : 0u;
        K_.item_order = (tn.item_order & 4u) && npix % tn.pix_group != 0 ? (tn.item_order & 3u) | 3u
                                                                        : tn.item_order;
        K_.div_nreg = make_fastdiv(rg.nreg ? (uint32_t)rg.nreg : 1u);
        K_.div_nfpix = make_fastdiv(rg.fp ? (uint32_t)rg.fp : 1u);  // frames with pixel pairs
        K_.div_ng4 = make_fastdiv(g1 > g0 ? (uint32_t)((g1 - g0 + 3) / 4) : 1u);
        K_.div_ng2 = make_fastdiv(g2 > g1 ? (uint32_t)((g2 - g1 + 1) / 2) : 1u);
        K_.div_ng1 = make_fastdiv(g_end > g2 ? (uint32_t)(g_end - g2) : 1u);
        const uint64_t items = (uint64_t)K_.main_all + K_.tail_items;
        // Work chunk per atomic: 64 items (knob wave_chunk). 128 measured, same
        // box: headline -1.7 % but spread 437-448 Mcycles against 449.1-449.9,
        // 4K +15 %, 10k spheres +6 %, the N = 8 shard +8-18 %: a wave holding
        // a larger chunk ends later (profiles/r05/wave_chunk/). Round 6, the
        // final kernel: headline -2.7 % (5 + 5 runs, 426-437 vs 442-443
        // Mcycles, profiles/r06/c19_chunk/; 96: -0.8 %) -- so by the call:
        // 128 for launches whose pixel region holds at least 8 whole frames
        // and >= 8,192 samples per lane (the multi-frame whole-frame launches:
        // a wave's refills then stay among neighbouring pixels' frames), 64
        // for the one-frame, block-only and row-shard launches it slowed.
        {
            const double spl = (double)npix * p.spp * ps.nframes / (double)std::max<uint64_t>(lanes, 1);
            const bool big = rg.fp >= 8 && spl >= 8192.0;
            K_.chunk = tn.wave_chunk > 0 ? (uint32_t)tn.wave_chunk : (big ? 128u : (uint32_t)RT_WAVE_CHUNK);
            // ... and with the s_setprio rotation: the headline with 128-item
            // chunks and no rotation ran a third of its runs ~3 % slow (the
            // age-ordered issue again), with it 6 of 6 runs fast (426.5-430.2
            // vs 427.6-446.9 Mcycles, profiles/r06/c23/)
            K_.prio_mode = (tn.prio_mode < 0 && big && tn.wave_chunk <= 0) ? 1u : prio_call;
        }
        const uint64_t chunks = (items + K_.chunk - 1) / K_.chunk;
        const uint64_t need_blocks = (chunks + (RT_BLOCK_THREADS / 64) - 1) / (RT_BLOCK_THREADS / 64);
        const uint32_t grid = (uint32_t)(need_blocks < grid_full ? need_blocks : grid_full);
        const uint64_t tail_items = 2ull * K_.chunk * grid * (RT_BLOCK_THREADS / 64);
        K_.tail_start = (uint32_t)(items > tail_items ? items - tail_items : 0);
        K_.chk_items = (uint32_t)items;
        K_.chk_out = tn.chk_shrink == 16 ? 0 : (uint64_t)ps.nframes * fstride;
        // Direct output of the launch's whole items. A frame is written
        // directly iff every item of it is whole: its pixel items cover all
        // its blocks ((f + 1) nb <= qpix), or its block items are whole (one
        // block per frame), or its tail samples are (spp == 1). Those frames
        // are a prefix of the launch; the collect folds the rest.
        K_.dout = nullptr;
        K_.dfull = 0;
        K_.collect_f0 = 0;
        if (direct && (uint64_t)ps.nframes * fstride < RT_INDEX_LIMIT) {
            const uint64_t nb = ps.nblocks;
            uint32_t fc = 0;
            while (fc < ps.nframes) {
                const uint64_t q0 = fc * nb, q1 = q0 + nb;
                const bool has_pix = q0 < K_.qpix, pix_whole = q1 <= K_.qpix;
                const bool has_blk = std::max<uint64_t>(q0, K_.qpix) < std::min<uint64_t>(q1, K_.qmain);
                const bool has_tail = q1 > K_.qmain;
                if ((has_pix && !pix_whole) || (has_blk && nb != 1) || (has_tail && p.spp != 1)) break;
                ++fc;
            }
            K_.dout = d_out + (size_t)ps.frame_begin * fstride;
            K_.dfull = K_.qpix / ps.nblocks;
            K_.collect_f0 = fc;
        }
        HIP_TRY_Q(hipEventRecord(f.ev[2 * i], stream));
        HIP_TRY_Q(rt_launch_render(&K_, cull ? ctx->d_grp_c : ctx->d_grp,
                                      cull ? ctx->d_sph_c : ctx->d_sph,
                                      cull ? ctx->d_shd_c : ctx->d_shd, f.d_pd,
                                      f.d_block_sums,
                                      f.d_counters + RT_CNT_WORK_OFFSET + i,
                                      reinterpret_cast<unsigned long long*>(f.d_counters),
                                      grid, stream));
        HIP_TRY_Q(hipEventRecord(f.ev[2 * i + 1], stream));
        const bool first_pass = ps.block_begin == 0;
        const bool last_pass = ps.block_begin + ps.nblocks == blocks_total;
        if (!tn.skip_collect)
            HIP_TRY_Q(rt_launch_collect(&K_, f.d_block_sums, f.d_acc, first_pass, last_pass,
                                           (float)p.spp, d_out + (size_t)ps.frame_begin * fstride,
                                           ctx->d_prog, prog_mode, prog_total, stream));
    }
    HIP_TRY_Q(hipMemcpyAsync(f.h_segs, f.d_counters, RT_CNT_U64 * sizeof(unsigned long long),
                                hipMemcpyDeviceToHost, stream));
#undef HIP_TRY_Q
    f.passes = (uint32_t)passes.size();
    f.short_math = K_.scene_fast;
    f.paths = (uint64_t)npix * p.spp * nframes;
    return RT_OK;
}

// Checked build (RT_CHECK_BOUNDS): the kernels' out-of-range index record
// since the last call (rt_kernels.hip RT_IDX), reset; a violation fails the
// call. The product library checks nothing here.
static int check_bounds(rt_ctx* ctx, const char* who) {
#ifdef RT_CHECK_BOUNDS
    unsigned int v[4] = {};
    if (rt_check_bounds_take(v) != 0) return fail(ctx, RT_ERR_DEVICE, "%s: bounds record unreadable", who);
    if (v[0])
        return fail(ctx, RT_ERR_DEVICE,
                    "%s: %u out-of-range index(es); first at site %u: index %u, bound %u", who, v[0],
                    v[1], v[2], v[3]);
#else
    (void)ctx;
    (void)who;
#endif
    return RT_OK;
}

// f.ev_t1 has been recorded after the frame's last operation.
static int finish(rt_ctx* ctx, Frame& f, rt_stats* st) {
    HIP_TRY(ctx, hipEventSynchronize(f.ev_t1));
    f.pending_stream = nullptr;
    {
        int rc = check_bounds(ctx, "render");
        if (rc) return rc;
    }
    for (int i = 0; i < RT_DBG_COUNTERS; ++i) ctx->dbg[i] = f.h_segs[2 + i];
    if (!st) return RT_OK;
    std::memset(st, 0, sizeof(*st));
    double kms = 0.0;
    for (uint32_t i = 0; i < f.passes; ++i) {
        float ms = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms, f.ev[2 * i], f.ev[2 * i + 1]));
        kms += ms;
    }
    float tms = 0.0f;
    HIP_TRY(ctx, hipEventElapsedTime(&tms, f.ev_t0, f.ev_t1));
    st->segments = f.h_segs[0];
    st->traced_segments = f.h_segs[1];
    st->sphere_tests = st->traced_segments * (uint64_t)ctx->n;
    st->paths = f.paths;
    st->kernel_ms = kms;
    st->total_ms = tms;
    st->kernel_launches = f.passes;
    st->short_math = f.short_math;
    // the waves' summed shader-clock ticks over their summed 100 MHz ticks
    const unsigned long long clk = f.h_segs[RT_CNT_CLOCK_OFFSET / 2],
                             real = f.h_segs[RT_CNT_CLOCK_OFFSET / 2 + 1];
    st->clock_ghz = real ? 0.1 * (double)clk / (double)real : 0.0;
    return RT_OK;
}

// The slot for the next frame, or nullptr (error set) when RT_MAX_PENDING
// frames are already in flight.
static Frame* next_slot(rt_ctx* ctx, const char* who) {
    if (ctx->npending >= RT_MAX_PENDING) {
        fail(ctx, RT_ERR_INVALID_ARG, "%s: %d calls already pending (rt_wait first)", who,
             RT_MAX_PENDING);
        return nullptr;
    }
    return &ctx->fr[(ctx->head + ctx->npending) % RT_MAX_PENDING];
}

static int no_pending(rt_ctx* ctx, const char* who) {
    if (ctx->npending)
        return fail(ctx, RT_ERR_INVALID_ARG, "%s: %u async call(s) not waited for", who,
                    ctx->npending);
    return RT_OK;
}

// Host-output bytes of one frame of `p` (rt_render_async; its staging buffer
// holds at least 16 bytes).
static size_t out_bytes(const rt_params* p) {
    const uint32_t K = p->shard_count ? p->shard_count : 1;
    const uint32_t rows = rt_shard_rows(p->height, p->row_block, K, p->shard_index);
    return (size_t)rows * p->width * sizeof(float4);
}

// The enqueue's completion: the optional device->host copy and the slot's end
// event, then the slot counts as pending. If either fails, the work already
// enqueued is waited for (nothing keeps running that no slot tracks).
static int commit(rt_ctx* ctx, Frame& f, hipStream_t s, void* host_dst, const void* dev_src,
                  size_t bytes) {
    hipError_t e = hipSuccess;
    if (bytes) e = hipMemcpyAsync(host_dst, dev_src, bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipEventRecord(f.ev_t1, s);
    if (e != hipSuccess) {
        hipStreamSynchronize(s);
        return fail(ctx, RT_ERR_DEVICE, "enqueue completion failed: %s", hipGetErrorString(e));
    }
    f.pending_stream = s;
    ++ctx->npending;
    return RT_OK;
}

int rt_reserve(rt_ctx* ctx, const rt_params* params, uint32_t nframes) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_reserve: ctx is NULL");
    int rc = no_pending(ctx, "rt_reserve");
    if (rc) return rc;
    for (int i = 0; i < RT_MAX_PENDING; ++i) {
        Frame& f = ctx->fr[i];
        rc = enqueue(ctx, f, nullptr, params, nframes, nullptr, nullptr, 0, 0.0f, true);
        if (rc) return rc;
        // and the host-output staging of rt_render / rt_render_async (one frame)
        rc = ensure(ctx, &f.d_out, &f.out_cap, std::max<size_t>(out_bytes(params), 16));
        if (rc) return rc;
    }
    return RT_OK;
}

int rt_render_device(rt_ctx* ctx, const rt_camera* camera, const rt_params* params,
                     float* out_rgba_device, void* stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_render_device: ctx is NULL");
    Frame* f = next_slot(ctx, "rt_render_device");
    if (!f) return RT_ERR_INVALID_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : f->stream;
    int rc = enqueue(ctx, *f, camera, params, 1, reinterpret_cast<float4*>(out_rgba_device), s);
    if (rc) return rc;
    return commit(ctx, *f, s, nullptr, nullptr, 0);
}

int rt_render_frames_device(rt_ctx* ctx, const rt_camera* camera, const rt_params* params,
                            uint32_t nframes, float* out_rgba_device, void* stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_render_frames_device: ctx is NULL");
    Frame* f = next_slot(ctx, "rt_render_frames_device");
    if (!f) return RT_ERR_INVALID_ARG;
    hipStream_t s = stream ? (hipStream_t)stream : f->stream;
    int rc = enqueue(ctx, *f, camera, params, nframes, reinterpret_cast<float4*>(out_rgba_device), s);
    if (rc) return rc;
    return commit(ctx, *f, s, nullptr, nullptr, 0);
}

int rt_render_async(rt_ctx* ctx, const rt_camera* camera, const rt_params* params, float* out_rgba) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_render_async: ctx is NULL");
    if (!out_rgba) return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_async: out_rgba is NULL");
    if (!params) return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_async: params is NULL");
    if (params->flags & RT_FLAG_IMAGE_OUT)
        return fail(ctx, RT_ERR_INVALID_ARG, "RT_FLAG_IMAGE_OUT is for device-output calls");
    if (!ctx->has_scene) return fail(ctx, RT_ERR_NO_SCENE, "rt_render before rt_set_scene");
    Frame* f = next_slot(ctx, "rt_render_async");
    if (!f) return RT_ERR_INVALID_ARG;
    const size_t bytes = out_bytes(params);
    int rc = ensure(ctx, &f->d_out, &f->out_cap, std::max<size_t>(bytes, 16));
    if (rc) return rc;
    rc = enqueue(ctx, *f, camera, params, 1, f->d_out, f->stream);
    if (rc) return rc;
    return commit(ctx, *f, f->stream, out_rgba, f->d_out, bytes);
}

int rt_host_register(rt_ctx* ctx, void* ptr, size_t bytes) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_host_register: ctx is NULL");
    if (!ptr || !bytes) return fail(ctx, RT_ERR_INVALID_ARG, "rt_host_register: empty buffer");
    for (const auto& r : ctx->host_regs)
        if (r.ptr == ptr) return fail(ctx, RT_ERR_INVALID_ARG, "rt_host_register: %p already registered", ptr);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    ctx->host_regs.push_back({ptr, bytes});
    return RT_OK;
}

int rt_host_unregister(rt_ctx* ctx, void* ptr) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_host_unregister: ctx is NULL");
    for (size_t i = 0; i < ctx->host_regs.size(); ++i) {
        if (ctx->host_regs[i].ptr != ptr) continue;
        int rc = quiesce(ctx);  // no pending copy may still target it
        if (rc) return rc;
        ctx->host_regs.erase(ctx->host_regs.begin() + (long)i);
        HIP_TRY(ctx, hipHostUnregister(ptr));
        return RT_OK;
    }
    return fail(ctx, RT_ERR_INVALID_ARG, "rt_host_unregister: %p is not registered", ptr);
}

int rt_wait(rt_ctx* ctx, rt_stats* stats) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_wait: ctx is NULL");
    if (!ctx->npending) return fail(ctx, RT_ERR_INVALID_ARG, "rt_wait: nothing pending");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    Frame& f = ctx->fr[ctx->head];
    ctx->head = (ctx->head + 1) % RT_MAX_PENDING;
    --ctx->npending;
    return finish(ctx, f, stats);
}

int rt_render(rt_ctx* ctx, const rt_camera* camera, const rt_params* params, float* out_rgba,
              rt_stats* stats) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_render: ctx is NULL");
    int rc = no_pending(ctx, "rt_render");
    if (rc) return rc;
    rc = rt_render_async(ctx, camera, params, out_rgba);
    if (rc) return rc;
    return rt_wait(ctx, stats);
}

int rt_render_progressive(rt_ctx* ctx, const rt_camera* camera, const rt_params* params,
                          int reset, float* out_rgba, uint64_t* total_spp) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_render_progressive: ctx is NULL");
    if (!out_rgba || !params)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_render_progressive: NULL argument");
    int rc = no_pending(ctx, "rt_render_progressive");
    if (rc) return rc;
    Frame& f = ctx->fr[ctx->head];
    const uint32_t K = params->shard_count ? params->shard_count : 1;
    const uint32_t B = params->row_block ? params->row_block : 1;
    const uint32_t rows = rt_shard_rows(params->height, B, K, params->shard_index);
    const size_t npix = (size_t)rows * params->width;
    const size_t bytes = npix * sizeof(float4);
    // the running sum belongs to one image geometry; another one restarts it
    const uint64_t key = ((uint64_t)params->width << 40) ^ ((uint64_t)params->height << 20) ^
                         ((uint64_t)B << 10) ^ ((uint64_t)K << 5) ^ params->shard_index;
    if (key != ctx->prog_key || !ctx->d_prog) reset = 1;
    rc = ensure(ctx, &ctx->d_prog, &ctx->prog_cap, bytes ? bytes : 16);
    if (rc) return rc;
    rc = ensure(ctx, &f.d_out, &f.out_cap, bytes ? bytes : 16);
    if (rc) return rc;
    const uint64_t total = (reset ? 0 : ctx->prog_total) + params->spp;
    rc = enqueue(ctx, f, camera, params, 1, f.d_out, f.stream, reset ? 1 : 2, (float)total);
    if (rc) return rc;
    if (bytes)
        HIP_TRY(ctx, hipMemcpyAsync(out_rgba, f.d_out, bytes, hipMemcpyDeviceToHost, f.stream));
    HIP_TRY(ctx, hipEventRecord(f.ev_t1, f.stream));
    HIP_TRY(ctx, hipEventSynchronize(f.ev_t1));
    rc = check_bounds(ctx, "rt_render_progressive");
    if (rc) return rc;
    ctx->prog_total = total;
    ctx->prog_key = key;
    if (total_spp) *total_spp = total;
    return RT_OK;
}

int rt_encode_srgb8(rt_ctx* ctx, const float* rgba_device, uint8_t* rgba8_device, uint64_t npix,
                    void* stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_encode_srgb8: ctx is NULL");
    if (npix == 0) return RT_OK;
    if (!rgba_device || !rgba8_device)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_encode_srgb8: NULL buffer");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    HIP_TRY(ctx, rt_launch_srgb8(reinterpret_cast<const float4*>(rgba_device),
                                 reinterpret_cast<uchar4*>(rgba8_device), npix, s));
    if (!stream) HIP_TRY(ctx, hipStreamSynchronize(s));
    return RT_OK;
}

int rt_acquire(rt_ctx* ctx, void* stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_acquire: ctx is NULL");
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    // a few waves per CU: every CU (and so every XCD's L2) runs the fence
    HIP_TRY(ctx, rt_launch_acquire((uint32_t)std::max(ctx->cu_count, 1) * 8u, s));
    if (!stream) HIP_TRY(ctx, hipStreamSynchronize(s));
    return RT_OK;
}

static int assemble(rt_ctx* ctx, const char* fn, const float* gathered_device, uint32_t max_rows,
                    uint32_t frames, float* image_device, uint32_t width, uint32_t height,
                    uint32_t row_block, uint32_t shard_count, void* stream) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "%s: ctx is NULL", fn);
    if (!gathered_device || !image_device || width == 0 || height == 0 || shard_count == 0 ||
        frames == 0 || frames > 65535)
        return fail(ctx, RT_ERR_INVALID_ARG, "%s: bad arguments", fn);
    const uint32_t B = row_block ? row_block : 1;
    for (uint32_t k = 0; k < shard_count; ++k)
        if (rt_shard_rows(height, B, shard_count, k) > max_rows)
            return fail(ctx, RT_ERR_INVALID_ARG, "%s: shard %u has more than %u rows", fn, k,
                        max_rows);
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    HIP_TRY(ctx, rt_launch_assemble(reinterpret_cast<const float4*>(gathered_device), max_rows,
                                    frames, reinterpret_cast<float4*>(image_device), width,
                                    height, B, shard_count, s));
    if (!stream) HIP_TRY(ctx, hipStreamSynchronize(s));
    return RT_OK;
}

int rt_assemble_shards(rt_ctx* ctx, const float* gathered_device, uint32_t max_rows,
                       float* image_device, uint32_t width, uint32_t height, uint32_t row_block,
                       uint32_t shard_count, void* stream) {
    return assemble(ctx, "rt_assemble_shards", gathered_device, max_rows, 1u, image_device, width,
                    height, row_block, shard_count, stream);
}

int rt_assemble_shard_frames(rt_ctx* ctx, const float* gathered_device, uint32_t max_rows,
                             uint32_t frames, float* image_device, uint32_t width,
                             uint32_t height, uint32_t row_block, uint32_t shard_count,
                             void* stream) {
    return assemble(ctx, "rt_assemble_shard_frames", gathered_device, max_rows, frames,
                    image_device, width, height, row_block, shard_count, stream);
}

int rt_intersect(rt_ctx* ctx, const float* rays, uint32_t n, int32_t* hit_index, float* hit_t) {
    return rt_intersect_ex(ctx, rays, n, 0u, hit_index, hit_t);
}

int rt_intersect_ex(rt_ctx* ctx, const float* rays, uint32_t n, uint32_t flags, int32_t* hit_index,
                    float* hit_t) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "rt_intersect: ctx is NULL");
    if (!ctx->has_scene) return fail(ctx, RT_ERR_NO_SCENE, "rt_intersect before rt_set_scene");
    if (n == 0) return RT_OK;
    if (!rays || !hit_index || !hit_t)
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_intersect: NULL array");
    ctx->isect_tiles[0] = ctx->isect_tiles[1] = 0;
    int rc = no_pending(ctx, "rt_intersect");
    if (rc) return rc;
    const bool cull = (flags & RT_FLAG_CULL) != 0;
    if ((rc = scene_ready(ctx, flags)) != RT_OK) return rc;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    void* buf = nullptr;
    const size_t rb = sizeof(float) * 6 * (size_t)n, ob = sizeof(int32_t) * (size_t)n;
    const size_t cb = (rb + 2 * ob + 15) & ~(size_t)15;  // the tile counters after the outputs
    HIP_TRY(ctx, hipMalloc(&buf, cb + 2 * sizeof(unsigned long long)));
    char* b = (char*)buf;
    unsigned long long* tiles = (unsigned long long*)(b + cb);
    hipError_t e = hipMemcpyAsync(b, rays, rb, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipMemsetAsync(tiles, 0, 2 * sizeof(unsigned long long), ctx->stream);
    // the brute-force walk takes the render's filter: the matrix-core tiles
    // when the scene fits them (unless RT_FLAG_VALU_FILTER)
    MfScene mf = {};
#ifdef RT_MFMA_FILTER
    if (!cull && ctx->mf_ok && !(flags & RT_FLAG_VALU_FILTER)) mf = mf_scene(ctx);
#endif
    if (e == hipSuccess)
    {
        e = rt_launch_intersect(cull ? ctx->d_grp_c : ctx->d_grp, cull ? ctx->d_sph_c : ctx->d_sph,
                                cull ? ctx->ngroups_c : ctx->ngroups,
                                ctx->scene_fast && ctx->tune.fast_exact ? 1u : 0u,
                                (const float*)b, n, (int*)(b + rb), (float*)(b + rb + ob),
                                cull ? ctx->d_bnd_c : nullptr, cull ? ctx->d_perm_c : nullptr,
                                cull ? ctx->nclusters_c : 0u, &mf, tiles, ctx->stream);
    }
    if (e == hipSuccess)
        e = hipMemcpyAsync(hit_index, b + rb, ob, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(hit_t, b + rb + ob, ob, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(ctx->isect_tiles, tiles, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    hipFree(buf);
    if (e != hipSuccess)
        return fail(ctx, RT_ERR_DEVICE, "rt_intersect: %s", hipGetErrorString(e));
    return check_bounds(ctx, "rt_intersect");
}

// Internal (not in include/rt_hip.h; tests/test_cull.py, CPU): the culled
// layout of a sphere list as build_cull makes it, without a device.
// counts[0..3] = (groups, clusters, records, supers); perm (records entries) and bnd
// ((supers + clusters) * 32 floats, supers = ceil(clusters / 8): per super
// its 8 cluster bounds, then per cluster its 8 group bounds, each record
// Cx[8] Cy[8] Cz[8] S_B[8]) are filled when their capacities suffice. Returns 0, or -1 on a NULL argument.
int rt_debug_cull_layout(const rt_sphere* spheres, uint32_t n, uint32_t* counts, uint32_t* perm,
                         uint32_t perm_cap, float* bnd, uint32_t bnd_cap) {
    if (!counts || (n && !spheres)) return -1;
    std::vector<float4> q(n);
    std::vector<float> S(n);
    std::vector<float2> rm(n);
    for (uint32_t i = 0; i < n; ++i) pack_record_to(spheres[i], q[i], S[i], rm[i]);
    CullLayout L;
    cull_layout(q.data(), S.data(), rm.data(), n, L);
    counts[0] = L.ngroups;
    counts[1] = L.nclusters;
    counts[2] = L.nrec;
    counts[3] = L.nsupers;
    if (perm && perm_cap >= L.nrec) std::copy(L.perm.begin(), L.perm.end(), perm);
    if (bnd && bnd_cap >= L.bnd.size() * 4) std::memcpy(bnd, L.bnd.data(), L.bnd.size() * sizeof(float4));
    return 0;
}

// Internal (not in include/rt_hip.h; tests/test_gpu_parity.py): matrix-core
// layouts this context built whole and updated in place (mf_update).
int rt_debug_mf_rebuilds(const rt_ctx* ctx, uint64_t* out2) {
    if (!ctx || !out2) return -1;
    out2[0] = ctx->mf_builds;
    out2[1] = ctx->mf_inplace;
    return 0;
}

#ifdef RT_MFMA_FILTER
// Internal, host only (not in include/rt_hip.h; tests/test_scene_update.py):
// the matrix-core layout of spheres s0, then the spheres idx[0..k) replaced
// by s1[0..k) as rt_update_spheres + the next render would apply them. ms3:
// the layout built from scratch for s0, the in-place update, and a build from
// scratch of the updated list (what the fallback costs), in ms of host time.
// Returns 1 when the update was applied in place AND its layout equals, byte
// for byte, the layout filled from scratch in the same walk order; 0 when it
// falls back to a full rebuild; -1 on a mismatch; -2 when s0 does not take
// the matrix-core walk.
int rt_debug_mf_update(const rt_sphere* s0, uint32_t n, const uint32_t* idx, const rt_sphere* s1,
                       uint32_t k, double* ms3) {
    if (!s0 || !n || (k && (!idx || !s1))) return -2;
    std::vector<float4> q(n);
    std::vector<float> S(n);
    std::vector<float2> rm(n);
    for (uint32_t i = 0; i < n; ++i) pack_record_to(s0[i], q[i], S[i], rm[i]);
    auto now = [] {
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
    };
    MfHost H;
    double t = now();
    if (!mf_build(q.data(), S.data(), n, H)) return -2;
    const double t_full0 = now() - t;
    std::vector<uint32_t> moved;
    for (uint32_t j = 0; j < k; ++j) {
        if (idx[j] >= n) return -2;
        pack_record_to(s1[j], q[idx[j]], S[idx[j]], rm[idx[j]]);
        moved.push_back(idx[j]);
    }
    std::sort(moved.begin(), moved.end());
    moved.erase(std::unique(moved.begin(), moved.end()), moved.end());
    std::vector<uint32_t> tb, tc, tp;
    t = now();
    const bool inplace = mf_update(H, q.data(), n, moved, tb, tc, tp);
    const double t_upd = now() - t;
    MfHost F;
    t = now();
    mf_build(q.data(), S.data(), n, F);
    const double t_full1 = now() - t;
    if (ms3) {
        ms3[0] = t_full0;
        ms3[1] = t_upd;
        ms3[2] = t_full1;
    }
    if (!inplace) return 0;
    MfHost G;
    if (!mf_fill(q.data(), n, H.order, H.sq, G)) return -1;
    const bool same = G.ok == H.ok && G.sq == H.sq && G.nblk == H.nblk && G.npos == H.npos &&
                      G.nchunk == H.nchunk && G.top == H.top && G.order == H.order && G.A == H.A &&
                      G.B == H.B && G.mperm == H.mperm && G.iperm == H.iperm && G.bqmax == H.bqmax &&
                      G.msph.size() == H.msph.size() &&
                      std::memcmp(G.msph.data(), H.msph.data(), G.msph.size() * sizeof(float4)) == 0;
    return same ? 1 : -1;
}
#endif

// Internal (not in include/rt_hip.h): the first 16 diagnostic counters of the
// last waited call; all zero unless the library was built with -DRT_PROFILE.
int rt_debug_counters(const rt_ctx* ctx, uint64_t* out16) {
    if (!ctx || !out16) return RT_ERR_INVALID_ARG;
    for (int i = 0; i < 16; ++i) out16[i] = ctx->dbg[i];
    return RT_OK;
}

// Internal: all RT_DBG_COUNTERS (32) diagnostic counters of the last waited
// call (RT_PROFILE builds; rt_dev_intersect.h "Prof" lists them).
int rt_debug_counters32(const rt_ctx* ctx, uint64_t* out32) {
    if (!ctx || !out32) return RT_ERR_INVALID_ARG;
    for (int i = 0; i < RT_DBG_COUNTERS; ++i) out32[i] = ctx->dbg[i];
    return RT_OK;
}

// Internal (tests/test_gpu_intersect.py): the last rt_intersect's matrix-core
// walk, out2 = (block-half tiles walked, tiles a walk without block bounds
// visits) summed over its waves; (0, 0) when it took the VALU walk or the
// culled list. Product build: the batch-query kernel counts, the render does not.
int rt_debug_intersect_tiles(const rt_ctx* ctx, uint64_t* out2) {
    if (!ctx || !out2) return RT_ERR_INVALID_ARG;
    out2[0] = ctx->isect_tiles[0];
    out2[1] = ctx->isect_tiles[1];
    return RT_OK;
}

// Internal (not in include/rt_hip.h): set one A/B or fault-injection knob of
// ctx (struct Tuning above; names: scratch_bytes, split_all, tail_split, tail
// "a4,a2,a1", prefetch, prio_mode, prio_shift, wg_per_cu, wide_max,
// fast_exact, fail_alloc_after, block_region, block_align, block_lead, wave_chunk, chk_shrink, direct_out, skip_collect). name == NULL restores every default. Used by
// the tests and tools/ only; the product path never calls it.
int rt_debug_tune(rt_ctx* ctx, const char* name, const char* value) {
    if (!ctx) return RT_ERR_INVALID_ARG;
    if (!name) {
        ctx->tune = Tuning();
        return RT_OK;
    }
    if (!value || !tune_set(ctx->tune, name, value))
        return fail(ctx, RT_ERR_INVALID_ARG, "rt_debug_tune: bad knob %s=%s", name,
                    value ? value : "(null)");
    return RT_OK;
}

// Internal: device allocations the ctx has made so far (tests: a reserved
// render allocates nothing).
uint64_t rt_debug_alloc_count(const rt_ctx* ctx) { return ctx ? ctx->allocs : 0; }

const char* rt_last_error(const rt_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

}  // extern "C"
