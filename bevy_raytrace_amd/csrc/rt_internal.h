// rt_internal.h — shared between the C-ABI host code and the kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt_hip.h"

#define RT_BLOCK_THREADS 256  // 4 waves per workgroup
#ifndef RT_WAVE_CHUNK
#define RT_WAVE_CHUNK 64      // work items a wave takes per atomic
#endif
#ifndef RT_WAVE_CHUNK_TAIL
// ... in the last 2 x 64 x waves items of the queue. Round 5, same box
// against 16 (profiles/r05/chunk_tail/): the N = 8 row shard -0.6 / -0.75 %
// (two calls), the N = 4 / 2 shards -0.25 % (c54), headline and 4K within
// +-0.1 %, 10k spheres +0.1 % (noise);
// 4 / 8 slower (shard +1.9 / +0.3 %, headline +0.4 / +0.2 %), 64: shard
// -0.4 %, headline -0.2 %, 10k +1 %
#define RT_WAVE_CHUNK_TAIL 32
#endif
// Counter block at the start of the ctx's counter buffer (u32 words):
// [0,4) two u64 segment counters, [4,68) 32 u64 diagnostic counters
// (RT_PROFILE builds), [68,72) two u64 clock sums (the render waves'
// s_memtime and s_memrealtime deltas: rt_stats.clock_ghz), [72, ...) one u32
// work counter per pass.
#define RT_DBG_COUNTERS 32
#define RT_CNT_CLOCK_OFFSET (4 + 2 * RT_DBG_COUNTERS)
#define RT_CNT_WORK_OFFSET (RT_CNT_CLOCK_OFFSET + 4)
#define RT_CNT_U64 (2 + RT_DBG_COUNTERS + 2)  // u64 counters copied back per call (segments, diagnostics, clocks)
#define RT_TAIL_ITEM 0x80000000u  // PathState::item flag: a tail item (per-sample slots)
// PathState::item / slot-buffer entry flag: the item covers every sample of
// its (frame, pixel) and writes the output pixel itself (KParams::dout); the
// entry's other bits are the output index f * dstride + pixel (< 2^30)
#define RT_DIRECT_ITEM 0x40000000u
#define RT_INDEX_LIMIT 0x40000000u  // slots, pixels and direct indices stay below it
// uint4 entries of one 32-sphere block of matrix-core A fragments: A0 for 64
// lanes + A1 for lanes 32..63 (lanes 0..31 of A1 equal their A0; build_mfma)
#define RT_MF_BLK 96u
#define RT_MF_BCHUNK 160u  // uint4 entries per bound chunk: line rows K 0..31, forward rows K 0..7
#define RT_GROUP 8            // spheres per filter group (SoA, 128 B)
#define RT_MF_SPH_LDS_MAX 512 // rt_render_kernel: the walk's records held in LDS (8 KB, <= 16 blocks)
#ifndef RT_SLOT_BUF_CAP
#define RT_SLOT_BUF_CAP 32    // slot-store buffer entries per wave (rt_kernels.hip)
#endif
#ifndef RT_SLOT_BUF_CAP_LDS
#define RT_SLOT_BUF_CAP_LDS 24  // ... in rt_render_kernel, whose LDS also holds the walk's records
#endif
#ifndef RT_CQ_CAP
#define RT_CQ_CAP 8           // candidate-queue entries per lane (LDS)
#endif
#ifndef RT_MIN_WAVES_PER_SIMD
#define RT_MIN_WAVES_PER_SIMD 6
#endif
#ifndef RT_MIN_WAVES_PER_SIMD_CULL
#define RT_MIN_WAVES_PER_SIMD_CULL 6
#endif

// Unsigned 32-bit division by a run-time invariant d >= 1 as a multiply-high
// (Granlund & Montgomery 1994, Fig. 4.1): exact for every 32-bit n.
struct FastDiv {
    uint32_t m, sh1, sh2, d;
};

// Kernel parameters (by value; lands in SGPRs). Camera constants are
// precomputed on the host exactly as generate.wgsl:67-95 computes them.
// The matrix-core walk's scene (RT_MFMA_FILTER builds; rt_api.cpp build_mfma):
// the list in the culled list's spatial order (large spheres first, the rest
// in k-d order of their centres) as f16 A fragments of
// v_mfma_f32_32x32x16_f16, RT_MF_BLK uint4 per 32-sphere block; per chunk of
// 32 blocks the blocks' bounding spheres as fragments of the same layout (2 x
// 64 uint4), tested against the wave's rays on the matrix cores so that a
// half-wave skips every block none of its rays passes near
// (rt_dev_intersect.h intersect_world_mfma); the records the drain's exact
// tests read, in the walk's order; and the walk position -> original index
// map (exact ties, the result).
struct MfScene {
    const uint4* A;         // null: no matrix-core walk
    const uint4* B;         // null: every block is walked (knob mf_cull 0)
    const float4* sph;      // (cx, cy, cz, r^2) in the walk's order, nblk * 32 records
    const uint32_t* perm;   // walk position -> original sphere index
    const float4* shd;      // shading records in the walk's order, 2 per position (render)
    const uint32_t* iperm;  // original sphere index -> walk position
    uint32_t nblk;          // 32-sphere blocks (<= 2048)
    uint32_t top;           // 1: B holds one more chunk after the ceil(nblk / 16) of block
                            // bounds, the chunk-level bounds (row j = chunk j; 2..32 chunks)
    float qs, abs;          // 2^sq (quadratic features' ray-side scale), threshold margin
};

struct KParams {
    uint32_t width, height, spp, max_depth, frame0;
    uint32_t row_block, shard_count, shard_index;
    uint32_t npix;         // pixels of this shard (rows * width)
    uint32_t block_begin;  // first sample block of this pass
    uint32_t nblocks;      // sample blocks in this pass
    // Work queue of one launch. The launch covers nframes frames (samples
    // sample_base + f*spp + [0, spp) of launch frame f; the seed frame is
    // frame0 + that) x blocks [block_begin, block_begin + nblocks) of each.
    // Its (frame, block) pairs q = f*nblocks + b: pairs q < qmain are the main
    // part, dealt as pixel items for q < qpix -- one item per (frame, pixel),
    // items [0, main_pix = ceil(qpix / nblocks) * npix), covering that
    // frame's pairs below qpix; the lane folds their block sums and stores
    // the fold at slot = f*npix + k -- then as block items for q in
    // [qpix, qmain): items [main_pix, main_all), one (pair, pixel) each,
    // storing the block's sum at slot = main_pix + r*npix + k (short items,
    // so no lane holds a long pixel item when the queue runs dry). The rest
    // -- the launch's tail, launch samples g = f*spp + s in [g0, g_end) -- is
    // dealt as shrinking items: 4-sample items over [g0, g1), 2-sample over
    // [g1, g2), single samples over [g2, g_end); a tail item stores every
    // sample's colour at slot main_all + (g - g0)*npix + k. Which item index
    // maps to which (frame / pair / sample group, pixel) is item_order's
    // business (below); the slots, and so the fold, do not depend on it.
    // rt_collect_kernel folds them per pixel in block / sample order.
    uint32_t nframes, sample_base, qmain, main_all;
    uint32_t qpix, main_pix;
    // lead items (knob block_lead): frames f >= fp (past the pixel pairs) with
    // main pairs get one pixel item of their first min(lead, ...) blocks, in
    // [0, main_pix) too; the block items are then the other pairs in
    // [qpix, qmain), in pair order: c0 = fp*nblocks - qpix of the pixel
    // region's last frame, then nblocks - lead per later frame (div_nbl)
    uint32_t fp, lead, c0;
    FastDiv div_nbl;
    // the lead items' place: items [main_fp = fp*npix, main_pix) after the
    // pixel items, grouped by 2^lead_group_shift pixels (0: pixel-major),
    // frame-major in the group (div_nlead: by the fl - fp lead frames)
    uint32_t main_fp, lead_group_shift;
    FastDiv div_nlead;
    uint32_t g0, g1, g2, g_end;
    uint32_t ti1, ti2, tail_items;  // tail item offsets of the 2- and 1-sample regions, count
    FastDiv div_nblocks;
    // a wave with at most wide_max live rays traces them sphere-parallel
    // (intersect_wide): the tail of the queue, where waves empty out
    uint32_t wide_max;
    uint32_t nspheres;
    uint32_t ngroups;      // padded sphere groups of RT_GROUP (see rt_set_scene)
    uint32_t scene_fast;   // 1: spheres inside the short-math domain (rt_api.cpp scene_fast_ok)
    uint32_t flags;
    float T[16];           // camera transform, column-major
    float tan_half, focus_plane, aspect, half_w, half_h;
    float coc;             // lens_focal_length / (2 * fstop), generate.wgsl:97 (thin-lens flag)
    FastDiv div_npix, div_width, div_row_block;
    uint32_t tail_start;   // queue position from which waves take RT_WAVE_CHUNK_TAIL items
    uint32_t chunk;        // items a wave takes per atomic before tail_start (rt_api.cpp: by the call)
    // processing order of a pass's pixels: tile_h x tile_w tiles (rows of
    // tiles, each tile row-major inside), then the rows % tile_h leftover rows
    // row-major (rt_dev_path.h order_to_pixel)
    uint32_t tile_h, tile_w;
    uint32_t tile_full_rows;  // rows / tile_h
    uint32_t tile_full_cols;  // width / tile_w
    uint32_t tile_wrem;       // width % tile_w
    FastDiv div_thw, div_tp, div_tw, div_wrem;  // by tile_h * width, tile_h * tile_w, tile_w, tile_wrem
    uint32_t prefetch;  // 1: waves prefetch their next work chunk (knob prefetch)
    uint32_t prio_mode;   // s_setprio rotation (knob prio_mode): 0 off, 1 by iteration, 3 by wall time
    uint32_t prio_shift;  // mode 3: one step per 2^prio_shift ticks of 10 ns (knob prio_shift)
    // culled list (RT_FLAG_CULL; rt_render_cull_kernel): grp / sph / sph_rm
    // are then the permuted arrays, nspheres / ngroups their padded sizes
    const float4* bnd;      // bound records, SoA like a group: per super its 8 cluster bounds,
                            // then per cluster its 8 group bounds; null = brute force
    const uint32_t* perm;   // permuted position -> original sphere index (ties)
    uint32_t nclusters;
    uint32_t cull_supers;   // 1: test the cluster bounds (many clusters); 0: walk every cluster
    const float4* acc_in;   // passes after the first (block_begin > 0): the fold so far, per pixel
    // matrix-core filter (RT_MFMA_FILTER builds, brute-force walk; mf.A null:
    // the packed VALU filter)
    MfScene mf;
    // queue order (knob item_order, bits; default 7, groups of 4): bit 0 the block items
    // and the tail items, bit 1 the pixel items, pixel-major
    // (consecutive items: one pixel's pairs / samples / frames) instead of
    // pair- / sample- / frame-major (consecutive items: neighbouring pixels);
    // bit 2 (npix % 8 == 0 only) every region grouped: 8 neighbouring
    // pixels' items back to back, frame / pair / sample-group major within
    // the group (rt_dev_path.h grouped_split)
    uint32_t item_order;
    uint32_t pix_group_shift;  // grouped order (bit 2): log2 of the pixel group (2 or 3)
    FastDiv div_nfpix; // by fp (frames with pixel pairs; main_fp / npix)
    FastDiv div_nreg;  // by the block items per pixel (qmain - qpix without lead items)
    // by the sample groups per pixel of the tail regions: (g1 - g0 + 3) / 4,
    // (g2 - g1 + 1) / 2, g_end - g2 (4-, 2-, 1-sample items)
    FastDiv div_ng4, div_ng2, div_ng1;
    // Sizes of the buffers the kernels index, in records: the bounds the
    // RT_CHECK_BOUNDS build checks every computed index against (rt_kernels.hip
    // RT_IDX; the product build reads none of them).
    uint32_t chk_nsph;   // sph / grp records (padded list)
    uint32_t chk_nrm;    // shading records (2 float4 each)
    uint32_t chk_wsph, chk_wrm;  // the same in the matrix-core walk's order (mf.sph, mf.shd)
    uint32_t chk_items;  // work items of the launch (main_all + tail_items)
    uint64_t chk_slots;  // block_sums slots
    uint64_t chk_out;    // float4 pixels behind the launch's output pointer
    // Direct output: an item that covers every
    // sample of its (frame, pixel) -- a pixel item of a launch frame below
    // dfull, a block item when the pass has one sample block (dwhole_blk), a
    // tail item when spp == 1 (dwhole_tail) -- writes out = its fold / spp
    // (rt_collect_kernel's own arithmetic, so the bits are the collect's) at
    // dout + f * dstride + pixel through the wave's slot buffer: no slot, no
    // slot re-read, no collect for its frame. Frames are either wholly direct
    // or wholly collected (rt_api.cpp); the collect runs over launch frames
    // [collect_f0, nframes). dout null: off.
    float4* dout;
    uint32_t dfull, dwhole_blk, dwhole_tail;
    uint32_t dstride;     // float4 pixels per output frame (the image, or the packed rows)
    uint32_t dsys;        // 1: the output is another device's image (RT_FLAG_IMAGE_OUT):
                          // the collect's system-scope write-through stores + a
                          // release per wave; no direct output then
    uint32_t collect_f0;  // first launch frame rt_collect_kernel folds
    uint32_t dsys_release;  // dsys: each collect wave also issues a system-scope release (knob)
};

// Row block b of the image -> owning shard (rt_params: serpentine deal).
__host__ __device__ inline uint32_t rt_block_owner(uint32_t b, uint32_t K) {
    const uint32_t g = b / K, i = b - g * K;
    return (g & 1u) ? K - 1u - i : i;
}
// j-th block of shard k -> image row block.
__host__ __device__ inline uint32_t rt_shard_block(uint32_t j, uint32_t K, uint32_t k) {
    return j * K + ((j & 1u) ? K - 1u - k : k);
}

extern "C" {
hipError_t rt_launch_render(const KParams* P, const float4* grp, const float4* sph,
                            const float4* shd, const float4* pd,
                            float4* block_sums,
                            uint32_t* work_counter, unsigned long long* seg_counter, uint32_t grid,
                            hipStream_t stream);
hipError_t rt_launch_collect(const KParams* P, const float4* block_sums,
                             float4* acc, int first_pass, int last_pass, float spp, float4* out,
                             float4* prog, int prog_mode, float prog_total, hipStream_t stream);
hipError_t rt_launch_srgb8(const float4* in, uchar4* out, uint64_t npix, hipStream_t stream);
hipError_t rt_launch_acquire(uint32_t blocks, hipStream_t stream);
hipError_t rt_launch_assemble(const float4* gathered, uint32_t max_rows, uint32_t frames,
                              float4* image, uint32_t width, uint32_t height, uint32_t row_block,
                              uint32_t shard_count, hipStream_t stream);
hipError_t rt_launch_intersect(const float4* grp, const float4* sph, uint32_t ngroups,
                               uint32_t scene_fast, const float* rays, uint32_t n, int* out_i, float* out_t,
                               const float4* bnd, const uint32_t* perm, uint32_t nclusters,
                               const MfScene* mf, unsigned long long* tile_cnt, hipStream_t stream);
hipError_t rt_render_occupancy(int* blocks_per_cu, int* blocks_per_cu_cull);
hipError_t rt_launch_primary(const KParams* P, float4* pd, hipStream_t stream);
#ifdef RT_CHECK_BOUNDS
int rt_check_bounds_take(unsigned int out[4]);  // checked build: read and reset the record
#endif
}
