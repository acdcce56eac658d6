// rt_dev_path.h -- lane path state, work items and shading (shade.wgsl:105-258)
// (included by rt_kernels.hip only: one translation unit, device code)
#pragma once

// Lane state of one in-flight path.
struct PathState {
    v3 o, d;            // current ray
    v3 color;           // throughput (intersection.color, clear.wgsl:86)
    v3 bsum;            // sum of finished samples of the current block
    v3 nseed;           // normalize(seed)
    float seedx;        // seed.x (dielectric Schlick test)
    uint32_t pix;       // global pixel x + W*y (the seed's pixel term, shade.wgsl:216-218)
    uint32_t item;      // main item: its output slot, or RT_DIRECT_ITEM | output index;
                        // tail: RT_TAIL_ITEM [| RT_DIRECT_ITEM] | pixel
    uint32_t s, s_end;  // current sample, end of the current sample block
    uint32_t bounce;
};

// Per-lane item state that changes at most once per sample, kept in LDS (no
// VGPRs: the kernel sits at its occupancy's register limit), one record per lane so a single
// VGPR address (+ immediate offsets) reaches every field: the pixel's primary
// direction, the item's running fold of its block sums (xyz; w != 0 once a
// block was folded), the primary hit (reuse mode) and the end of its samples.
struct LaneLds {
    float4 pd;        // primary direction of the lane's pixel (xyz)
    float4 acc;       // fold of the item's block sums so far
    float2 cache;     // primary hit (index bits, t) -- primary-hit reuse only
    uint32_t iend;    // end of the item's samples
    uint32_t pad;
};
typedef LaneLds* ItemLds;  // the lane's own record

// New sample s of the lane's pixel: seed (shade.wgsl:216-218; u32 wrap, so
// (x + W*y) + W*H*frame is the reference's index), primary ray
// (generate.wgsl:109-129; origin = camera translation, direction from the
// pixel table since it depends on the pixel only), throughput 1 (clear.wgsl:86).
__device__ __forceinline__ void start_sample(const KParams& P, PathState& st, ItemLds L) {
    const uint32_t frame = P.frame0 + st.s;
    const uint32_t idx = st.pix + (P.width * P.height) * frame;
    const v3 seed = hash3(idx);
    st.seedx = seed.x;
    st.nseed = normalize_seed(seed);
    // (with the opt-in camera sampling the main loop replaces this primary
    // ray before tracing it: one call site for sampled_primary_ray)
    st.o = mk(0.0f + P.T[12], 0.0f + P.T[13], 0.0f + P.T[14]);
    const float4 pd = L->pd;
    st.d = mk(pd.x, pd.y, pd.z);
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
// (row-major). Order: tile_h x tile_w tiles (8 x 8; a shard's tiles one row
// block high, rt_api.cpp), so the 64 lanes of a wave trace a compact patch of
// the image (coherent rays: fewer sphere groups with a candidate in the wave);
// tile rows run bottom-up so the queue ends on the cheap sky rows.
__device__ __forceinline__ uint32_t order_to_pixel(const KParams& P, uint32_t k) {
    k = P.npix - 1 - k;
    const uint32_t W = P.width, th = P.tile_h, tw = P.tile_w;
    const uint32_t tiled = P.tile_full_rows * th * W;
    uint32_t x, r;
    if (k < tiled) {
        const uint32_t tr = fdiv(k, P.div_thw);
        const uint32_t rem = k - tr * th * W;
        const uint32_t tx = fdiv(rem, P.div_tp);
        if (tx < P.tile_full_cols) {
            const uint32_t j = rem - tx * th * tw;
            const uint32_t jr = fdiv(j, P.div_tw);
            x = tx * tw + (j - jr * tw);
            r = tr * th + jr;
        } else {  // the narrow last tile of the tile row
            const uint32_t j = rem - P.tile_full_cols * th * tw;
            const uint32_t jr = fdiv(j, P.div_wrem);
            x = P.tile_full_cols * tw + (j - jr * P.tile_wrem);
            r = tr * th + jr;
        }
    } else {
        const uint32_t j = k - tiled;
        const uint32_t jr = fdiv(j, P.div_width);
        x = j - jr * W;
        r = P.tile_full_rows * th + jr;
    }
    return r * W + x;
}

// Pixel table entry (rt_primary_kernel), 16 B: the k-th pixel of the
// processing order -> its primary direction (xyz) and x + W*y (w, as bits).
struct PixelEntry {
    float4 d;
};

// Work item -> samples, pixel. The launch's main pairs (q = f*nblocks + b <
// qmain) are dealt in two regions. Pairs q < qpix as pixel items (item <
// main_pix): (frame f, pixel k) with all of f's pairs below qpix, in block
// order -- the lane sums each block of RT_SAMPLE_BLOCK samples in registers
// (st.s_end = the block's end), folds the block sums in block order (acc =
// bsum_0; acc = acc + bsum_b, rt_collect_kernel's fold) and stores the fold
// once, at slot f*npix + k. Pairs [qpix, qmain) as block items (item <
// main_all): one block of one pixel, its sum stored at slot main_pix +
// r*npix + k (r = q - qpix) -- short items at the end of the main part, so
// no lane holds a long pixel item when the queue runs dry. With lead items
// (P.lead > 0, knob block_lead) every frame f >= fp with main pairs also has
// a pixel item, of its first min(lead, ...) blocks, and the block items are
// the other pairs, r counting them in pair order. A tail item is
// z = 4, 2 or 1 consecutive samples of one pixel, each sample's colour
// stored on its own. item_order picks the item -> (frame / pair / group,
// pixel) map: pixel-major (bits 0, 1) puts one pixel's items back to back;
// with bit 2 (grouped; npix a multiple of the group, rt_api.cpp) the pixels
// go in groups of G = 2^P.pix_group_shift (4 or 8) consecutive ones (one
// row of a tile: 64 / 128 contiguous output / slot bytes) and a group's
// items back to back, frame / pair / sample group major, pixel minor: a
// wave's 64 items then hold G pixels of 64 / G frames, so the slots and
// output pixels it writes are whole 64- / 128-B pieces (one XCD's L2 merges
// them) instead of 16-B pieces of lines that other waves -- on other XCDs
// -- complete.
// Grouped: item j of a region with X entries per pixel -> group g = (j >> s)
// / X (floor division nests), rem = j - G g X, entry rem >> s, pixel
// G g + (rem & (G - 1)).
#ifndef RT_GROUPED_ON
#define RT_GROUPED_ON 1  // (0: the grouped order compiled out -- A/B builds only)
#endif
__device__ __forceinline__ void grouped_split(uint32_t j, const FastDiv& dx, uint32_t gs,
                                              uint32_t& entry, uint32_t& k) {
    const uint32_t g = fdiv(j >> gs, dx);
    const uint32_t rem = j - ((g * dx.d) << gs);
    entry = rem >> gs;
    k = (g << gs) + (rem & ((1u << gs) - 1u));
}
__device__ __forceinline__ void start_item(const KParams& P, PathState& st, uint32_t item,
                                           const PixelEntry* __restrict__ tab, ItemLds L) {
    // The launch parameters are read as values (scalar loads) and the item
    // kinds pick among values: selecting among fields of P by reference let
    // the compiler load them through a per-lane selected address (a vector
    // load from the kernarg segment on every item start).
    const uint32_t npix = P.npix, main_all = P.main_all, sample_base = P.sample_base;
    uint32_t k, s0, s1;  // pixel in processing order; the (first block's) samples [s0, s1)
    item = RT_IDX(item, P.chk_items, RT_SITE_ITEM);
    uint32_t slot = item;  // a main item's output slot
    bool whole = false;    // the item covers every sample of its (frame, pixel)
    uint32_t fo = 0;       // its launch frame
    if (item < main_all) {
        const uint32_t main_pix = P.main_pix, nblocks = P.nblocks, qpix = P.qpix;
        const uint32_t block_begin = P.block_begin, spp = P.spp;
        uint32_t f, b0, b1;  // frame, the item's blocks [b0, b1) (pass-relative)
        float4 a0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (item < main_pix) {
            if (item >= P.main_fp) {  // lead items: after the pixel items, own order
                grouped_split(item - P.main_fp, P.div_nlead, P.lead_group_shift, f, k);
                f += P.fp;
                slot = f * npix + k;
            } else if (RT_GROUPED_ON && (P.item_order & 4u)) {  // grouped: 8 pixels' frames, frame-major in the group
                grouped_split(item, P.div_nfpix, P.pix_group_shift, f, k);
                slot = f * npix + k;
            } else if (P.item_order & 2u) {  // pixel-major: one pixel's frames back to back
                k = fdiv(item, P.div_nfpix);
                f = item - k * P.div_nfpix.d;
                slot = f * npix + k;
            } else {
                f = fdiv(item, P.div_npix);
                k = item - f * npix;
            }
            b0 = 0;
            b1 = f < P.fp ? min(nblocks, qpix - f * nblocks) : min(P.lead, P.qmain - f * nblocks);
            whole = f < P.dfull;
            // a later pass over the frame's blocks (frames above the scratch
            // budget) continues the fold of the earlier passes (rt_collect_kernel
            // left it in acc_in): ((acc + b0) + b1) ..., the single-pass order
            if (block_begin) {
                a0 = P.acc_in[RT_IDX(order_to_pixel(P, k), npix, RT_SITE_ACC_IN)];
                a0.w = 1.0f;
            }
        } else {
            const uint32_t j = item - main_pix;
            uint32_t r;  // the pair (relative to qpix); slot main_pix + r * npix + k
            if (RT_GROUPED_ON && (P.item_order & 4u)) {  // grouped: 8 pixels' pairs, pair-major in the group
                grouped_split(j, P.div_nreg, P.pix_group_shift, r, k);
                slot = main_pix + r * npix + k;
            } else if (P.item_order & 1u) {  // pixel-major: one pixel's pairs back to back
                k = fdiv(j, P.div_nreg);
                r = j - k * P.div_nreg.d;
                slot = main_pix + r * npix + k;
            } else {
                r = fdiv(j, P.div_npix);
                k = j - r * npix;
            }
            // pair order: the pixel region's last frame's c0 pairs, then
            // nblocks - lead per frame (lead items take the first lead)
            if (r < P.c0) {
                f = P.fp - 1u;
                b0 = qpix + r - f * nblocks;
            } else {
                const uint32_t r1 = r - P.c0, fr = fdiv(r1, P.div_nbl);
                f = P.fp + fr;
                b0 = P.lead + (r1 - fr * P.div_nbl.d);
            }
            b1 = b0 + 1;
            whole = P.dwhole_blk != 0;
        }
        fo = f;
        const uint32_t base = sample_base + f * spp;
        s0 = base + (block_begin + b0) * RT_SAMPLE_BLOCK;
        const uint32_t iend = base + min(spp, (block_begin + b1) * RT_SAMPLE_BLOCK);
        s1 = min(s0 + RT_SAMPLE_BLOCK, iend);
        L->iend = iend;
        L->acc = a0;
    } else {  // tail item: z = 4, 2 or 1 consecutive samples, each stored on its own
        const uint32_t ti1 = P.ti1, ti2 = P.ti2, g0 = P.g0, g1 = P.g1, g2 = P.g2,
                       g_end = P.g_end;
        uint32_t j = item - main_all;
        const bool four = j < ti1, two = !four && j < ti2;
        const uint32_t z = four ? 4u : (two ? 2u : 1u);
        j -= four ? 0u : (two ? ti1 : ti2);
        const uint32_t gb = four ? g0 : (two ? g1 : g2), ge = four ? g1 : (two ? g2 : g_end);
        uint32_t g;  // the item's sample group within its region
        if (RT_GROUPED_ON && (P.item_order & 4u)) {  // grouped: 8 pixels' sample groups, group-major
            const FastDiv dz = four ? P.div_ng4 : (two ? P.div_ng2 : P.div_ng1);
            grouped_split(j, dz, P.pix_group_shift, g, k);
        } else if (P.item_order & 1u) {  // pixel-major: one pixel's groups back to back
            const FastDiv dz = four ? P.div_ng4 : (two ? P.div_ng2 : P.div_ng1);
            k = fdiv(j, dz);
            g = j - k * dz.d;
        } else {
            g = fdiv(j, P.div_npix);
            k = j - g * npix;
        }
        s0 = sample_base + gb + g * z;
        s1 = sample_base + min(gb + g * z + z, ge);
        whole = P.dwhole_tail != 0;  // (spp == 1: each sample is its frame's pixel)
    }
    const float4 q4 = tab[RT_IDX(k, npix, RT_SITE_TAB)].d;
    st.pix = __float_as_uint(q4.w);
    // main item: its output slot, or (whole, direct output) the output
    // index; tail item: RT_TAIL_ITEM | k, RT_DIRECT_ITEM when whole (its
    // samples' output indices follow from the sample, shade loop)
    if (P.dout && whole && item < P.main_all)
        slot = RT_DIRECT_ITEM | (fo * P.dstride + st.pix);
    st.item = item < P.main_all ? slot
                                : (RT_TAIL_ITEM | (P.dout && whole ? RT_DIRECT_ITEM : 0u) | k);
    st.s = s0;
    st.s_end = s1;
    st.bsum = mk(0.0f, 0.0f, 0.0f);
    L->pd = q4;
    start_sample(P, st, L);
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
// sph / shd: the exact-test records and the shading records in the index
// space of hi (the original list, or the matrix-core walk's order with its
// records in LDS or global memory: SP); nsph / nshd: their counts.
template <typename SP>
__device__ __forceinline__ bool shade(const KParams& P, PathState& st, int hi, float t,
                                      SP sph, const float4* __restrict__ shd, uint32_t nsph,
                                      uint32_t nshd) {
    const bool miss = hi < 0;
    if (!miss && st.bounce == P.max_depth - 1) {  // shade.wgsl:236-238
        st.color = mk(0.0f, 0.0f, 0.0f);
        return true;
    }
    // ---- record (hit lanes). Values read only under the condition that set
    // them are left unset: no register copies of defaults at the merge points
    // (-1.6 % kernel time).
    v3 pos, nrm;
    bool front;
    float4 mc;
    float fuzz, ior;
    int refl = -1;
    if (!miss) {
        // the centre (exact-test record) and the shading record (radius, the
        // material's reflectance / fuzziness / index of refraction, colour):
        // three independent loads (rt_api.cpp shade_records)
        const float4 s = rec_load(sph, RT_IDX((uint32_t)hi, nsph, RT_SITE_SPH));
        const uint32_t r = RT_IDX((uint32_t)hi, nshd, RT_SITE_RM);
        const float4 a = shd[2 * r];
        mc = shd[2 * r + 1];
        const float radius = a.x;
        pos = add(st.o, scale(st.d, t));
        const v3 q = sub(pos, mk(s.x, s.y, s.z));
        nrm = normalize_x(div3_x(q, radius));
        front = true;
        if (dot(st.d, nrm) > 0.0f) {
            nrm = neg(nrm);
            front = false;
        }
        refl = __float_as_int(a.y);
        fuzz = a.z;
        ior = a.w;
    }
    // ---- pre-normalize: metal normalize(reflect(d, n)) (shade.wgsl:140),
    //      dielectric unit_dir = normalize(d) (shade.wgsl:169)
    v3 un;
    if (refl == RT_METALLIC || refl == RT_DIELECTRIC)
        un = normalize_x(refl == RT_METALLIC ? reflect(st.d, nrm) : st.d);
    // ---- select
    v3 v = st.d;           // vector to normalize (sky: d, shade.wgsl:190)
    bool post = true;      // false: dielectric reflection keeps reflect(d, n) unnormalized
    v3 e_dir_raw;
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
    v3 vn;
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

// ---- collect: the fold of one (frame, pixel) ------------------------------
// Frame f's results for pixel k (processing order), in block / sample order
// (collect.wgsl:115-120 generalised, rt_hip.h "sample accumulation order"):
// its pixel item's fold (pairs below qpix, already folded by the lane that
// traced them, continuing an earlier pass's sum), then its block items' sums,
// then its tail blocks, whose samples' colours are summed here exactly as a
// lane sums a block, ((0 + c0) + c1) + ..., in sample order; each folded as
// the lane folds (first as is, then acc + it). `have` / (ax, ay, az) carry an
// earlier pass's partial sum. ld(slot) reads one slot.
template <typename LD>
__device__ __forceinline__ void fold_frame(const KParams& P, uint32_t f, uint32_t k, bool& have,
                                           float& ax, float& ay, float& az, LD ld) {
    const uint32_t q0 = f * P.nblocks;
    auto blocks_below = [&](uint32_t q) { return q > q0 ? min(P.nblocks, q - q0) : 0u; };
    // frames past the pixel pairs (f >= fp): their lead item's blocks
    const bool lf = f >= P.fp;
    const uint32_t bm = blocks_below(P.qmain), bp = lf ? min(P.lead, bm) : blocks_below(P.qpix);
    auto fold = [&](float vx, float vy, float vz) {
        if (have) {
            ax = ax + vx; ay = ay + vy; az = az + vz;
        } else {
            ax = vx; ay = vy; az = vz;
            have = true;
        }
    };
    if (bp) {  // the lane's fold already continued acc (start_item, later passes)
        const float4 v = ld((size_t)f * P.npix + k);
        ax = v.x; ay = v.y; az = v.z;
        have = true;
    }
    for (uint32_t b = bp; b < bm; ++b) {  // block items
        const uint32_t r = lf ? P.c0 + (f - P.fp) * P.div_nbl.d + (b - P.lead) : q0 + b - P.qpix;
        const float4 v = ld((size_t)P.main_pix + (size_t)r * P.npix + k);
        fold(v.x, v.y, v.z);
    }
    for (uint32_t b = bm; b < P.nblocks; ++b) {  // tail blocks: their samples' colours
        const uint32_t sl = (P.block_begin + b) * RT_SAMPLE_BLOCK;
        const uint32_t g_end = f * P.spp + min(P.spp, sl + RT_SAMPLE_BLOCK);
        float vx = 0.0f, vy = 0.0f, vz = 0.0f;
        for (uint32_t g = f * P.spp + sl; g < g_end; ++g) {
            const float4 c = ld((size_t)P.main_all + (size_t)(g - P.g0) * P.npix + k);
            vx = vx + c.x; vy = vy + c.y; vz = vz + c.z;
        }
        fold(vx, vy, vz);
    }
}

// Where frame f's pixel p (shard-local, row-major) goes: the shard layout
// (frame f at out + f*npix) or, with RT_FLAG_IMAGE_OUT, the image layout
// (frame f at out + f*width*height, the pixel at its image row).
__device__ __forceinline__ float4* out_pixel(const KParams& P, float4* out, uint32_t f, uint32_t p) {
    if (P.flags & RT_FLAG_IMAGE_OUT) {
        uint32_t x, y;
        pixel_xy(P, p, x, y);
        return out + RT_IDX((size_t)f * P.width * P.height + (size_t)y * P.width + x, P.chk_out,
                            RT_SITE_OUT);
    }
    return out + RT_IDX((size_t)f * P.npix + p, P.chk_out, RT_SITE_OUT);
}
