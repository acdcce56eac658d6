// rt_kernels.hip — the MI355X (gfx950) path-tracer kernels.
//
// ONE persistent kernel replaces the reference's whole WGSL chain
//   clear.wgsl:71-87 -> generate.wgsl:109-130 -> 3 x (prepass.wgsl:55-63,
//   intersect.wgsl:145-163, shade.wgsl:199-258) -> collect.wgsl:99-125
// dispatched by RayTraceNode::run (src/ray_trace_node.rs:195-224). Nothing is
// exchanged through HBM between stages: each lane keeps its whole path state
// (ray, throughput, seed, sample-block sum) in VGPRs.
//
// Work decomposition: a launch covers F frames; its work
// queue is pixel-major and holds three regions: *pixel items* (one per
// (frame, pixel), covering the frame's sample blocks of RT_SAMPLE_BLOCK
// samples in the region, folded in block order in LDS), then *block items*
// (pixel, one block), then *tail items* (2-sample, then single-sample; knob
// `tail`, default 0,1,0.5), so no lane holds a long item when the queue runs
// dry. Waves take chunks of items with one atomic (prefetched a chunk ahead);
// a lane whose path ends starts the next sample of its item, a lane whose item
// ends stores its slot (through a per-wave LDS buffer) and takes the next
// item (wave-ballot refill), so lanes do not idle while the wave's longest
// path finishes. An item covering every sample of its (frame, pixel) writes
// the output pixel itself (direct output); rt_collect_kernel folds the other
// frames' slots in block / sample order -- the oracle's summation order.
//
// Intersection (the hot loop, intersect.wgsl:133-143): the closest hit over
// the whole list, with the brute-force loop's result, in stages that skip
// most of its work. By default, the matrix-core walk: each 16-sphere half of
// a 32-sphere block (the list in k-d spatial order) has a bounding sphere,
// tested against the wave's rays on the matrix cores first, and a 32-ray
// half-wave walks only the blocks whose bounds one of its rays passes near
// (proof in rt_dev_intersect.h "Block bounds"); in a walked block a
// conservative filter proves most (sphere, ray) pairs miss -- one 32-term
// f16 hi/lo dot product per pair, two chained v_mfma_f32_32x32x16_f16 per
// 32-sphere x 32-ray tile giving V = T0 - H0, a pair a candidate iff V < 0
// (intersect_world_mfma). The packed VALU filter -- every
// sphere, no bounds -- serves RT_FLAG_VALU_FILTER, waves with a ray outside
// the f16 split's range and scenes outside it; the culled list (RT_FLAG_CULL)
// runs it behind group bounds. It evaluates the same test as packed fp32
// FMAs over groups of 8 spheres read with scalar loads (filter8):
//   H - T = hb^2 + r^2 - (1 - m)|o - c|^2 + mu (|o|^2 + |c|^2),  hb = dn.(o - c)
// H < T proves the reference's discriminant (intersect.wgsl:102) is negative.
// Lanes queue their candidates in LDS; after the walk each lane runs the
// reference's exact op sequence (intersect.wgsl:97-115) on its own candidates
// with the strict `<` tie-break (:137; a (t, index) lexicographic minimum
// where the candidates come in another order), so the result is
// bit-identical to the brute-force reference loop.
//
// Sources: rt_dev_math.h (vector ops, correctly rounded short forms, camera
// rays), rt_dev_intersect.h (exact test, filter8, candidate queues,
// intersect_world / intersect_wide), rt_dev_path.h (lane state, work items,
// shading); this file holds the kernels and their launchers.
//
// Floating point: compiled with -ffp-contract=off; every expression below
// except the explicit FMAs of the filter is one IEEE f32 round-to-nearest op
// in the same order as oracle/rt_oracle.c. Divides and square roots are
// correctly rounded: the short forms of rt_math.h where their domain is
// proved (exact test) or checked per lane (shading), IEEE otherwise.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_internal.h"
#include "rt_math.h"

// Wave ballot on a bool straight into the intrinsic: HIP's __ballot(int)
// round-trips the lane mask through a VGPR (v_cndmask + v_cmp, 2 VALU) when
// the predicate comes from another block.
__device__ __forceinline__ uint64_t rt_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Keeps a rare fallback in its branch: LLVM prices sqrt / fdiv as one IR
// instruction and speculates them out of the branch (then the backend's
// 11-17 instruction IEEE expansion runs on every pass, measured). A volatile
// asm cannot be speculated.
__device__ __forceinline__ float rt_cold(float x) {
    asm volatile("" : "+v"(x));
    return x;
}

#define VERY_FAR 1e20f
#define EPSILON 0.001f

// ---- checked build (make checked: -DRT_CHECK_BOUNDS, librt_hip_checked.so;
// never the product library). Every computed index into a buffer or an LDS
// array goes through RT_IDX(i, n, site): out of range, the first violation's
// (site, index, bound) is recorded in g_rt_check, the count incremented, and
// index 0 used instead, so the launch completes and the host reports it
// (rt_api.cpp check_bounds fails the call with RT_ERR_DEVICE) instead of the
// GPU faulting. Sites: enum RtSite below.
enum RtSite : uint32_t {
    RT_SITE_ITEM = 1,        // work item index < items of the launch (start_item)
    RT_SITE_TAB = 2,         // pixel table tab[k], k < npix
    RT_SITE_ACC_IN = 3,      // acc_in[p] of a later pass, p < npix
    RT_SITE_SPH = 4,         // sph[hi] in shade
    RT_SITE_RM = 5,          // shd[2 hi], shd[2 hi + 1] (shading record) in shade
    RT_SITE_SLOT = 7,        // block_sums slot written by the render kernel
    RT_SITE_SLOTBUF = 8,     // per-wave slot buffer entry
    RT_SITE_MFQ = 9,         // matrix-core queue append (entries per lane and half)
    RT_SITE_MFQ_READ = 10,   // matrix-core drain: queue entry read
    RT_SITE_MF_SPH = 11,     // matrix-core drain: candidate sphere record
    RT_SITE_CQ = 12,         // VALU-walk queue append
    RT_SITE_CQ_SPH = 13,     // VALU-walk drain: candidate sphere record
    RT_SITE_CACHE = 14,      // primary-hit cache: hi in [-1, nsph)
    RT_SITE_COLLECT = 15,    // collect: slot read
    RT_SITE_OUT = 16,        // collect: output pixel
    RT_SITE_WIDE_SPH = 17,   // sphere-parallel walk: sph[i]
    RT_SITE_PERM = 18,       // culled list: perm[idx]
    RT_SITE_MFA = 19,        // matrix-core walk: A-fragment block
    RT_SITE_DEAD_QUEUE = 20, // matrix-core walk: a lane without a ray queued a candidate
    RT_SITE_MF_BOUND = 21,   // matrix-core walk: block-bound chunk
};
#ifdef RT_CHECK_BOUNDS
__device__ unsigned int g_rt_check[4];  // violations, first (site, index, bound)
__device__ __noinline__ void rt_check_fail(uint32_t site, uint64_t i, uint64_t n) {
    if (atomicAdd(&g_rt_check[0], 1u) == 0u) {
        g_rt_check[1] = site;
        g_rt_check[2] = (unsigned int)min(i, (uint64_t)0xFFFFFFFFu);
        g_rt_check[3] = (unsigned int)min(n, (uint64_t)0xFFFFFFFFu);
    }
}
template <typename I>
__device__ __forceinline__ I rt_idx(I i, uint64_t n, uint32_t site) {
    if ((uint64_t)i >= n) {
        rt_check_fail(site, (uint64_t)i, n);
        return (I)0;
    }
    return i;
}
#define RT_IDX(i, n, site) rt_idx((i), (uint64_t)(n), (site))
#else
#define RT_IDX(i, n, site) (i)
#endif

#include "rt_dev_math.h"
#include "rt_dev_intersect.h"
#include "rt_dev_path.h"


#ifdef RT_CHUNK_TRACE
#define RT_CHUNK_TRACE_MAX (1u << 22)
__device__ unsigned long long g_chunk_trace[RT_CHUNK_TRACE_MAX];
__device__ unsigned long long g_chunk_clk[RT_CHUNK_TRACE_MAX];  // shader clock (s_memtime)
#endif
#ifdef RT_WAVE_TRACE
// Diagnostic build only (-DRT_WAVE_TRACE): per wave (start, end, exhausted-at)
// in s_memrealtime ticks (100 MHz) and (iterations, items) -- the schedule's
// tail shape. Read back with rt_debug_wave_trace().
#define RT_TRACE_MAX_WAVES 32768
__device__ unsigned long long g_wave_trace[RT_TRACE_MAX_WAVES * 4];
#endif

#ifdef RT_RAY_DUMP
// Diagnostic build only (-DRT_RAY_DUMP): every lane's ray (o, pixel; d,
// bounce) of waves 0..RT_RAY_DUMP_WAVES-1 at their loop iteration
// RT_RAY_DUMP_ITER, read back with rt_debug_ray_dump() (tools/ray_dump.py).
#define RT_RAY_DUMP_WAVES 1024
#ifndef RT_RAY_DUMP_ITER
#define RT_RAY_DUMP_ITER 5000
#endif
__device__ float4 g_ray_dump[RT_RAY_DUMP_WAVES * 64 * 2];
#endif

#ifndef RT_PARAMS_HOLD
// The launch parameters re-read from the kernarg segment where they are used
// (scalar loads) instead of being held in SGPRs across the whole loop: the
// volatile asm makes the pointer opaque per iteration, so no load of a field
// is hoisted out of the loop. Held, they spilled ~47 SGPRs to VGPR lanes
// (~110 v_readlane/v_writelane in the loop, one VGPR to scratch); re-read:
// no spills, 76 VGPRs, -1.8 % VALU, -1.5 % time (RT_PARAMS_HOLD: the old form).
__device__ __forceinline__ const KParams& fresh_params() {
    typedef __attribute__((address_space(4))) const KParams cKParams;
    cKParams* p = (cKParams*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const KParams*)p;
}
#endif

// A 16-B store at system scope, write-through (global_store_dwordx4 ... sc0
// sc1: the AMDGPU memory model's system-scope store; a vector store). Used for
// rows that may belong to another device's image (RT_FLAG_IMAGE_OUT). hipcc
// does not count an asm store in its waits: the caller waits (vmcnt(0)).
__device__ __forceinline__ void store_system(float4* p, float4 v) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(x) : "memory");
}

// The persistent render loop; CULL = false is rt_render_kernel (the brute-force
// walk of the headline), CULL = true rt_render_cull_kernel (the permuted list
// with group bounds, P.bnd / P.perm / P.nclusters; identical results).
// SPH_LDS (rt_render_kernel): the matrix-core walk's records (mf.sph, at
// most RT_MF_SPH_LDS_MAX = 512 for a list of at most 16 blocks) copied into
// the workgroup's LDS at the start, so the drain's dependent record load is
// an LDS read, not an L1 hit: -1.2 % cycles per headline launch net of the
// queue entries it costs (9 per lane and half instead of 12; slot buffer 24
// instead of 32: 4 workgroups per CU still fit), profiles/r05/lds/.
// MULTI: the matrix-core walk for any list (rt_render_multi_kernel); false:
// lists of at most 16 blocks (rt_render_kernel; intersect_world_mfma MULTI).
template <bool CULL, bool SPH_LDS = false, bool MULTI = false>
__device__ __forceinline__ void render_body(
    const KParams& P, const float4* grp, const float4* __restrict__ sph,
    const float4* __restrict__ shd,
    const PixelEntry* __restrict__ tab, float4* __restrict__ block_sums,
    uint32_t* __restrict__ work_counter,
    unsigned long long* __restrict__ seg_counter, unsigned long long* __restrict__ dbg) {
    const uint32_t lane = __lane_id();
    // the queue and slot-buffer capacities of this kernel (LDS budget)
    constexpr uint32_t MFCAP = SPH_LDS ? RT_MF_CAP_LDS : RT_MF_CAP;
    constexpr uint32_t SBCAP = SPH_LDS ? RT_SLOT_BUF_CAP_LDS : RT_SLOT_BUF_CAP;
    __shared__ float4 s_msph[SPH_LDS ? RT_MF_SPH_LDS_MAX : 1];
    if constexpr (SPH_LDS) {
        if (P.mf.A) {  // nblk <= 16: nblk * 32 <= RT_MF_SPH_LDS_MAX (rt_launch_render)
            const uint32_t nrec = P.mf.nblk * 32u;
            for (uint32_t i = threadIdx.x; i < nrec; i += RT_BLOCK_THREADS) s_msph[i] = P.mf.sph[i];
        }
        __syncthreads();
    }
    PROF_DECL
    PROF_START();
#ifdef RT_PROFILE
    const unsigned long long t_begin = prof_.last;
#endif
    // the launch's shader clock (rt_stats.clock_ghz): every wave adds its
    // lifetime in shader cycles (s_memtime) and in 100 MHz ticks
    // (s_memrealtime) to two sums -- the start as a subtraction now, the end
    // as an addition at the end, so nothing stays live across the loop
    unsigned long long* const clk_sum = seg_counter + RT_CNT_CLOCK_OFFSET / 2;
    if (lane == 0) {
        atomicAdd(clk_sum, 0ull - (unsigned long long)__builtin_amdgcn_s_memtime());
        atomicAdd(clk_sum + 1, 0ull - (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
    // the wave's slices of the workgroup's LDS arrays: wave-uniform bases
    // (SGPRs) indexed by the lane id, so no VGPR holds an LDS address
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x) >> 6;
    // per-lane candidate queues: RT_CQ_CAP entries per lane for the VALU walk,
    // 2 halves x RT_MF_CAP for the matrix-core walk (RT_MFMA_FILTER); a wave
    // drains the queue of one walk before it starts another, so both share
    // one array (the brute-force kernel's LDS: 36 KB per workgroup)
#ifdef RT_MFMA_FILTER
    constexpr uint32_t QW = CULL ? 64u * RT_CQ_CAP : 2u * MFCAP * 64u;  // words per wave
    static_assert(2u * MFCAP >= RT_CQ_CAP, "the shared queue holds the VALU walk's");
#else
    constexpr uint32_t QW = 64u * RT_CQ_CAP;
#endif
    __shared__ __attribute__((aligned(8))) uint32_t s_cq[(RT_BLOCK_THREADS / 64) * QW];
    uint32_t* cq = s_cq + wave * QW;
#ifdef RT_MFMA_FILTER
    uint32_t* cqm = cq;
#endif
    __shared__ LaneLds s_lane[RT_BLOCK_THREADS];  // per-lane item state (rt_dev_path.h)
    const ItemLds lds = s_lane + wave * 64u + lane;
#ifndef RT_NO_SLOT_BUF
    // Slot-store buffer: a finished block / item / tail sample goes to the
    // wave's LDS buffer, and the wave writes the buffer out with one store
    // when it would overflow (and at the end). A vector store holds vmcnt
    // until the memory acknowledges it, so a store issued on its own makes the
    // wave's next wait on a load (table entry, A fragments) wait for the
    // store too: one such wait per SBCAP slots instead of one per
    // iteration that stores. sbn: entries held (wave-uniform).
    __shared__ float4 s_sbv[(RT_BLOCK_THREADS / 64) * SBCAP];
    __shared__ uint32_t s_sbs[(RT_BLOCK_THREADS / 64) * SBCAP];
    float4* const sbv = s_sbv + wave * SBCAP;
    uint32_t* const sbs = s_sbs + wave * SBCAP;
    uint32_t sbn = 0;
    // one finished slot: a block-sum slot, or (RT_DIRECT_ITEM) an output pixel
    // = fold / spp, alpha 1 -- rt_collect_kernel's arithmetic
    auto put = [&](uint32_t e, float4 v) {
        if (e & RT_DIRECT_ITEM) {
            const float spp = (float)P.spp;
            const float4 o = make_float4(v.x / spp, v.y / spp, v.z / spp, 1.0f);
            // (device-local outputs only: rt_api.cpp turns direct output off
            // for another device's image)
            P.dout[RT_IDX(e & ~RT_DIRECT_ITEM, P.chk_out, RT_SITE_OUT)] = o;
        } else {
            block_sums[RT_IDX(e, P.chk_slots, RT_SITE_SLOT)] = v;
        }
    };
    auto sb_flush = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < sbn) put(sbs[lane], sbv[lane]);
        sbn = 0;
    };
#endif
#ifdef RT_SPHERES_LDS
    // Experiment variant: the filter reads the sphere groups from LDS (staged
    // once per workgroup) instead of the scalar cache.
    extern __shared__ float4 s_grp[];
    for (uint32_t i = threadIdx.x; i < (P.ngroups + 1) * 8; i += RT_BLOCK_THREADS) s_grp[i] = grp[i];
    __syncthreads();
    grp = s_grp;
#endif
    const uint32_t total = P.main_all + P.tail_items;
#ifdef RT_WAVE_TRACE
#ifdef RT_WAVE_TRACE_LITE
    if (lane == 0) {  // stored at once: nothing stays live across the loop
        const uint32_t wid0 = blockIdx.x * (RT_BLOCK_THREADS / 64) + threadIdx.x / 64;
        if (wid0 < RT_TRACE_MAX_WAVES) g_wave_trace[wid0 * 4 + 0] = __builtin_amdgcn_s_memrealtime();
    }
    const unsigned long long tr_t0 = 0;
#else
    const unsigned long long tr_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    unsigned long long tr_ex = 0;
    uint32_t tr_iters = 0, tr_items = 0, tr_after = 0;
#ifdef RT_WAVE_TRACE_LITE  // start/end only: keeps the product's register budget
#define TR_COUNT(x)
#else
#define TR_COUNT(x) x
#endif
#endif
    // primary-hit reuse: the primary ray is pixel-only unless the opt-in
    // camera sampling varies it per sample
    const bool use_cache =
        (P.flags & (RT_FLAG_NO_PRIMARY_CACHE | RT_FLAG_JITTER | RT_FLAG_THIN_LENS)) == 0;

    // Shading by walk position (round 5): with the matrix-core walk the hit
    // is its walk position, shaded from the records in the walk's order
    // (LDS in rt_render_kernel, MfScene.sph / .shd) -- no permutation load
    // between the drain and the shading; the other walks' answers map
    // through MfScene.iperm. Without it (the culled list, or no matrix-core
    // scene) the original list.
#ifdef RT_MFMA_FILTER
    const bool widx = !CULL && P.mf.A != nullptr;
#else
    const bool widx = false;
#endif
    const uint32_t nsph_sh = widx ? P.chk_wsph : P.chk_nsph;  // (RT_IDX bounds)
    PathState st;
    bool has_item = false;
    uint32_t q_next = 0, q_end = 0;  // wave-uniform chunk of work items
    bool exhausted = false;
    uint32_t traced = 0, segs = 0;  // wave totals (wave-uniform: SGPRs, not a VGPR per lane)
    // Chunk prefetch: the atomic for the wave's NEXT chunk is issued as soon as
    // the current one is taken, so its round trip to the device-scope counter
    // (one address shared by every wave of the chip) overlaps a whole filter
    // walk instead of stalling the refill. Every prefetched chunk is consumed:
    // a wave only stops after consuming a base >= total, and issues no further
    // prefetch from then on.
    uint32_t iter = 0;            // loop iterations of this wave (wave-uniform)
    // hardware wave slot on its SIMD (HW_ID[3:0]): distinct for co-resident waves
    const uint32_t wave_slot = __builtin_amdgcn_s_getreg((3 << 11) | 4);
    uint32_t pref = 0;            // lane 0: base of the prefetched chunk
    uint32_t pref_chunk = 0;      // its size (0 = none in flight)

    for (;;) {
#ifndef RT_PARAMS_HOLD
        const KParams& P = fresh_params();
#endif
        // ---- refill: lanes without an item take the next ones (wave ballot)
        uint64_t need = rt_ballot(!has_item);
        while (need != 0 && !exhausted) {
            if (q_next >= q_end) {
                // big chunks keep the counter cold; small ones near the end of
                // the queue keep the waves' finishing times together
                uint32_t chunk, base = 0;
                if (pref_chunk) {
                    chunk = pref_chunk;
                    base = pref;
                } else {
                    chunk = q_end >= P.tail_start ? RT_WAVE_CHUNK_TAIL : P.chunk;
                    if (lane == 0) base = atomicAdd(work_counter, chunk);
                }
                base = __builtin_amdgcn_readlane(base, 0);
                pref_chunk = 0;
                if (base >= total) {
#ifdef RT_WAVE_TRACE
                    TR_COUNT(tr_ex = __builtin_amdgcn_s_memrealtime());
#endif
                    exhausted = true;
                    break;
                }
                q_next = base;
                q_end = min(base + chunk, total);
#ifdef RT_CHUNK_TRACE
                // diagnostic: time at which each 64-item slice of the queue is taken
                if (lane == 0 && (base >> 6) < RT_CHUNK_TRACE_MAX) {
                    g_chunk_trace[base >> 6] = __builtin_amdgcn_s_memrealtime();
                    g_chunk_clk[base >> 6] = __builtin_amdgcn_s_memtime();
                }
#endif
                if (P.prefetch) {
                    pref_chunk = q_end >= P.tail_start ? RT_WAVE_CHUNK_TAIL : P.chunk;
                    if (lane == 0) pref = atomicAdd(work_counter, pref_chunk);
                }
            }
            const uint32_t avail = q_end - q_next;
            const uint32_t rank = lanemask_lt_count(need);
            const uint32_t cnt = (uint32_t)__popcll(need);
            if (!has_item && rank < avail) {
                start_item(P, st, q_next + rank, tab, lds);
                has_item = true;
            }
#ifdef RT_WAVE_TRACE
            TR_COUNT(tr_items += min(avail, cnt));
#endif
            q_next += min(avail, cnt);
            need = rt_ballot(!has_item);
        }
        if (rt_ballot(has_item) == 0) break;
        // ---- issue fairness: the SIMD arbiter issues by priority, then age
        // (MI355X_MICROARCH.md "Two waves per SIMD"), so in a persistent
        // launch the waves of a SIMD progress at geometrically falling rates
        // by dispatch order (measured per iteration, 1st..6th wave: 17, 21,
        // 33, 57, 113, 248 us) and the youngest waves' items become the
        // launch's stragglers. Mode 1 (default) rotates the priority level
        // with the wave's iteration count offset by its hardware wave slot
        // (20, 24, 30, 42, 69, 144 us); mode 3 rotates it by wall time
        // (s_memrealtime >> prio_shift), all waves of a SIMD stepping together.
        if (P.prio_mode) {
            const uint32_t lvl =
                P.prio_mode == 1
                    ? (iter + wave_slot) & 3u
                    : ((uint32_t)(__builtin_amdgcn_s_memrealtime() >> P.prio_shift) + wave_slot) & 3u;
            switch (lvl) {
                case 0: __builtin_amdgcn_s_setprio(0); break;
                case 1: __builtin_amdgcn_s_setprio(1); break;
                case 2: __builtin_amdgcn_s_setprio(2); break;
                default: __builtin_amdgcn_s_setprio(3); break;
            }
        }
        ++iter;
#ifdef RT_WAVE_TRACE
        TR_COUNT(++tr_iters);
        TR_COUNT(tr_after += exhausted ? 1u : 0u);
#endif
        PROF_MARK(0);
        PROF_ADD(4, 1);
#ifdef RT_PROFILE
        {   // diagnostic: distinct pixels per half-wave (c[6]) and lanes at bounce 0 (c[14]);
            // its own time goes to c[26] (excluded from the phase shares)
            uint64_t rest = rt_ballot(has_item);
            uint32_t distinct = 0;
            while (rest) {
                const uint32_t l0 = (uint32_t)__builtin_ctzll(rest);
                const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane((int)st.pix, (int)l0);
                const uint64_t half = l0 < 32u ? 0x00000000FFFFFFFFull : 0xFFFFFFFF00000000ull;
                const uint64_t same = rt_ballot(has_item && st.pix == p0) & half;
                rest &= ~same;
                ++distinct;
            }
            PROF_ADD(6, distinct);
            PROF_ADD(14, (unsigned long long)__popcll(rt_ballot(has_item && st.bounce == 0)));
            PROF_MARK(26);
        }
#endif
        PROF_ADD(9, (unsigned long long)__popcll(rt_ballot(has_item)));

        // ---- opt-in camera sampling: a lane at bounce 0 holds a fresh sample
        // whose primary ray varies per sample (no primary-hit reuse then)
        if ((P.flags & (RT_FLAG_JITTER | RT_FLAG_THIN_LENS)) && has_item && st.bounce == 0) {
            const uint32_t idx = st.pix + (P.width * P.height) * (P.frame0 + st.s);
            const uint32_t y = fdiv(st.pix, P.div_width);
            sampled_primary_ray(P, st.pix - y * P.width, y, idx, st.o, st.d);
        }

#ifdef RT_RAY_DUMP
        if (iter == RT_RAY_DUMP_ITER) {
            const uint32_t wid = blockIdx.x * (RT_BLOCK_THREADS / 64) + threadIdx.x / 64;
            if (wid < RT_RAY_DUMP_WAVES) {
                const uint32_t k = (wid * 64u + lane) * 2u;
                g_ray_dump[k] = make_float4(st.o.x, st.o.y, st.o.z, __uint_as_float(has_item ? st.pix : 0xFFFFFFFFu));
                g_ray_dump[k + 1] = make_float4(st.d.x, st.d.y, st.d.z, __uint_as_float(st.bounce));
            }
        }
#endif
        // ---- intersect (intersect.wgsl:145-163): every lane with an item holds
        // a ray that needs tracing here.
        int hi = -1;
        float t = VERY_FAR;
        const uint64_t live = rt_ballot(has_item);
        // (branch weights: the matrix-core walk is the hot path; the
        // sphere-parallel and VALU walks are placed out of its way, so the
        // loop's hot blocks stay together in the instruction cache)
        if (__builtin_expect((uint32_t)__popcll(live) <= P.wide_max, 0)) {  // nearly empty wave: sphere-parallel
            PROF_ADD(20, 1);
            intersect_wide<CULL>(sph, P.nspheres, P.scene_fast, live, st.o, st.d, hi, t, P.perm);
#ifdef RT_MFMA_FILTER
            if (widx && hi >= 0) hi = (int)P.mf.iperm[hi];
#endif
#ifdef RT_MFMA_FILTER
        } else if (__builtin_expect(!CULL && P.mf.A && mfma_wave_ok(st.o, has_item), 1)) {  // the whole wave
            PROF_ADD(18, 1);
            const int h2 = intersect_world_mfma<false, SPH_LDS, MULTI, MFCAP, false>(
                P.mf, P.scene_fast, st.o, st.d, has_item, live, t, cqm
#ifdef RT_PROFILE
                , prof_
#endif
                , nullptr, (lds_cfloat4*)s_msph);
            if (has_item) hi = h2;
            else t = VERY_FAR;
#endif
        } else if (has_item) {
            PROF_ADD(19, 1);
            hi = intersect_world<CULL>(grp, sph, P.ngroups, P.scene_fast, st.o, st.d, t, cq,
#ifdef RT_PROFILE
                                       prof_,
#endif
                                       P.bnd, P.perm, P.nclusters, P.cull_supers != 0);
#ifdef RT_MFMA_FILTER
            if (widx && hi >= 0) hi = (int)P.mf.iperm[hi];
#endif
        }
        traced = __builtin_amdgcn_readfirstlane(traced + (uint32_t)__popcll(live));
        if (use_cache && has_item && st.bounce == 0)  // the item's first sample: its primary hit
            lds->cache = make_float2(__int_as_float(hi), t);
        // ---- shade; a finished path starts the next sample, whose primary hit
        // is reused (result-identical) so the lane goes on to its bounce-1 ray.
        bool shading = has_item;
#ifndef RT_NO_SLOT_BUF
        bool spend = false;  // this round finished a slot: sslot <- sval
        uint32_t sslot = 0;
        float4 sval;
#endif
        PROF_MARK(12);  // bookkeeping between the drain and the shading loop
        // uniform loop (the segment count is a wave total): one round per
        // path step, lanes without a step to shade idle through the round
        for (;;) {
            const uint64_t sh = rt_ballot(shading);
            if (sh == 0) break;
            PROF_ADD(22, 1);  // shading rounds (wave-level)
            segs = __builtin_amdgcn_readfirstlane(segs + (uint32_t)__popcll(sh));
            if (shading) {
                bool done;
                if constexpr (SPH_LDS)  // (only with the matrix-core scene: rt_launch_render)
                    done = shade(P, st, hi, t, (lds_cfloat4*)s_msph, P.mf.shd,
                                 P.chk_wsph < RT_MF_SPH_LDS_MAX ? P.chk_wsph : RT_MF_SPH_LDS_MAX,
                                 P.chk_wrm);  // (the checked build's bound: the LDS array's)
                else
                    done = shade(P, st, hi, t, widx ? P.mf.sph : sph, widx ? P.mf.shd : shd, nsph_sh,
                                 widx ? P.chk_wrm : P.chk_nrm);
                shading = false;
                if (done) {
                    // path finished: accumulate (collect.wgsl:115-120, blocked);
                    // a tail item stores every sample's colour for the collect
                    if (st.item & RT_TAIL_ITEM) {
                        const v3 c = add(mk(0.0f, 0.0f, 0.0f), st.color);
                        // a whole (spp == 1) tail sample is its frame's pixel:
                        // the output index of launch frame s - sample_base
                        const uint32_t slot =
                            (st.item & RT_DIRECT_ITEM)
                                ? RT_DIRECT_ITEM | ((st.s - P.sample_base) * P.dstride + st.pix)
                                : P.main_all + (st.s - P.sample_base - P.g0) * P.npix +
                                      (st.item & ~(RT_TAIL_ITEM | RT_DIRECT_ITEM));
#ifndef RT_NO_SLOT_BUF
                        spend = true;
                        sslot = slot;
                        sval = make_float4(c.x, c.y, c.z, 0.0f);
#else
#ifdef RT_DIAG_NO_BSTORE  // timing diagnostic only: no slot stores (wrong image)
                        if (c.x == -1234.5f)
#endif
                        block_sums[slot] = make_float4(c.x, c.y, c.z, 0.0f);
#endif
                    } else {
                        st.bsum = add(st.bsum, st.color);
                    }
                    ++st.s;
                    bool next = st.s < st.s_end;
                    if (!next && !(st.item & RT_TAIL_ITEM)) {
                        // a sample block of a main item ends: fold its sum into
                        // the item's running sum in block order (as
                        // rt_collect_kernel folds: first block as is, then
                        // acc + bsum); the item's last block stores the fold
                        const float4 a = lds->acc;
                        const v3 acc = a.w != 0.0f ? add(mk(a.x, a.y, a.z), st.bsum) : st.bsum;
                        const uint32_t iend = lds->iend;
                        if (st.s < iend) {
                            lds->acc = make_float4(acc.x, acc.y, acc.z, 1.0f);
                            st.bsum = mk(0.0f, 0.0f, 0.0f);
                            st.s_end = min(st.s + RT_SAMPLE_BLOCK, iend);
                            next = true;
                        } else {
#ifndef RT_NO_SLOT_BUF
                            spend = true;
                            sslot = st.item;
                            sval = make_float4(acc.x, acc.y, acc.z, 0.0f);
#else
#ifdef RT_DIAG_NO_BSTORE
                            if (acc.x == -1234.5f)
#endif
                            block_sums[st.item] = make_float4(acc.x, acc.y, acc.z, 0.0f);
#endif
                        }
                    }
                    if (next) {
                        start_sample(P, st, lds);
                        if (use_cache) {
                            const float2 c = lds->cache;
                            hi = (int)RT_IDX((uint32_t)(__float_as_int(c.x) + 1), nsph_sh + 1u,
                                             RT_SITE_CACHE) - 1;
                            t = c.y;
                            shading = true;
                        }
                    } else {
                        has_item = false;
                    }
                }
            }
#ifndef RT_NO_SLOT_BUF
            // this round's finished slots into the buffer (a burst larger
            // than the buffer goes straight out)
            const uint64_t sm = rt_ballot(spend);
            if (sm != 0) {
                const uint32_t n = (uint32_t)__popcll(sm);
                if (sbn + n > SBCAP) sb_flush();
                if (n > SBCAP) {
                    if (spend) put(sslot, sval);
                } else {
                    if (spend) {
                        const uint32_t r = sbn + lanemask_lt_count(sm);
                        sbv[RT_IDX(r, SBCAP, RT_SITE_SLOTBUF)] = sval;
                        sbs[RT_IDX(r, SBCAP, RT_SITE_SLOTBUF)] = sslot;
                    }
                    sbn = __builtin_amdgcn_readfirstlane(sbn + n);
                }
                spend = false;
            }
#endif
        }
        PROF_MARK(3);
    }
#ifndef RT_NO_SLOT_BUF
    sb_flush();
#endif

#ifdef RT_PROFILE
    PROF_MARK(7);
    prof_.c[8] = __builtin_amdgcn_s_memtime() - t_begin;
    if (lane == 0)
        for (int i = 0; i < RT_DBG_COUNTERS; ++i) atomicAdd(dbg + i, prof_.c[i]);
#endif
#ifdef RT_WAVE_TRACE
    {
        const uint32_t wid = blockIdx.x * (RT_BLOCK_THREADS / 64) + threadIdx.x / 64;
        if (lane == 0 && wid < RT_TRACE_MAX_WAVES) {
#ifndef RT_WAVE_TRACE_LITE
            g_wave_trace[wid * 4 + 0] = tr_t0;
#else
            (void)tr_t0;
#endif
            g_wave_trace[wid * 4 + 1] = __builtin_amdgcn_s_memrealtime();
#ifdef RT_PROFILE  // combined diagnostic build: where the wave ran (HW_ID, XCC_ID)
            g_wave_trace[wid * 4 + 2] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                                        ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20)
                                         << 32);
            (void)tr_ex;
#else
            g_wave_trace[wid * 4 + 2] = tr_ex;
#endif
#ifdef RT_PROFILE  // combined diagnostic build: exact tests (wave max, summed) instead of items
            g_wave_trace[wid * 4 + 3] = ((unsigned long long)min(prof_.c[13], 0xFFFFFFFFull) << 32) |
                                        (min(tr_after, 65535u) << 16) | min(tr_iters, 65535u);
#else
            g_wave_trace[wid * 4 + 3] = ((unsigned long long)tr_items << 32) |
                                        (min(tr_after, 65535u) << 16) | min(tr_iters, 65535u);
#endif
        }
    }
#endif
    // ---- segment counts and the wave's end stamps: one atomic each per wave
    if (lane == 0) {
        atomicAdd(seg_counter, (unsigned long long)segs);
        atomicAdd(seg_counter + 1, (unsigned long long)traced);
        atomicAdd(clk_sum, (unsigned long long)__builtin_amdgcn_s_memtime());
        atomicAdd(clk_sum + 1, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    }
}

__global__ __launch_bounds__(RT_BLOCK_THREADS, RT_MIN_WAVES_PER_SIMD) void rt_render_kernel(
    KParams P, const float4* grp, const float4* __restrict__ sph,
    const float4* __restrict__ shd,
    const PixelEntry* __restrict__ tab, float4* __restrict__ block_sums,
    uint32_t* __restrict__ work_counter,
    unsigned long long* __restrict__ seg_counter, unsigned long long* __restrict__ dbg) {
    render_body<false, true, false>(P, grp, sph, shd, tab, block_sums, work_counter, seg_counter, dbg);
}

// lists of more than 16 blocks (the bound-chunk loop, chunk-level bounds)
__global__ __launch_bounds__(RT_BLOCK_THREADS, RT_MIN_WAVES_PER_SIMD) void rt_render_multi_kernel(
    KParams P, const float4* grp, const float4* __restrict__ sph,
    const float4* __restrict__ shd,
    const PixelEntry* __restrict__ tab, float4* __restrict__ block_sums,
    uint32_t* __restrict__ work_counter,
    unsigned long long* __restrict__ seg_counter, unsigned long long* __restrict__ dbg) {
    render_body<false, false, true>(P, grp, sph, shd, tab, block_sums, work_counter, seg_counter, dbg);
}


__global__ __launch_bounds__(RT_BLOCK_THREADS, RT_MIN_WAVES_PER_SIMD_CULL) void rt_render_cull_kernel(
    KParams P, const float4* grp, const float4* __restrict__ sph,
    const float4* __restrict__ shd,
    const PixelEntry* __restrict__ tab, float4* __restrict__ block_sums,
    uint32_t* __restrict__ work_counter,
    unsigned long long* __restrict__ seg_counter, unsigned long long* __restrict__ dbg) {
    render_body<true>(P, grp, sph, shd, tab, block_sums, work_counter, seg_counter, dbg);
}

// Pixel table, once per frame: for the k-th pixel of the processing order
// its shard pixel index, global (x, y) and primary ray direction
// (generate.wgsl:66-126; the direction depends on the pixel only: lens
// offset 0, no jitter).
__global__ void rt_primary_kernel(KParams P, PixelEntry* __restrict__ tab) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P.npix) return;
    const uint32_t p = order_to_pixel(P, k);
    uint32_t x, y;
    pixel_xy(P, p, x, y);
    v3 o, d;
    primary_ray(P, x, y, o, d);
    tab[k].d = make_float4(d.x, d.y, d.z, __uint_as_float(x + P.width * y));
}

// Batch closest-hit query (rt_intersect): one ray per lane, same intersect_world.
// CULL: the permuted list with its bounds; the index returned is the original.
template <bool CULL>
__device__ __forceinline__ void intersect_body(
    const float4* __restrict__ grp, const float4* __restrict__ sph, uint32_t ngroups,
    uint32_t scene_fast, const float* __restrict__ rays, uint32_t n, int* __restrict__ out_i,
    float* __restrict__ out_t, const float4* bnd, const uint32_t* perm, uint32_t nclusters) {
    __shared__ uint32_t s_cq[RT_BLOCK_THREADS * RT_CQ_CAP];
    uint32_t* cq = s_cq + (threadIdx.x / 64u) * (64u * RT_CQ_CAP);
#ifdef RT_PROFILE
    PROF_DECL
    PROF_START();
#endif
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* r = rays + (size_t)i * 6;
    float t;
    const int hi = intersect_world<CULL>(grp, sph, ngroups, scene_fast, mk(r[0], r[1], r[2]),
                                         mk(r[3], r[4], r[5]), t, cq,
#ifdef RT_PROFILE
                                         prof_,
#endif
                                         bnd, perm, nclusters);
    out_i[i] = (CULL && hi >= 0) ? (int)perm[hi] : hi;
    out_t[i] = t;
}

__global__ __launch_bounds__(RT_BLOCK_THREADS) void rt_intersect_kernel(
    const float4* __restrict__ grp, const float4* __restrict__ sph, uint32_t ngroups,
    uint32_t scene_fast, const float* __restrict__ rays, uint32_t n, int* __restrict__ out_i,
    float* __restrict__ out_t) {
    intersect_body<false>(grp, sph, ngroups, scene_fast, rays, n, out_i, out_t, nullptr, nullptr, 0);
}

__global__ __launch_bounds__(RT_BLOCK_THREADS) void rt_intersect_cull_kernel(
    const float4* __restrict__ grp, const float4* __restrict__ sph, uint32_t ngroups,
    uint32_t scene_fast, const float* __restrict__ rays, uint32_t n, int* __restrict__ out_i,
    float* __restrict__ out_t, const float4* bnd, const uint32_t* perm, uint32_t nclusters) {
    intersect_body<true>(grp, sph, ngroups, scene_fast, rays, n, out_i, out_t, bnd, perm, nclusters);
}

#ifdef RT_MFMA_FILTER
// The same batch query through the render's matrix-core filter (rt_render_kernel
// takes it for every wave whose rays fit the split's range): the whole wave
// runs the tiles, lanes past n trace a dummy ray that never has a candidate; a
// wave with a ray outside the range takes the VALU filter, as in the render.
// tile_cnt: the matrix-core walk's (tiles walked, tiles without block bounds)
// summed over its waves (rt_debug_intersect_tiles); a VALU-walk wave adds none.
__global__ __launch_bounds__(RT_BLOCK_THREADS) void rt_intersect_mfma_kernel(
    const MfScene mf, const float4* __restrict__ grp,
    const float4* __restrict__ sph, uint32_t ngroups, uint32_t scene_fast,
    const float* __restrict__ rays, uint32_t n, int* __restrict__ out_i, float* __restrict__ out_t,
    unsigned long long* __restrict__ tile_cnt) {
    __shared__ uint32_t s_cq[RT_BLOCK_THREADS * RT_CQ_CAP];
    __shared__ __attribute__((aligned(8))) uint32_t s_cqm[(RT_BLOCK_THREADS / 64) * RT_MF_QW];
    const uint32_t wave = threadIdx.x / 64u;
    PROF_DECL
    PROF_START();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < n;
    const uint64_t lm = rt_ballot(live);
    if (lm == 0) return;  // wave-uniform: the whole wave is past n
    v3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 1.0f);
    if (live) {
        const float* r = rays + (size_t)i * 6;
        o = mk(r[0], r[1], r[2]);
        d = mk(r[3], r[4], r[5]);
    }
    float t = VERY_FAR;
    int hi = -1;
#ifdef RT_ISECT_FORCE_VALU  // diagnostic build: the VALU walk for every wave
    if (false) {
#else
    if (mfma_wave_ok(o, live)) {
#endif
        hi = intersect_world_mfma<true>(mf, scene_fast, o, d, live, lm, t,
                                        s_cqm + wave * RT_MF_QW
#ifdef RT_PROFILE
                                        , prof_
#endif
                                        , tile_cnt);
    } else if (live) {
        hi = intersect_world<false>(grp, sph, ngroups, scene_fast, o, d, t,
                                    s_cq + wave * (64u * RT_CQ_CAP),
#ifdef RT_PROFILE
                                    prof_,
#endif
                                    nullptr, nullptr, 0u);
    }
#ifdef RT_ISECT_PATHTAG  // diagnostic build: bit 24 of the index marks the matrix-core walk
    if (mfma_wave_ok(o, live)) hi += 1 << 24;
#endif
    if (live) {
        out_i[i] = hi;
        out_t[i] = t;
    }
}
#endif

// Fold one frame's results into acc (block order) and, on the frame's last
// pass, write out = acc / spp with alpha 1 (collect.wgsl:115-125). One thread
// per pixel of the processing order k (-> image pixel p = order_to_pixel).
// Launch frame f = blockIdx.y, its blocks in order: those of its pixel item
// (pairs q = f*nblocks + b < qpix, or a later frame's first `lead` blocks),
// already folded by the lane that traced them (first block as is -- or acc +
// it on a later pass -- then acc + block sum) at slot f*npix + k; then its
// block items (the other pairs below qmain), each sum at main_pix + r*npix + k
// (r: the pair's rank among them, rt_dev_path.h fold_frame); then its tail blocks, whose samples' colours
// sit at main_all + (g - g0)*npix + k (g = f*spp + s), summed here exactly as
// a lane sums a block, ((0 + c0) + c1) + ..., in sample order. Each is folded
// as the lane folds (first as is, then acc + it).
// Progressive mode (rt_render_progressive): on the last pass the frame's sum
// is folded into the running sum, prog = prog + sum (prog_mode 2) or
// prog = sum (1, reset), and out = prog / total_spp.
__global__ void rt_collect_kernel(KParams P, const float4* __restrict__ block_sums,
                                  float4* __restrict__ acc, int first_pass,
                                  int last_pass, float spp, float4* __restrict__ out,
                                  float4* __restrict__ prog, int prog_mode, float prog_total) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= P.npix) return;
    const uint32_t f = blockIdx.y + P.collect_f0;  // (earlier frames: written directly)
    const uint32_t p = RT_IDX(order_to_pixel(P, k), P.npix, RT_SITE_OUT);
    float ax = 0.0f, ay = 0.0f, az = 0.0f;
    bool have = !first_pass;
    if (have) {
        const float4 v = acc[p];
        ax = v.x; ay = v.y; az = v.z;
    }
    fold_frame(P, f, k, have, ax, ay, az,
               [&](size_t slot) { return block_sums[RT_IDX(slot, P.chk_slots, RT_SITE_COLLECT)]; });
    if (!last_pass) {
        acc[p] = make_float4(ax, ay, az, 0.0f);
    } else if (prog_mode == 0) {
        const float4 v = make_float4(ax / spp, ay / spp, az / spp, 1.0f);
        float4* const o = out_pixel(P, out, f, p);
        if (P.dsys)
            store_system(o, v);  // host memory or another device's image: write-through
        else
            *o = v;
    } else {
        if (prog_mode == 2) {
            const float4 v = prog[p];
            ax = v.x + ax; ay = v.y + ay; az = v.z + az;
        }
        prog[p] = make_float4(ax, ay, az, 0.0f);
        out[RT_IDX((size_t)f * P.npix + p, P.chk_out, RT_SITE_OUT)] = make_float4(ax / prog_total, ay / prog_total, az / prog_total, 1.0f);
    }
    // P.dsys (RT_FLAG_IMAGE_OUT, or a host-output call writing the caller's
    // registered buffer): the rows may live in another device's memory (rank
    // 0's image mapped over HIP IPC, bevy_raytrace_amd/distributed.py) or in
    // host memory. Every byte the reader takes from this wave was stored
    // above with a system-scope write-through store (sc0 sc1: the line leaves
    // this device's L2, nothing of it stays dirty here), and the wave waits
    // for every one of those stores to be acknowledged (vmcnt(0)) before it
    // ends; the reader acquires (rt_acquire) after the host has seen the
    // launch complete -- MI355X_MICROARCH.md's write-through
    // producer form, which needs no release. P.dsys_release adds the
    // per-wave system-scope release of the round-4 form (buffer_wbl2 sc0 sc1,
    // a write-back of the whole L2: 2.3 ms per N = 8 shard call; A/B only).
    if (P.dsys) {
        if (P.dsys_release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the asm store is invisible to hipcc)
    }
}

// System-scope acquire on every CU of the device (rt_acquire): invalidates
// the vector L1 of the CU and the L2 lines the fence scope covers, so kernels
// launched after it read what other devices wrote into this device's memory
// (after the host observed those writers complete).
__global__ void rt_acquire_kernel() {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Display encode: linear RGBA32F -> sRGB RGBA8 (IEC 61966-2-1 transfer curve),
// channels clamped to [0, 1] (NaN -> 0), alpha 255. The reference shows the
// linear texture through Bevy's sprite pass (ray_trace_output.rs:62-77).
__global__ void rt_srgb8_kernel(const float4* __restrict__ in, uchar4* __restrict__ out,
                                uint64_t npix) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const float4 v = in[i];
    const float c[3] = {v.x, v.y, v.z};
    unsigned char q[3];
    for (int k = 0; k < 3; ++k) {
        float x = c[k] > 0.0f ? fminf(c[k], 1.0f) : 0.0f;  // NaN -> 0
        x = x <= 0.0031308f ? 12.92f * x : 1.055f * powf(x, 1.0f / 2.4f) - 0.055f;
        q[k] = (unsigned char)fminf(fmaxf(rintf(x * 255.0f), 0.0f), 255.0f);
    }
    out[i] = make_uchar4(q[0], q[1], q[2], 255);
}

// gathered: shard_count slabs of max_rows*W float4; image: H*W float4.
// (grid.y = frame: slab k holds shard k's `frames` frames of max_rows rows)
__global__ void rt_assemble_kernel(const float4* __restrict__ gathered, uint32_t max_rows,
                                   uint32_t frames, float4* __restrict__ image, uint32_t width,
                                   uint32_t height, uint32_t row_block, uint32_t shard_count) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (size_t)width * height) return;
    const uint32_t f = blockIdx.y;
    const uint32_t y = (uint32_t)(i / width);
    const uint32_t x = (uint32_t)(i - (size_t)y * width);
    const uint32_t blk = y / row_block;
    const uint32_t k = rt_block_owner(blk, shard_count);
    const uint32_t r = (blk / shard_count) * row_block + (y % row_block);
    image[(size_t)f * width * height + i] =
        gathered[(((size_t)k * frames + f) * max_rows + r) * width + x];
}

extern "C" {

hipError_t rt_launch_render(const KParams* P, const float4* grp, const float4* sph,
                            const float4* shd, const float4* pd,
                            float4* block_sums, uint32_t* work_counter,
                            unsigned long long* seg_counter, uint32_t grid, hipStream_t stream) {
#ifdef RT_SPHERES_LDS
    const size_t dyn = (size_t)(P->ngroups + 1) * 8 * sizeof(float4);
#else
    const size_t dyn = 0;
#endif
    if (P->bnd)
        hipLaunchKernelGGL(rt_render_cull_kernel, dim3(grid), dim3(RT_BLOCK_THREADS), dyn, stream,
                           *P, grp, sph, shd, reinterpret_cast<const PixelEntry*>(pd),
                           block_sums, work_counter, seg_counter, seg_counter + 2);
    else if (!P->mf.A || P->mf.nblk > 16u)  // more than one bound chunk, or no matrix-core walk
        hipLaunchKernelGGL(rt_render_multi_kernel, dim3(grid), dim3(RT_BLOCK_THREADS), dyn, stream, *P,
                           grp, sph, shd, reinterpret_cast<const PixelEntry*>(pd),
                           block_sums, work_counter, seg_counter, seg_counter + 2);
    else
        hipLaunchKernelGGL(rt_render_kernel, dim3(grid), dim3(RT_BLOCK_THREADS), dyn, stream, *P,
                           grp, sph, shd, reinterpret_cast<const PixelEntry*>(pd),
                           block_sums, work_counter, seg_counter, seg_counter + 2);
    return hipGetLastError();
}

hipError_t rt_launch_primary(const KParams* P, float4* pd, hipStream_t stream) {
    const uint32_t T = 256;
    hipLaunchKernelGGL(rt_primary_kernel, dim3((P->npix + T - 1) / T), dim3(T), 0, stream, *P,
                       reinterpret_cast<PixelEntry*>(pd));
    return hipGetLastError();
}

hipError_t rt_launch_collect(const KParams* P, const float4* block_sums,
                             float4* acc, int first_pass, int last_pass, float spp, float4* out,
                             float4* prog, int prog_mode, float prog_total, hipStream_t stream) {
    const uint32_t T = 256;
    if (P->collect_f0 >= P->nframes) return hipSuccess;  // every frame written directly
    hipLaunchKernelGGL(rt_collect_kernel, dim3((P->npix + T - 1) / T, P->nframes - P->collect_f0),
                       dim3(T), 0, stream, *P,
                       block_sums, acc, first_pass, last_pass, spp, out, prog, prog_mode,
                       prog_total);
    return hipGetLastError();
}

hipError_t rt_launch_acquire(uint32_t blocks, hipStream_t stream) {
    hipLaunchKernelGGL(rt_acquire_kernel, dim3(blocks), dim3(64), 0, stream);
    return hipGetLastError();
}

hipError_t rt_launch_srgb8(const float4* in, uchar4* out, uint64_t npix, hipStream_t stream) {
    const uint32_t T = 256;
    hipLaunchKernelGGL(rt_srgb8_kernel, dim3((uint32_t)((npix + T - 1) / T)), dim3(T), 0, stream,
                       in, out, npix);
    return hipGetLastError();
}

hipError_t rt_launch_assemble(const float4* gathered, uint32_t max_rows, uint32_t frames,
                              float4* image, uint32_t width, uint32_t height, uint32_t row_block,
                              uint32_t shard_count, hipStream_t stream) {
    const uint32_t T = 256;
    const size_t n = (size_t)width * height;
    hipLaunchKernelGGL(rt_assemble_kernel, dim3((uint32_t)((n + T - 1) / T), frames), dim3(T), 0,
                       stream, gathered, max_rows, frames, image, width, height, row_block,
                       shard_count);
    return hipGetLastError();
}

hipError_t rt_launch_intersect(const float4* grp, const float4* sph, uint32_t ngroups,
                               uint32_t scene_fast, const float* rays, uint32_t n, int* out_i,
                               float* out_t, const float4* bnd, const uint32_t* perm,
                               uint32_t nclusters, const MfScene* mf, unsigned long long* tile_cnt,
                               hipStream_t stream) {
    const uint32_t T = RT_BLOCK_THREADS;
#ifdef RT_MFMA_FILTER
    if (mf && mf->A && !bnd) {
        hipLaunchKernelGGL(rt_intersect_mfma_kernel, dim3((n + T - 1) / T), dim3(T), 0, stream, *mf,
                           grp, sph, ngroups, scene_fast, rays, n, out_i, out_t, tile_cnt);
        return hipGetLastError();
    }
#else
    (void)mf;
    (void)tile_cnt;
#endif
    if (bnd)
        hipLaunchKernelGGL(rt_intersect_cull_kernel, dim3((n + T - 1) / T), dim3(T), 0, stream, grp,
                           sph, ngroups, scene_fast, rays, n, out_i, out_t, bnd, perm, nclusters);
    else
        hipLaunchKernelGGL(rt_intersect_kernel, dim3((n + T - 1) / T), dim3(T), 0, stream, grp, sph,
                           ngroups, scene_fast, rays, n, out_i, out_t);
    return hipGetLastError();
}

#ifdef RT_WAVE_TRACE
int rt_debug_wave_trace(unsigned long long* out, uint32_t max_waves) {
    if (max_waves > RT_TRACE_MAX_WAVES) max_waves = RT_TRACE_MAX_WAVES;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_trace),
                               (size_t)max_waves * 4 * sizeof(unsigned long long)) == hipSuccess
               ? (int)max_waves : -1;
}
#endif

#ifdef RT_RAY_DUMP
int rt_debug_ray_dump(float* out, uint32_t max_waves) {
    if (max_waves > RT_RAY_DUMP_WAVES) max_waves = RT_RAY_DUMP_WAVES;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ray_dump), (size_t)max_waves * 64 * 2 * sizeof(float4)) ==
                   hipSuccess
               ? (int)max_waves : -1;
}
#endif

#ifdef RT_DRAIN_DUMP
int rt_debug_drain_dump(uint32_t* out, uint32_t max_drains) {
    unsigned int n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_drain_rec), sizeof(n)) != hipSuccess) return -1;
    if (n > RT_DRAIN_DUMP_MAX) n = RT_DRAIN_DUMP_MAX;
    if (n > max_drains) n = max_drains;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_drain_dump), (size_t)n * 64 * 4) != hipSuccess) return -1;
    const unsigned int zero = 0;
    hipMemcpyToSymbol(HIP_SYMBOL(g_drain_rec), &zero, sizeof(zero));
    hipMemcpyToSymbol(HIP_SYMBOL(g_drain_seq), &zero, sizeof(zero));
    return (int)n;
}
#endif

#ifdef RT_CHUNK_TRACE
int rt_debug_chunk_trace(unsigned long long* out, unsigned long long* clk, uint32_t n) {
    if (n > RT_CHUNK_TRACE_MAX) n = RT_CHUNK_TRACE_MAX;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chunk_trace), (size_t)n * 8) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_chunk_clk), (size_t)n * 8) != hipSuccess) return -1;
    return (int)n;
}
#endif

// Diagnostic entry (not part of include/rt_hip.h; tests/test_gpu_math.py):
// the hot path's guarded short forms on caller-given operands, to compare with
// the IEEE operations on zeros, denormals, huge values, inf and NaN.
// mode 0: out[i] = sqrt_x(in[i]); 1: out[3i..3i+2] = normalize_x(in[3i..3i+2]);
// 2: out[3i..3i+2] = div3_x(in[4i..4i+2], in[4i+3]);
// 3: out[i] = div_x(in[2i], in[2i+1], recip_or_nan(in[2i+1])).
__global__ void rt_math_kernel(int mode, const float* __restrict__ in, uint32_t n,
                               float* __restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (mode == 0) {
        out[i] = sqrt_x(in[i]);
    } else if (mode == 1) {
        const v3 r = normalize_x(mk(in[3 * i], in[3 * i + 1], in[3 * i + 2]));
        out[3 * i] = r.x; out[3 * i + 1] = r.y; out[3 * i + 2] = r.z;
    } else if (mode == 2) {
        const v3 r = div3_x(mk(in[4 * i], in[4 * i + 1], in[4 * i + 2]), in[4 * i + 3]);
        out[3 * i] = r.x; out[3 * i + 1] = r.y; out[3 * i + 2] = r.z;
    } else {
        out[i] = div_x(in[2 * i], in[2 * i + 1], recip_or_nan(in[2 * i + 1]));
    }
}

int rt_debug_math(int mode, const float* in_device, uint32_t n, float* out_device) {
    if (mode < 0 || mode > 3 || (n && (!in_device || !out_device))) return -1;
    if (!n) return 0;
    hipLaunchKernelGGL(rt_math_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, mode, in_device, n,
                       out_device);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}

// Diagnostic entry (not part of include/rt_hip.h; tests/test_gpu_mfma_acc.py):
// the matrix-core filter's accumulation, the one hardware property its margin
// proof assumes rather than derives (rt_dev_intersect.h above RT_MF_MU: at
// most one rounding of <= 2^-24 |running sum| per added term, 33 over the two
// chained MFMAs). Per 32 x 32 tile, the walk's own chain -- D = mfma(A1, B1,
// mfma(A0, B0, 0)), v_mfma_f32_32x32x16_f16 twice, K 0..15 then 16..31 --
// built with the product's flags. A: 32 rows x 32 K, B: 32 K x 32 columns,
// f16 bits row-major per tile; D: 32 x 32 f32 row-major. One wave per tile.
#ifdef RT_MFMA_FILTER
__global__ void __launch_bounds__(64) rt_mfma_acc_kernel(const uint16_t* __restrict__ A,
                                                         const uint16_t* __restrict__ B,
                                                         float* __restrict__ D, uint32_t ntiles) {
    const uint32_t l = threadIdx.x, t = blockIdx.x;
    if (t >= ntiles) return;
    const uint16_t* a = A + (size_t)t * 1024;
    const uint16_t* b = B + (size_t)t * 1024;
    h8v a0, a1, b0, b1;
    for (int i = 0; i < 8; ++i) {  // lane l: row / column l & 31, K 8 (l >> 5) + i of each group
        const uint32_t k = 8 * (l >> 5) + i;
        a0[i] = __builtin_bit_cast(_Float16, a[(l & 31) * 32 + k]);
        a1[i] = __builtin_bit_cast(_Float16, a[(l & 31) * 32 + 16 + k]);
        b0[i] = __builtin_bit_cast(_Float16, b[k * 32 + (l & 31)]);
        b1[i] = __builtin_bit_cast(_Float16, b[(16 + k) * 32 + (l & 31)]);
    }
    const f16x zero = {};
    const f16x d = __builtin_amdgcn_mfma_f32_32x32x16_f16(
        a1, b1, __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, zero, 0, 0, 0), 0, 0, 0);
    for (int i = 0; i < 16; ++i) {  // D row (i & 3) + 8 (i >> 2) + 4 (l >> 5), column l & 31
        const uint32_t row = (i & 3) + 8 * (i >> 2) + 4 * (l >> 5);
        D[(size_t)t * 1024 + row * 32 + (l & 31)] = d[i];
    }
}

int rt_debug_mfma_acc(const uint16_t* a_device, const uint16_t* b_device, float* d_device,
                      uint32_t ntiles) {
    if (ntiles && (!a_device || !b_device || !d_device)) return -1;
    if (!ntiles) return 0;
    hipLaunchKernelGGL(rt_mfma_acc_kernel, dim3(ntiles), dim3(64), 0, 0, a_device, b_device, d_device,
                       ntiles);
    return hipDeviceSynchronize() == hipSuccess ? 0 : -3;
}
#endif  // RT_MFMA_FILTER

#ifdef RT_CHECK_BOUNDS
int rt_check_bounds_take(unsigned int out[4]) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_check), 4 * sizeof(unsigned int)) != hipSuccess) return -1;
    if (out[0] == 0) return 0;
    const unsigned int zero[4] = {0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rt_check), zero, sizeof(zero)) == hipSuccess ? 0 : -1;
}
#endif

// resident workgroups per CU of the brute-force and the culled kernel (their
// register and LDS footprints differ: the matrix-core filter's tiles)
hipError_t rt_render_occupancy(int* blocks_per_cu, int* blocks_per_cu_cull) {
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, rt_render_kernel,
                                                                RT_BLOCK_THREADS, 0);
    if (e != hipSuccess) return e;
    int multi = 0;  // the two brute-force kernels take the same grid
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&multi, rt_render_multi_kernel, RT_BLOCK_THREADS, 0);
    if (e != hipSuccess) return e;
    if (multi < *blocks_per_cu) *blocks_per_cu = multi;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu_cull, rt_render_cull_kernel,
                                                        RT_BLOCK_THREADS, 0);
}

}  // extern "C"
