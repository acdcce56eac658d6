"""tools/executed.py's raw counters (the RT_PROFILE build, one bench-shaped
launch per workload) -> profiles/executed.json, the `roofline.executed` block
of bench.py: per frame what the render kernel executes -- wave iterations,
matrix-core tiles (walk tiles, block-bound and chunk-bound tiles) and their
f16 flops, exact fp32 sphere tests (all, and past the certain-miss shortcut)
against the reference's N per segment, shading rounds -- and the share of
wave time per phase (s_memtime stamps around each phase; the stamps and the
diagnostic reductions are timed apart, c[26], and left out).
usage: python tools/executed_summary.py <executed_raw.json> [pmc_traffic.json]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MFMA_32x32x16 = 2 * 32 * 32 * 16  # flops of one v_mfma_f32_32x32x16_f16
MFMA_32x32x8 = 2 * 32 * 32 * 8
# fp32 flops of one exact test (intersect.wgsl:97-115 as exact_core runs it):
# oc 3, half_b 5, |oc|^2 5 and the shortcut's compare product 1 = 14; past
# the shortcut + sqrt, lo*lo - r^2 2, disc 3, sqrt, one root 2 + divide = 24
FLOPS_SHORT, FLOPS_FULL = 14, 24
PHASES = ("t_refill", "t_setup_bounds", "t_walk", "t_drain", "t_bookkeep", "t_shade")


def summarize(run):
    c, st, nf = run["counters"], run["stats"], run["frames"]
    it = max(c["wave_iterations"], 1)
    segs = st["segments"]
    bound = c["bound_chunks"] + c.get("top_bound_tiles", 0)
    mf_flops = (c["tiles_walked"] * 2 * MFMA_32x32x16 +
                bound * 2 * (2 * MFMA_32x32x16 + MFMA_32x32x8))
    full, tests = c["exact_tests_full"], c["exact_tests"]
    tot = sum(c[p] for p in PHASES)
    per_frame = {
        "segments": segs / nf,
        "wave_iterations": c["wave_iterations"] / nf,
        "walk_tiles_32x32": c["tiles_walked"] / nf,
        "bound_chunk_tiles": c["bound_chunks"] / nf,
        "chunk_level_bound_tiles": c.get("top_bound_tiles", 0) / nf,
        "mfma_f16_flops": mf_flops / nf,
        "exact_tests": tests / nf,
        "exact_tests_past_shortcut": full / nf,
        "exact_fp32_flops": (FLOPS_SHORT * (tests - full) + FLOPS_FULL * full) / nf,
        "exact_wave_rounds": c["exact_rounds"] / nf,
        "shading_rounds": c["shade_rounds"] / nf,
    }
    n = run["spheres"]
    per_segment = {
        "reference_sphere_tests": n,
        "exact_tests": tests / segs,
        "exact_tests_past_shortcut": full / segs,
        "walk_tiles_per_wave_iteration": c["tiles_walked"] / it,
        "bound_chunks_per_wave_iteration": bound / it,
        "exact_rounds_per_wave_iteration": c["exact_rounds"] / it,
        "live_lanes_per_wave_iteration": c["live_lanes"] / it,
    }
    # (sphere, ray) pairs the matrix-core walk filters per traced segment:
    # each walked 32x32 tile covers 1,024 pairs of the wave's 64 rays
    per_segment["matrix_core_pairs_filtered"] = c["tiles_walked"] * 1024 / segs
    share = {p[2:]: c[p] / tot for p in PHASES}
    useful = share["drain"] + share["shade"]
    return {
        "per_frame": {k: round(v, 1) for k, v in per_frame.items()},
        "per_segment": {k: round(v, 4) for k, v in per_segment.items()},
        "phase_wave_time_share": {k: round(v, 4) for k, v in share.items()},
        "useful_wave_time_share": round(useful, 4),
        "profile_build_kernel_ms": round(st["kernel_ms"], 2),
        "diagnostic_share_excluded": round(c["t_diag"] / (tot + c["t_diag"]), 4),
    }


def main():
    raw = json.load(open(sys.argv[1]))
    path = os.path.join(ROOT, "profiles", "executed.json")
    # the workloads of this raw record replace theirs; the others are kept
    out = json.load(open(path)) if os.path.exists(path) else {}
    for key, run in raw["runs"].items():
        e = summarize(run)
        e["source"] = ("tools/executed.py (RT_PROFILE build of the same sources, one launch of "
                       f"{run['frames']} frame(s) as the bench runs it) -> tools/executed_summary.py")
        e["note"] = ("counts are the product kernel's work (the same code paths); phase shares are "
                     "shares of WAVE time (issue + waits) from s_memtime stamps at the phase "
                     "boundaries, the stamps' own cost and the diagnostic reductions excluded; "
                     "'useful' = the exact fp32 sphere tests (drain) + shading, the reference "
                     "algorithm's own per-segment arithmetic; setup_bounds + walk are the "
                     "matrix-core filter that replaces its brute-force loop")
        out[key] = e
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
