"""What the render kernel executes per launch, per BASELINE workload: the
RT_PROFILE diagnostic build's counters (tools/librt_hip_prof.so, the same
sources with -DRT_PROFILE: per-wave event counts and s_memtime phase clocks,
rt_dev_intersect.h "Prof") for one launch of the bench's own shape, written
raw to a JSON file that tools/executed_summary.py turns into
profiles/executed.json (bench.py's `roofline.executed`).
The counts are the product kernel's work (same code paths; the phase stamps
perturb the timing, not the work). usage:
  python tools/executed.py OUT.json [workload:frames ...]
  (default rtiow1080:20 rtiow4k:1 spheres10k1080:2 rtiow8k:1)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

LIB = os.environ.get("RT_PROF_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                    "librt_hip_prof.so")
# counter index -> name (rt_kernels.hip / rt_dev_intersect.h PROF_MARK / PROF_ADD sites)
NAMES = {
    0: "t_refill", 1: "t_walk", 2: "t_drain", 3: "t_shade", 7: "t_tail", 12: "t_bookkeep",
    16: "t_setup_bounds",
    4: "wave_iterations", 5: "tiles_with_candidate", 6: "distinct_pixels_per_half_sum",
    8: "wave_cycles", 9: "live_lanes", 10: "tiles_walked", 11: "queue_flushes",
    13: "exact_rounds", 14: "bounce0_lanes", 15: "exact_tests", 17: "bound_chunks",
    18: "iters_mfma_walk", 19: "iters_valu_walk", 20: "iters_wide", 21: "exact_tests_full",
    22: "shade_rounds", 23: "group_appends", 24: "valu_walk_queue_max", 25: "valu_walk_full_max",
    26: "t_diag", 27: "top_bound_tiles",
}


def main():
    out = sys.argv[1]
    cases = sys.argv[2:] or ["rtiow1080:20", "rtiow4k:1", "spheres10k1080:2", "rtiow8k:1"]
    cam = default_camera_block()
    res = {"lib": os.path.relpath(LIB), "names": {str(k): v for k, v in NAMES.items()}, "runs": {}}
    r = Renderer(0, lib_path=LIB)
    for case in cases:
        # key:frames, or key:frames:N:k -- row shard k of N (the bench's row blocks)
        parts = case.split(":")
        key, nf = parts[0], int(parts[1])
        nsh, ksh = (int(parts[2]), int(parts[3])) if len(parts) == 4 else (1, 0)
        wl = configs.WORKLOADS[key]
        sc = wl.make_scene()
        sp, mt = sc.objects_gpu(), sc.materials_gpu()
        r.set_scene(sp, mt)
        W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
        rb = configs.pick_row_block(H, nsh)
        rows = len(abi.shard_rows(H, rb, nsh, ksh))
        buf = torch.empty((nf, rows, W, 4), dtype=torch.float32, device="cuda:0")
        flags = abi.RT_FLAG_NO_PRIMARY_CACHE
        runs = []
        for rep in range(2):  # warm, then the recorded launch
            t0 = time.perf_counter()
            r.render_frames_device(cam, nf, buf.data_ptr(), W, H, S, D, 0, rb, nsh, ksh, flags)
            st = r.wait()
            c = r.debug_counters()
            runs.append({"wall_s": time.perf_counter() - t0, "stats": st, "counters": c})
            print(f"{key} x{nf} rep {rep}: kernel {st['kernel_ms']:.1f} ms, "
                  f"iters {c[4]}, tiles {c[10]}, exact rounds {c[13]}", flush=True)
        last = runs[-1]
        if nsh > 1:
            key = f"{key}_shard{ksh}of{nsh}"
        res["runs"][key] = {"frames": nf, "shard": [nsh, ksh], "width": W, "height": H, "spp": S, "max_depth": D,
                            "spheres": int(len(sp)), "stats": last["stats"],
                            "counters": {NAMES.get(i, f"c{i}"): int(v)
                                         for i, v in enumerate(last["counters"])},
                            "kernel_ms_warm": runs[0]["stats"]["kernel_ms"]}
        del buf
        torch.cuda.empty_cache()
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
