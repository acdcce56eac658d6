"""Phase breakdown of rt_render_kernel from the -DRT_PROFILE diagnostic build
(tools/librt_hip_prof.so), per launch shape / item policy. Shares (not
absolute times) are meaningful: the stamps perturb the kernel.
usage: python tools/prof_phases.py [F,n,k[,ENV=VAL;ENV=VAL]] ...   (CULL=1: RT_FLAG_CULL)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bevy_raytrace_amd import abi, configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer
import _knobs

LIB = os.environ.get("RT_PROF_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_hip_prof.so")
NAMES = {0: "refill", 1: "filter", 2: "drain", 12: "bookkeep", 3: "shade", 7: "tail"}
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=LIB)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
nsp = len(sc.objects_gpu())
cases = sys.argv[1:] or ["4,1,0", "4,1,0,RT_SPLIT_ALL=1", "4,8,7", "8,8,7"]
# the output holds the largest case's frames (the library cannot check a
# device pointer's extent)
buf = torch.empty((max(int(c.split(",")[0]) for c in cases), H, W, 4), dtype=torch.float32,
                  device="cuda:0")
for case in cases:
    parts = case.split(",", 3)  # F,n,k[,ENV=VAL;ENV=VAL...] (values may hold commas)
    F, n, k = int(parts[0]), int(parts[1]), int(parts[2])
    env = dict(p.split("=", 1) for p in parts[3].split(";")) if len(parts) > 3 else {}
    flags = abi.RT_FLAG_NO_PRIMARY_CACHE | (abi.RT_FLAG_CULL if env.pop("CULL", "0") == "1" else 0)
    _knobs.apply(r, env)
    rb = configs.pick_row_block(H, n)
    for _ in range(2):
        r.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                               shard_index=k, flags=flags)
        st = r.wait()
    c = r.debug_counters()
    r.tune(None)
    tot = sum(c[i] for i in NAMES)
    it = max(c[4], 1)
    print(f"{case}: kernel {st['kernel_ms']:.2f} ms ({st['kernel_ms'] / F:.2f}/frame), "
          f"traced {st['traced_segments']}, wave-iters {c[4]}, lanes/iter {c[9] / it:.1f}, "
          f"wave-cycles/iter {c[8] / it:.0f}", flush=True)
    print("   shares: " + ", ".join(f"{NAMES[i]}={c[i] / tot:.3f}" for i in NAMES) +
          f" | cand-groups/iter {c[5] / it:.2f} drain-max/iter {c[6] / it:.2f} "
          f"exact wave-max {c[13] / it:.2f} full {c[14] / it:.2f} flushes/iter {c[11] / it:.3f} "
          f"groups(VALU)/tiles(MFMA) per iter {c[10] / it:.2f} exact lane-mean {c[15] / max(c[9], 1):.2f} "
          f"c14/lane {c[14] / max(c[9], 1):.2f} | MFMA runs: distinct pixels per half {c[6] / it / 2:.2f}, "
          f"bounce-0 lanes share {c[14] / max(c[9], 1):.2f}",
          flush=True)
