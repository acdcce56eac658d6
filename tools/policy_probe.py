"""Development probe: item policy (env settings) x frames per launch ->
ms per frame for the full frame and the N=8 row shards (predicted speedup)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bevy_raytrace_amd import abi, configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer
import _knobs

wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=os.environ.get("PROBE_LIB") or None)  # PROBE_LIB: another build (A/B)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
FS = [int(x) for x in os.environ.get("PROBE_F", "4,8").split(",")]
buf = torch.empty((max(FS), H, W, 4), dtype=torch.float32, device="cuda:0")


def per_frame(F, n=1, k=0, reps=2):
    rb = configs.pick_row_block(H, n)
    best = 1e9
    for _ in range(reps):
        r.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                               shard_index=k, flags=abi.RT_FLAG_NO_PRIMARY_CACHE)
        st = r.wait()
        best = min(best, st["total_ms"] / F)
    return best


per_frame(2, reps=1)
settings = sys.argv[1:] or ["", "RT_SPLIT_ALL=1"]
for rep in range(2):
    for setting in settings:
        env = dict(p.split("=") for p in setting.split(";") if p)
        _knobs.apply(r, env)
        for F in FS:
            full = per_frame(F)
            sh = [per_frame(F, 8, k) for k in range(8)]
            print(f"[{setting or 'default'}] F={F}: full {full:.3f} ms/frame | N=8 shards "
                  f"{' '.join('%.3f' % t for t in sh)} -> pred {full / max(sh):.2f}x, "
                  f"vs full@default-ish {23.5 / max(sh):.2f}x", flush=True)
        r.tune(None)
