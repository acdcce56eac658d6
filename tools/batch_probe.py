"""Development probe: frames per launch (rt_render_frames_device) x tail-split
length (RT_SPLIT_SCALE) -> ms per frame, full frame and the N=8 row shards."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bevy_raytrace_amd import abi, configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

wl = configs.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "rtiow1080"]
flags = int(sys.argv[2]) if len(sys.argv) > 2 else abi.RT_FLAG_NO_PRIMARY_CACHE
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
buf = torch.empty((8, H, W, 4), dtype=torch.float32, device="cuda:0")


def per_frame(F, n=1, k=0, reps=2):
    rb = configs.pick_row_block(H, n)
    best = 1e9
    for _ in range(reps):
        r.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                               shard_index=k, flags=flags)
        st = r.wait()
        best = min(best, st["total_ms"] / F)
    return best


per_frame(2, reps=1)
for tail in (sys.argv[3].split(";") if len(sys.argv) > 3 else ("2,1,1",)):
    r.tune(tail=tail)
    for F in (1, 2, 4, 8):
        full = per_frame(F)
        sh = [per_frame(F, 8, k) for k in (0, 3, 7)]
        print(f"tail={tail} F={F}: full {full:.3f} ms/frame | N=8 shards {' '.join('%.3f' % t for t in sh)}"
              f" -> pred {full / max(sh):.2f}x", flush=True)
r.tune(split_all=1)
print(f"split-all F=1: full {per_frame(1):.3f} | N=8 k=7 {per_frame(1, 8, 7):.3f}", flush=True)
