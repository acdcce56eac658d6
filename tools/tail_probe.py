"""Development probe: is the N-shard overhead a fixed tail or lost coherence?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bevy_raytrace_amd import configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H = 1920, 1080
buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")


def run(S, n=1, k=0, rb=8, reps=3, D=16):
    ts = []
    for _ in range(reps):
        r.render_device(cam, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                        shard_index=k, flags=1)
        st = r.wait()
        ts.append(st["kernel_ms"])
    return min(ts), st["segments"]


run(8)
for S in (8, 16, 32, 64, 128):
    t, seg = run(S)
    print(f"full S={S}: {t:.3f} ms  segs {seg}  ns/seg {t * 1e6 / seg:.4f}", flush=True)
for rb in (135, 45, 27, 5, 1):
    ts = [run(64, 8, k, rb)[0] for k in range(8)]
    print(f"N=8 rb={rb}: max {max(ts):.3f} sum {sum(ts):.3f} " + " ".join('%.2f' % t for t in ts),
          flush=True)
