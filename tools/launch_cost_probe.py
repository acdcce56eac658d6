"""Development probe: per-launch fixed cost vs per-frame cost of the N=8 row
shard and of the full frame. Times one launch of F frames for several F and
fits t(F) = fixed + F * per_frame, per knob setting (tools/_knobs.py names).
usage: python tools/launch_cost_probe.py [SETTING ...]   e.g. RT_TAIL=0,0,0"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _knobs  # noqa: E402
from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=os.environ.get("PROBE_LIB") or None)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
FS = [int(x) for x in os.environ.get("PROBE_F", "5,10,20,40").split(",")]
NO_REUSE = abi.RT_FLAG_NO_PRIMARY_CACHE
buf = torch.empty((max(FS), H, W, 4), dtype=torch.float32, device="cuda:0")


def launch_ms(F, n, k):
    rb = configs.pick_row_block(H, n)
    best = 1e9
    for _ in range(2):
        r.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                               shard_index=k, flags=NO_REUSE)
        best = min(best, r.wait()["total_ms"])
    return best


launch_ms(2, 1, 0)
for setting in sys.argv[1:] or [""]:
    _knobs.apply(r, dict(p.split("=", 1) for p in setting.split(";") if p))
    for n, k in ((1, 0), (8, 7), (8, 0)):
        t = [launch_ms(F, n, k) for F in FS]
        slope, fixed = np.polyfit(FS, t, 1)
        print(f"[{setting or 'default'}] N={n} shard {k}: " +
              " ".join(f"F={F}:{v:.2f}" for F, v in zip(FS, t)) +
              f" ms -> fixed {fixed:.2f} ms + {slope:.3f} ms/frame", flush=True)
    r.tune(None)
