"""Development probe: primary-hit reuse with 2-/4-sample tail items, small
images first, then the 1080p single frame; stops at the first error."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bevy_raytrace_amd import abi, scene  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402
from oracle import oracle as O  # noqa: E402

sc = scene.rtiow_final_scene()
sp, mt = sc.objects_gpu(), sc.materials_gpu()
cam = default_camera_block()
r = Renderer(0)
r.set_scene(sp, mt)
cases = [(72, 40, 64, 10, "0,0.001,0.001", 0), (72, 40, 64, 10, "0.001,0.001,0.001", 0),
         (72, 40, 64, 10, "0,0.001,0.001", abi.RT_FLAG_NO_PRIMARY_CACHE),
         (1920, 1080, 64, 16, "0,0,6", 0), (1920, 1080, 64, 16, "0,1,1", abi.RT_FLAG_NO_PRIMARY_CACHE),
         (1920, 1080, 64, 16, "0,1,1", 0)]
for W, H, S, D, tail, flags in cases:
    r.tune(None)
    r.tune(tail=tail)
    print(f"case {W}x{H} S={S} tail={tail} flags={flags} ...", flush=True)
    img, st = r.render(cam, W, H, S, D, flags=flags)
    if W < 100:
        ref, segs = O.render(cam, sp, mt, W, H, S, D)
        ok = np.array_equal(img, ref, equal_nan=True) and st["segments"] == segs
    else:
        ok = True
    print(f"  done: segments {st['segments']} exact={ok}", flush=True)
