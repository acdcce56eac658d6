"""Development probe: render-kernel time against resident workgroups per CU
(knob wg_per_cu; 4 = the occupancy limit) for launches of different sizes --
how much work per lane a launch needs before the full grid pays.

usage: python tools/grid_probe.py   (GPU; prints one line per case)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bevy_raytrace_amd import abi, scene  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.configs import WORKLOADS  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

r = Renderer(0)
cam = default_camera_block()
CASES = [  # (scene, W, H, spp, depth, frames)
    ("reference", 1920, 1080, 1, 3, 1),
    ("rtiow", 1920, 1080, 1, 16, 1),
    ("rtiow", 1920, 1080, 4, 16, 1),
    ("rtiow", 1920, 1080, 16, 16, 1),
    ("rtiow", 1920, 1080, 64, 16, 1),
    ("rtiow", 960, 540, 64, 16, 1),
    ("rtiow", 1920, 1080, 64, 16, 4),
]
scenes = {"reference": WORKLOADS["reference1080"].make_scene(), "rtiow": scene.rtiow_final_scene()}
for name, W, H, S, D, F in CASES:
    sc = scenes[name]
    r.set_scene(sc.objects_gpu(), sc.materials_gpu())
    out = torch.empty((F, H, W, 4), dtype=torch.float32, device="cuda")
    res = []
    for wg in (4, 3, 2, 1):
        r.tune(None)
        r.tune("wg_per_cu", str(wg))
        r.reserve(F, W, H, S, D, flags=abi.RT_FLAG_NO_PRIMARY_CACHE)
        ks, cyc = [], []
        for rep in range(6):
            r.render_frames_device(cam, F, out.data_ptr(), W, H, S, D, frame0=rep * S * F,
                                   flags=abi.RT_FLAG_NO_PRIMARY_CACHE)
            st = r.wait()
            if rep:
                ks.append(st["kernel_ms"])
                cyc.append(st["kernel_ms"] * st["clock_ghz"])
        res.append(f"wg{wg} {np.median(ks):8.3f} ms {np.median(cyc):9.3f} Mcyc")
    lanes = 256 * 4 * 256
    print(f"{name:9s} {W}x{H} spp {S:3d} D {D:2d} F {F}: samples/lane(4 wg) "
          f"{W * H * S * F / lanes:9.1f} | " + " | ".join(res), flush=True)
r.tune(None)
r.close()
