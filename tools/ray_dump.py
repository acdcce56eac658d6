"""Development probe: the rays every lane of the first 1024 waves holds at one
loop iteration of the headline launch (tools/librt_hip_raydump.so, built with
-DRT_RAY_DUMP), saved for the CPU analysis of the matrix-core walk's block
skipping (tools/sim_block_cull.py --dump).
usage: python tools/ray_dump.py <out.npy>"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_hip_raydump.so")
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
r = Renderer(0, lib_path=LIB)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
F = 20
out = torch.empty((F, wl.height, wl.width, 4), dtype=torch.float32, device="cuda:0")
r.render_frames_device(default_camera_block(), F, out.data_ptr(), wl.width, wl.height, wl.spp,
                       wl.max_depth, flags=abi.RT_FLAG_NO_PRIMARY_CACHE)
st = r.wait()
buf = np.zeros((1024, 64, 2, 4), dtype=np.float32)
r.lib.rt_debug_ray_dump.restype = ctypes.c_int
r.lib.rt_debug_ray_dump.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
n = r.lib.rt_debug_ray_dump(buf.ctypes.data_as(ctypes.c_void_p), 1024)
np.save(sys.argv[1], buf)
print("waves", n, "kernel ms", st["kernel_ms"], flush=True)
r.close()
