"""Development probe: per-lane candidate counts of a sample of the matrix-core
walk's drains (every 61st drain, up to 65,536) in one bench-shaped launch, from
the -DRT_DRAIN_DUMP build (tools/librt_hip_draindump.so), for the CPU model of
drain balancing schemes (tools/drain_model.py).
usage: python tools/drain_dump.py <workload> <out.npy>"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_hip_draindump.so")
wl = configs.WORKLOADS[sys.argv[1]]
sc = wl.make_scene()
r = Renderer(0, lib_path=LIB)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
F = {"rtiow1080": 20, "spheres10k1080": 2}.get(wl.key, 1)
out = torch.empty((F, wl.height, wl.width, 4), dtype=torch.float32, device="cuda:0")
r.render_frames_device(default_camera_block(), F, out.data_ptr(), wl.width, wl.height, wl.spp,
                       wl.max_depth, flags=abi.RT_FLAG_NO_PRIMARY_CACHE)
st = r.wait()
buf = np.zeros((65536, 64), dtype=np.uint32)
r.lib.rt_debug_drain_dump.restype = ctypes.c_int
r.lib.rt_debug_drain_dump.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
n = r.lib.rt_debug_drain_dump(buf.ctypes.data_as(ctypes.c_void_p), 65536)
np.save(sys.argv[2], buf[:max(n, 0)])
e, b = buf[:n] & 0xFFFF, buf[:n] >> 16
print(wl.key, "drains", n, "kernel ms", round(st["kernel_ms"], 2),
      "mean tests/lane %.3f  mean max %.3f  mean entries/lane %.3f  mean max entries %.3f" % (
          b.mean(), b.max(1).mean(), e.mean(), e.max(1).mean()), flush=True)
r.close()
