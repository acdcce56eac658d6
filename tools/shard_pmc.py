"""Development probe for PMC passes: one F-frame launch of the full 1080p/64
frame, then one of N=8 shard 7 (row blocks of pick_row_block), in that
order, printing each launch's segment count -- run under
`rocprofv3 --kernel-trace --pmc ...`; the render-kernel dispatches are the
2nd and 4th (primary, render, collect per launch), so counters per segment
compare a shard with the full frame.
usage: python tools/shard_pmc.py [F]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 8
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
buf = torch.empty((F, H, W, 4), dtype=torch.float32, device="cuda:0")
for n, k in ((1, 0), (8, 7)):
    rb = configs.pick_row_block(H, n)
    r.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                           shard_index=k, flags=abi.RT_FLAG_NO_PRIMARY_CACHE)
    st = r.wait()
    print(f"n={n} k={k} F={F}: segments {st['segments']} traced {st['traced_segments']} "
          f"kernel {st['kernel_ms']:.3f} ms", flush=True)
