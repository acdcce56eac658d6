"""Development probe: is a launch's fixed cost a warm-up effect? Kernel time of
one F-frame launch of the full frame and of N=8 shard 7 (a) after the GPU
idled (host sync + sleep), (b) as the second of two launches enqueued back to
back on one stream, (c) right behind ~100 ms of GEMMs on the same stream.
usage: python tools/warm_probe.py [F]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 20
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=os.environ.get("PROBE_LIB") or None)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
NO_REUSE = abi.RT_FLAG_NO_PRIMARY_CACHE
buf = torch.empty((2, F, H, W, 4), dtype=torch.float32, device="cuda:0")
s = torch.cuda.Stream()
a = torch.randn(4096, 4096, device="cuda:0", dtype=torch.float16)


def enq(n, k, j):
    rb = configs.pick_row_block(H, n)
    r.render_frames_device(cam, F, buf[j].data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                           shard_index=k, flags=NO_REUSE, stream=s.cuda_stream)


for n, k in ((8, 7), (1, 0), (8, 7)):
    r.reserve(F, W, H, S, D, row_block=configs.pick_row_block(H, n), shard_count=n,
              shard_index=k, flags=NO_REUSE)
    enq(n, k, 0)
    r.wait()
    iso, b2b1, b2b2, hot = [], [], [], []
    for rep in range(3):
        time.sleep(0.05)
        enq(n, k, 0)
        iso.append(r.wait()["kernel_ms"])
        time.sleep(0.05)
        enq(n, k, 0)
        enq(n, k, 1)
        b2b1.append(r.wait()["kernel_ms"])
        b2b2.append(r.wait()["kernel_ms"])
        time.sleep(0.05)
        with torch.cuda.stream(s):
            for _ in range(60):
                a = (a @ a).clamp_(-1, 1)
        enq(n, k, 0)
        hot.append(r.wait()["kernel_ms"])
    f = lambda v: " ".join("%.2f" % x for x in v)
    print(f"N={n} shard {k} F={F}: isolated {f(iso)} | back-to-back 1st {f(b2b1)} 2nd {f(b2b2)} "
          f"| behind GEMMs {f(hot)} ms", flush=True)
