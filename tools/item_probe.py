"""Development probe: warm kernel time (the 3rd of 3 launches enqueued back to
back on one stream) of one F-frame launch of the full frame and of N=8 shard
7, per knob setting, plus an idle-gap sweep (host sync, sleep g ms, launch).
usage: python tools/item_probe.py F "setting;..." ...   (e.g. block_region=100000)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

F = int(sys.argv[1])
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=os.environ.get("PROBE_LIB") or None)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
NO_REUSE = abi.RT_FLAG_NO_PRIMARY_CACHE
buf = torch.empty((2, F, H, W, 4), dtype=torch.float32, device="cuda:0")
s = torch.cuda.Stream()


def enq(n, k, j):
    rb = configs.pick_row_block(H, n)
    r.render_frames_device(cam, F, buf[j].data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                           shard_index=k, flags=NO_REUSE, stream=s.cuda_stream)


def warm(n, k):
    out = []
    for _ in range(2):
        enq(n, k, 0)
        enq(n, k, 1)
        r.wait()
        out.append(r.wait()["kernel_ms"])
    return min(out)


for setting in sys.argv[2:] or [""]:
    kn = {}
    for p in setting.split(";"):
        if p:
            name, v = p.split("=", 1)
            kn[name] = v
    r.tune(None)
    for name, v in kn.items():
        r.tune(name, v)
    res = []
    for n, k in ((1, 0), (8, 7), (8, 0)):
        res.append(warm(n, k))
    print(f"[{setting or 'default'}] F={F} warm: full {res[0]:.2f} ms, shard 7 {res[1]:.2f}, "
          f"shard 0 {res[2]:.2f} -> {res[0] / max(res[1], res[2]):.3f}x", flush=True)
r.tune(None)
for n, k in ((8, 7),):
    for g in (0.0, 0.0002, 0.001, 0.005, 0.02, 0.1):
        v = []
        for _ in range(3):
            enq(n, k, 0)
            r.wait()
            if g:
                time.sleep(g)
            enq(n, k, 1)
            v.append(r.wait()["kernel_ms"])
        print(f"idle gap {g * 1e3:.1f} ms before a shard-{k} launch: " +
              " ".join("%.2f" % x for x in v) + " ms", flush=True)
