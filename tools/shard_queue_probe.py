"""Queue-region settings on one row shard of the N-GPU layout (development
tool): shard k of N of the headline frame rendered as one FPL-frame launch
(rt_render_frames_device, as a bench rank does), for several (block_region,
tail) knob settings, interleaved over reps; prints the median kernel ms per
setting and checks that every setting writes the same bits.

usage: python tools/shard_queue_probe.py [N] [k] [FPL] [reps] "br=96,tail=0:0:12" ...
"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from bevy_raytrace_amd import configs
from bevy_raytrace_amd.abi import shard_rows
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
FPL = int(sys.argv[3]) if len(sys.argv) > 3 else 24
REPS = int(sys.argv[4]) if len(sys.argv) > 4 else 4
SETTINGS = sys.argv[5:] or ["br=96,tail=0:0:6"]

wl = configs.WORKLOADS[configs.HEADLINE]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
flags = 1  # headline: no primary reuse
rb = configs.pick_row_block(H, N)
rows = len(shard_rows(H, rb, N, K))
buf = torch.empty((FPL, rows, W, 4), dtype=torch.float32, device="cuda:0")


def apply(setting):
    r.tune(None)
    for kv in setting.split(","):
        name, val = kv.split("=")
        name = {"br": "block_region"}.get(name, name)
        r.tune(name, val.replace(":", ","))


def once(setting):
    apply(setting)
    buf.zero_()
    torch.cuda.synchronize()  # the render runs on the context's own stream
    r.render_frames_device(cam, FPL, buf.data_ptr(), W, H, S, D, 0, rb, N, K, flags)
    st = r.wait()
    # bit pattern checksum (NaN-safe): sum of the words as int64
    return st["kernel_ms"], int(buf.view(torch.int32).to(torch.int64).sum().item())


ref_sum = None
LABELS = [f"{i}:{s}" for i, s in enumerate(SETTINGS)]
times = {l: [] for l in LABELS}
for rep in range(REPS + 1):
    for lab, s in zip(LABELS, SETTINGS):
        ms, cs = once(s)
        if rep == 0:
            if ref_sum is None:
                ref_sum = cs
            print(f"{lab}: checksum {'same' if cs == ref_sum else 'DIFFERENT'}", flush=True)
            continue
        times[lab].append(ms)
base = float(np.median(times[LABELS[0]]))
for s in LABELS:
    m = float(np.median(times[s]))
    print(f"N={N} k={K} FPL={FPL} {s:28s} median {m:8.3f} ms  min {min(times[s]):8.3f}  "
          f"ratio {m / base:.4f}", flush=True)
