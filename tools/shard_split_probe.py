"""Development probe: wall time of F frames of one row shard (or the full
frame) rendered as one persistent launch on one stream, against the same
frames split into L launches alternating over the library's two slot streams
(rt_render_frames_device with stream NULL), so a launch's drain overlaps the
next launch's start. Prints ms per frame and the predicted N=8 speedup
(full frame / slowest shard).
usage: python tools/shard_split_probe.py [F] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 20
REPS = int(sys.argv[2]) if len(sys.argv) > 2 else 2
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=os.environ.get("PROBE_LIB") or None)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
NO_REUSE = abi.RT_FLAG_NO_PRIMARY_CACHE
buf = torch.empty((F, H, W, 4), dtype=torch.float32, device="cuda:0")
one = torch.cuda.Stream()


def wall(n, k, launches, split_streams):
    rb = configs.pick_row_block(H, n)
    rows = len(abi.shard_rows(H, rb, n, k))
    sizes = [F // launches + (1 if j < F % launches else 0) for j in range(launches)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    first, pending = 0, 0
    for nf in sizes:
        if pending == abi.RT_MAX_PENDING:
            r.wait()
            pending -= 1
        ptr = buf.data_ptr() + first * rows * W * 16
        r.render_frames_device(cam, nf, ptr, W, H, S, D, first * S, rb, n, k, NO_REUSE,
                               stream=None if split_streams else one.cuda_stream)
        first += nf
        pending += 1
    while pending:
        r.wait()
        pending -= 1
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / F


r.reserve(F, W, H, S, D, flags=NO_REUSE)
for n, k in ((1, 0), (8, 0), (8, 7)):
    r.reserve(F, W, H, S, D, row_block=configs.pick_row_block(H, n), shard_count=n,
              shard_index=k, flags=NO_REUSE)
wall(1, 0, 1, False)
for rep in range(REPS):
    for launches, split in ((1, False), (2, True), (4, True)):
        full = wall(1, 0, launches, split)
        sh = [wall(8, k, launches, split) for k in (0, 3, 7)]
        print(f"rep {rep} F={F} launches={launches} {'2 streams' if split else '1 stream'}: "
              f"full {full:.3f} ms/frame | shards 0,3,7 {' '.join('%.3f' % t for t in sh)} "
              f"-> pred {full / max(sh):.2f}x", flush=True)
