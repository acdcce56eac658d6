"""Development probe: the N-way row shards' render time at the driver's
--steps 20 form (one F-frame launch), every shard, two ways: warm (the 2nd of
two launches enqueued back to back) and as bench.py runs it (a launch after a
host sync and a short idle gap, best of 3), next to the full frame the same
ways; prints the predicted render-only speedup.
usage: [PROBE_TUNE="knob=v;knob=v"] python tools/shard_all_probe.py [F] [N]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=os.environ.get("PROBE_LIB") or None)
for kv in filter(None, (os.environ.get("PROBE_TUNE") or "").split(";")):
    r.tune(*kv.split("=", 1))  # A/B knobs, e.g. PROBE_TUNE="wave_chunk=128;prio_mode=1"
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
    v = []
    for _ in range(2):
        enq(n, k, 0)
        enq(n, k, 1)
        r.wait()
        v.append(r.wait()["kernel_ms"])
    return min(v)


def benchlike(n, k):
    v = []
    enq(n, k, 0)
    r.wait()
    for _ in range(3):
        enq(n, k, 0)
        r.wait()
        torch.cuda.synchronize()
        time.sleep(0.0005)
        enq(n, k, 1)
        v.append(r.wait()["kernel_ms"])
    return min(v)


full_w, full_b = warm(1, 0), benchlike(1, 0)
sw = [warm(N, k) for k in range(N)]
sb = [benchlike(N, k) for k in range(N)]
print(f"F={F} N={N}: full warm {full_w:.2f} ms, bench-like {full_b:.2f} ms", flush=True)
print("shards warm      " + " ".join("%.2f" % x for x in sw) +
      f" | max {max(sw):.2f} -> {full_w / max(sw):.3f}x", flush=True)
print("shards bench-like " + " ".join("%.2f" % x for x in sb) +
      f" | max {max(sb):.2f} -> {full_b / max(sb):.3f}x", flush=True)
