"""Development probe: what splitting an N-way shard's launch costs. Shard k of
N (the bench's row blocks) of the headline, F frames written with
RT_FLAG_IMAGE_OUT into a whole image on this device (the collect's
system-scope stores, here into local memory), as one launch or as two calls
of a + b frames back to back on one stream: render-kernel ms, the rest of
the call (primary table, collect), and the stream's wall time (events), best
of 3 after a warm-up.
usage: python tools/split_probe.py [F] [N] [k] [a,b ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bevy_raytrace_amd import abi, configs  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = int(sys.argv[2]) if len(sys.argv) > 2 else 8
K = int(sys.argv[3]) if len(sys.argv) > 3 else N - 1
splits = [tuple(int(x) for x in s.split(",")) for s in sys.argv[4:]] or [(F,), (10, 10), (14, 6), (16, 4)]
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=os.environ.get("PROBE_LIB") or None)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
rb = configs.pick_row_block(H, N)
rows = abi.shard_rows(H, rb, N, K)
img = torch.empty((F, H, W, 4), dtype=torch.float32, device="cuda:0")
s = torch.cuda.Stream()
IMAGE = os.environ.get("PROBE_PACKED", "0") != "1"  # PROBE_PACKED=1: the shard's packed rows, plain stores
FL = abi.RT_FLAG_NO_PRIMARY_CACHE | (abi.RT_FLAG_IMAGE_OUT if IMAGE else 0)
for kv in filter(None, os.environ.get("PROBE_TUNE", "").split(";")):  # knob=value;knob=value
    r.tune(*kv.split("=", 1))
r.reserve(F, W, H, S, D, row_block=rb, shard_count=N, shard_index=K, flags=FL)


def run(parts):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(s)
    first, pend, stats = 0, 0, []
    for nf in parts:
        if pend == abi.RT_MAX_PENDING:
            stats.append(r.wait())
            pend -= 1
        dst = img[first].data_ptr() if IMAGE else img.data_ptr() + first * len(rows) * W * 16
        r.render_frames_device(cam, nf, dst, W, H, S, D, first * S, rb, N, K, FL,
                               stream=s.cuda_stream)
        first += nf
        pend += 1
    while pend:
        stats.append(r.wait())
        pend -= 1
    e1.record(s)
    torch.cuda.synchronize()
    return (e0.elapsed_time(e1), sum(x["kernel_ms"] for x in stats),
            sum(x["total_ms"] - x["kernel_ms"] for x in stats))


for parts in splits:
    run(parts)
    best = min((run(parts) for _ in range(3)), key=lambda v: v[0])
    print(f"shard {K}/{N} F={F} {'image' if IMAGE else 'packed'} {os.environ.get('PROBE_TUNE', '')} "
          f"split {'+'.join(map(str, parts))}: wall {best[0]:.3f} ms, "
          f"render {best[1]:.3f} ms, rest of calls {best[2]:.3f} ms", flush=True)
