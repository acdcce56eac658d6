"""Development probe: per-shard render time of the N-way row tiling for
several row_block sizes (12-frame launches, primary reuse off): the slowest
shard sets the N-GPU frame time; the sum over shards shows the coherence cost
of blocks that do not hold whole 8x8 pixel tiles.
usage: python tools/rowblock_probe.py N B1 B2 ..."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bevy_raytrace_amd import abi, configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
N = int(sys.argv[1])
Bs = [int(b) for b in sys.argv[2:]] or [configs.pick_row_block(H, N), 8]
F = int(os.environ.get("PROBE_F", "20"))
buf = torch.empty((F, H, W, 4), dtype=torch.float32, device="cuda:0")


def shard_ms(B, k):
    best = 1e9
    for _ in range(2):
        r.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D, row_block=B, shard_count=N,
                               shard_index=k, flags=abi.RT_FLAG_NO_PRIMARY_CACHE)
        st = r.wait()
        best = min(best, st["total_ms"] / F)
    return best


r.render_frames_device(cam, 2, buf.data_ptr(), W, H, S, D, flags=abi.RT_FLAG_NO_PRIMARY_CACHE)
r.wait()
for B in Bs:
    t = [shard_ms(B, k) for k in range(N)]
    rows = [len(abi.shard_rows(H, B, N, k)) for k in range(N)]
    print(f"N={N} B={B}: rows {min(rows)}-{max(rows)}, ms/frame per shard "
          f"{' '.join('%.3f' % v for v in t)} | max {max(t):.3f} sum {sum(t):.2f}", flush=True)
