"""Tail shape of rt_render_kernel from the -DRT_WAVE_TRACE diagnostic build
(tools/librt_hip_trace.so): per-wave start/end/queue-exhausted times."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from bevy_raytrace_amd import configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer
import _knobs

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_hip_trace.so")
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=LIB)
r.lib.rt_debug_wave_trace.restype = ctypes.c_int
_knobs.from_environ(r, os.environ)  # RT_WG_PER_CU=6 etc.
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H = wl.width, wl.height
CASES = [tuple(int(v) for v in c.split(",")) for c in
         os.environ.get("TRACE_CASES", "4,8,7;8,8,7;8,8,7;4,1,0").split(";")]
buf = torch.empty((max(c[0] for c in CASES), H, W, 4), dtype=torch.float32, device="cuda:0")
MAXW = 32768


def trace(S, n=1, k=0, rb=8, D=16, F=1):
    for _ in range(2):
        r.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                               shard_index=k, flags=1)
        st = r.wait()
    out = np.zeros(MAXW * 4, dtype=np.uint64)
    r.lib.rt_debug_wave_trace(out.ctypes.data_as(ctypes.c_void_p), MAXW)
    t = out.reshape(-1, 4)
    t = t[t[:, 1] > 0].astype(np.int64)
    t0 = t[:, 0].min()
    start, end, ex = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0, t[:, 2]
    ex = np.where(ex > 0, (ex - t0) / 100.0, np.nan)
    if np.isnan(ex).all():  # lite build: start/end only
        ex = np.full_like(end, end.min())
    iters = (t[:, 3] & 0xFFFF).astype(np.int64)
    after = ((t[:, 3] >> 16) & 0xFFFF).astype(np.int64)
    items = (t[:, 3] >> 32).astype(np.int64)
    span = end.max()
    eff = (end - start).sum() / (len(t) * span)
    q = np.percentile(end, [0, 10, 50, 90, 99, 100])
    print(f"F={F} S={S} n={n} k={k}: kernel {st['kernel_ms']:.3f} ms, waves {len(t)}, span {span:.1f} us, "
          f"start max {start.max():.1f} us, queue dry at {np.nanmin(ex):.1f} us, "
          f"wave-busy eff {eff:.3f}", flush=True)
    print("   end pct (0/10/50/90/99/100) us: " + " ".join(f"{v:.0f}" for v in q))
    print(f"   iters/wave mean {iters.mean():.1f} max {iters.max()}, items/wave mean {items.mean():.1f}; "
          f"us/iter {span / iters.mean():.2f}; iters after dry mean {after.mean():.1f} "
          f"p90 {np.percentile(after, 90):.0f} max {after.max()}")
    late = end > np.percentile(end, 90)
    print(f"   slowest 10% waves: iters after dry mean {after[late].mean():.1f}, "
          f"us per post-dry iter {((end - ex)[late] / np.maximum(after[late], 1)).mean():.1f}")
    order = np.argsort(end)[-5:]
    for w in order[::-1]:
        print(f"   straggler wave {w}: end {end[w]:.0f} us, dry seen {ex[w]:.0f} us, iters {iters[w]}, "
              f"after dry {after[w]}, items {items[w]}")
    hist, edges = np.histogram(end, bins=20, range=(0, span))
    print("   ends histogram:", hist.tolist())


for F, n, k in CASES:
    trace(64, n, k, configs.pick_row_block(H, n), F=F)
