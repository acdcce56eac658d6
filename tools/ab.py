"""Interleaved A/B of library builds in ONE process (guide §5.4 rule 24).
usage: python tools/ab.py lib1.so lib2.so ... [--reps N] [--config rtiow1080]"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from bevy_raytrace_amd import abi
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.configs import WORKLOADS
from bevy_raytrace_amd.renderer import Renderer

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--config", default="rtiow1080")
ap.add_argument("--spp", type=int, default=0)
ap.add_argument("--flags", type=int, default=abi.RT_FLAG_NO_PRIMARY_CACHE)
ap.add_argument("--shards", type=int, default=1, help="render one row shard of N (tail-heavy)")
ap.add_argument("--shard-index", type=int, default=0)
a = ap.parse_args()
wl = WORKLOADS[a.config]
sc = wl.make_scene(); sp, mt = sc.objects_gpu(), sc.materials_gpu()
S = a.spp or wl.spp
cam = default_camera_block()
rs = []
for p in a.libs:
    r = Renderer(0, lib_path=p); r.set_scene(sp, mt); rs.append(r)
ref = None
times = {p: [] for p in a.libs}
for rep in range(a.reps + 1):
    for p, r in zip(a.libs, rs):
        from bevy_raytrace_amd.configs import pick_row_block
        img, st = r.render(cam, wl.width, wl.height, S, wl.max_depth, flags=a.flags,
                           row_block=pick_row_block(wl.height, a.shards), shard_count=a.shards,
                           shard_index=a.shard_index)
        if rep == 0:
            if ref is None:
                ref = img
            ok = np.array_equal(img, ref, equal_nan=True)
            print(f"{os.path.basename(p)}: identical_to_first={ok}", flush=True)
            continue
        times[p].append(st["kernel_ms"])
base = np.array(times[a.libs[0]])
for p in a.libs:
    t = np.array(times[p])
    segs = st["traced_segments"]
    tf = segs * 18 * len(sp) / (np.median(t) * 1e-3) / 1e12
    ratio = t / base  # same-round ratio vs the first library (round-to-round drift cancels)
    print(f"{os.path.basename(p):40s} median {np.median(t):8.3f} ms  min {t.min():8.3f}  "
          f"frac {tf/157.3:.3f}  ratio-vs-first median {np.median(ratio):.4f} "
          f"[{ratio.min():.4f}, {ratio.max():.4f}]", flush=True)
