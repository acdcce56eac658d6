"""Quick GPU parity + timing probe (development tool)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from bevy_raytrace_amd import scene
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer
from oracle import oracle as O

cam = default_camera_block()
r = Renderer(0)
for name, sc, W, H, S, D in [("config1", scene.config1_scene(), 400, 225, 16, 8),
                             ("rtiow", scene.rtiow_final_scene(), 192, 108, 12, 16),
                             ("ref", scene.reference_scene(), 160, 90, 4, 3)]:
    sp, mt = sc.objects_gpu(), sc.materials_gpu()
    r.set_scene(sp, mt)
    ref, segs = O.render(cam, sp, mt, W, H, S, D)
    for flags in (0, 1):
        img, st = r.render(cam, W, H, S, D, flags=flags)
        eq = np.array_equal(img, ref, equal_nan=True)
        diff = np.nan_to_num(np.abs(img - ref))
        print(f"{name} flags={flags}: exact={eq} maxdiff={diff.max():.3g} "
              f"segs gpu={st['segments']} traced={st['traced_segments']} cpu={segs} kernel_ms={st['kernel_ms']:.3f}", flush=True)

sc = scene.rtiow_final_scene(); sp, mt = sc.objects_gpu(), sc.materials_gpu()
r.set_scene(sp, mt)
n = len(sp)
for flags in (0, 1, 0, 1):
    img, st = r.render(cam, 1920, 1080, 64, 16, flags=flags)
    mrays = st['segments'] / st['kernel_ms'] / 1e3
    tf = st['traced_segments'] * 18 * n / st['kernel_ms'] / 1e9
    print(f"1080p64 flags={flags}: kernel_ms={st['kernel_ms']:.2f} total_ms={st['total_ms']:.2f} segs={st['segments']} "
          f"traced={st['traced_segments']} Mrays/s={mrays:.1f} TF(traced)={tf:.2f} frac={tf/157.3:.3f} nan={np.isnan(img[...,0]).sum()}", flush=True)
rows = [0, 300, 415, 540, 777, 1079]
ref, segs = O.render_rows(cam, sp, mt, 1920, 1080, 64, 16, rows)
print("1080p rows exact:", np.array_equal(img[rows], ref, equal_nan=True))
sc = scene.ten_thousand_scene(); sp, mt = sc.objects_gpu(), sc.materials_gpu()
r.set_scene(sp, mt)
img, st = r.render(cam, 1920, 1080, 8, 16)
tf = st['traced_segments'] * 18 * len(sp) / st['kernel_ms'] / 1e9
print(f"10k spp8: kernel_ms={st['kernel_ms']:.2f} segs={st['segments']} traced={st['traced_segments']} Mrays/s={st['segments']/st['kernel_ms']/1e3:.1f} frac={tf/157.3:.3f}")
