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
                             ("rtiow", scene.rtiow_final_scene(), 192, 108, 8, 16),
                             ("ref", scene.reference_scene(), 160, 90, 4, 3)]:
    sp, mt = sc.objects_gpu(), sc.materials_gpu()
    r.set_scene(sp, mt)
    img, st = r.render(cam, W, H, S, D)
    t = time.time(); ref, segs = O.render(cam, sp, mt, W, H, S, D); tc = time.time() - t
    diff = np.abs(img - ref)
    print(f"{name}: exact={np.array_equal(img, ref)} maxdiff={diff.max():.3g} "
          f"nbad={(diff > 0).any(-1).sum()} rmse={np.sqrt((diff[..., :3]**2).mean()):.3g} "
          f"segs gpu={st['segments']} cpu={segs} oracle_s={tc:.2f} kernel_ms={st['kernel_ms']:.3f}", flush=True)

sc = scene.rtiow_final_scene(); sp, mt = sc.objects_gpu(), sc.materials_gpu()
r.set_scene(sp, mt)
for i in range(3):
    img, st = r.render(cam, 1920, 1080, 64, 16)
    n = len(sp)
    mrays = st['segments'] / st['kernel_ms'] / 1e3
    tf = st['segments'] * 18 * n / st['kernel_ms'] / 1e9
    print(f"1080p64: kernel_ms={st['kernel_ms']:.2f} total_ms={st['total_ms']:.2f} segs={st['segments']} "
          f"Mrays/s={mrays:.1f} TF={tf:.2f} frac={tf/157.3:.3f} nan={np.isnan(img).sum()}", flush=True)
rows = [0, 300, 540, 777, 1079]
ref, segs = O.render_rows(cam, sp, mt, 1920, 1080, 64, 16, rows)
print("1080p rows exact:", np.array_equal(img[rows], ref), np.abs(img[rows] - ref).max())
