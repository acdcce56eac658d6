"""Per-frame cost of an animated scene on the GPU box: the
reference's own frame shape (1080p, 1 spp, depth 3, the shim's call) with one
sphere moved before every frame -- rt_update_spheres + the render (its
mfma_ready moves the sphere into the matrix-core layout in place) -- against
the same frames with no edit, and with a move that leaves the block's box
every frame (the whole layout rebuilt: what every edit cost through round 5).
Also checks the last edited frame against a fresh context's render of the
same scene (bit-identical). usage: python tools/scene_edit_probe.py [out.json]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bevy_raytrace_amd import abi, scene  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402

W, H, S, D, N = 1920, 1080, 1, 3, 60
cam = default_camera_block()
out = {"frame": f"{W}x{H} {S}spp depth {D}", "frames": N}
for name, sc in (("rtiow_484", scene.rtiow_final_scene()), ("spheres_10000", scene.ten_thousand_scene())):
    sp0, mt = sc.objects_gpu(), sc.materials_gpu()
    res = {}
    for mode in ("no_edit", "small_move", "far_move", "small_move"):
        r = Renderer(0)
        r.set_scene(sp0, mt)
        r.reserve(1, W, H, S, D)
        buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        sp = sp0.copy()
        rng = np.random.default_rng(5)
        upd_ms, t0 = [], None
        for f in range(N + 5):
            if f == 5:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                upd_ms = []
            if mode != "no_edit":
                i = int(rng.integers(1, len(sp) - 4))
                step = 0.01 if mode == "small_move" else 60.0
                sp["center"][i, 0] += np.float32(step if f % 2 == 0 else -step)
                tu = time.perf_counter()
                r.update_spheres(i, sp[i:i + 1])
                upd_ms.append((time.perf_counter() - tu) * 1e3)
            r.render_device(cam, buf.data_ptr(), W, H, S, D, frame0=f)
            r.wait()
        dt = (time.perf_counter() - t0) / N * 1e3
        cnt = (ctypes.c_uint64 * 2)()
        r.lib.rt_debug_mf_rebuilds(r.ctx, cnt)
        fresh = Renderer(0)
        fresh.set_scene(sp, mt)
        ref, _ = fresh.render(cam, W, H, S, D, frame0=N + 4)
        fresh.close()
        exact = bool(np.array_equal(buf.cpu().numpy(), ref, equal_nan=True))
        res[mode] = {"frame_ms": round(dt, 4),
                     "update_call_ms": round(float(np.median(upd_ms)), 4) if upd_ms else 0.0,
                     "layouts_built_whole": int(cnt[0]), "layouts_updated_in_place": int(cnt[1]),
                     "last_frame_equals_fresh_context": exact}
        r.close()
        print(name, mode, res[mode], flush=True)
    out[name] = res
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
