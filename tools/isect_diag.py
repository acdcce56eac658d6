"""Diagnostic: repeat rt_intersect on one adversarial ray set per walk and
report mismatches against the oracle, per repetition, with the wave class
(matrix-core filter vs VALU fallback) of every mismatching ray.
Usage: python tools/isect_diag.py [scene] [reps]"""
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from bevy_raytrace_amd.abi import MATERIAL_DTYPE, RT_FLAG_VALU_FILTER  # noqa: E402
from bevy_raytrace_amd.renderer import Renderer  # noqa: E402
from oracle import oracle as O  # noqa: E402
from raygen import adversarial_rays  # noqa: E402
from test_gpu_intersect import SCENES  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "mixed"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
libs = sys.argv[3:] or [None]
sp, off = SCENES[name]()
mt = np.zeros(int(sp["material"].max()) + 1, dtype=MATERIAL_DTYPE)
n = 400_000 if len(sp) < 1000 else 60_000
rays = adversarial_rays(sp, n, seed=zlib.crc32(name.encode()) % 1000)
if off is not None:
    sp = sp.copy()
    sp["center"] += np.asarray(off, np.float32)
    rays[:, :3] += np.asarray(off, np.float32)
if os.environ.get("FAR_ONLY"):  # only the waves with a ray outside the f16 split's range
    om = np.abs(rays[:, :3]).max(1).reshape(-1, 64)
    rays = rays.reshape(-1, 64, 6)[(om > 4096).any(1)].reshape(-1, 6).copy()
    n = len(rays)
    print("far-only rays", n, flush=True)
ci, ct = O.intersect_batch(sp, rays)
om = np.abs(rays[:, :3]).max(1)
wave_mfma = ~(om.reshape(-1, 64) > 4096).any(1) if n % 64 == 0 else None
burn = None
if os.environ.get("CONCURRENT"):  # fp16 GEMMs (matrix cores) on a side stream during each call
    import torch
    side = torch.cuda.Stream()
    ga = torch.randn(8192, 8192, device="cuda", dtype=torch.float16)
    gb = torch.randn(8192, 8192, device="cuda", dtype=torch.float16)

    def burn():
        with torch.cuda.stream(side):
            for _ in range(40):
                ga @ gb
for lib in libs:
  print("lib", lib, flush=True)
  with Renderer(0, lib_path=lib) as r:
    r.set_scene(sp, mt)
    for fast in (1, 0):
        r.tune(fast_exact=fast)
        for flags, lab in ((0, "brute"), (RT_FLAG_VALU_FILTER, "valu")):
            for k in range(reps):
                if burn is not None:
                    burn()
                gi, gt = r.intersect(rays, flags=flags)
                tag = (gi + (1 << 23)) >> 24  # RT_ISECT_PATHTAG builds: 1 = matrix-core walk
                gi = gi - (tag << 24)
                bad = np.nonzero((gi != ci) | (gt.view(np.uint32) != ct.view(np.uint32)))[0]
                cls = ""
                if bad.size and wave_mfma is not None:
                    wm = wave_mfma[bad // 64]
                    cls = f" mfma-waves {int(wm.sum())} valu-waves {int((~wm).sum())}"
                    cls += f" tagged-mfma {int(tag[bad].sum())}"
                print(f"fast={fast} {lab} rep {k}: {bad.size} differ{cls} first {bad[:8].tolist()}",
                      flush=True)
    r.tune(None)
