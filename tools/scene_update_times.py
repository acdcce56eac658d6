"""Host cost of a scene edit: the matrix-core layout built
from scratch (spatial order + rows + bounds, what every rt_update_spheres cost
at the next render through round 5) against the in-place update of one moved
sphere (rt_api.cpp mf_update), at 484, 10,000 and 60,000 spheres, through the
host-only entry rt_debug_mf_update (median of 7). CPU only.
usage: python tools/scene_update_times.py [out.json]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bevy_raytrace_amd import abi, scene  # noqa: E402

lib = abi.load()
res = {}
for name, sc in (("rtiow_484", scene.rtiow_final_scene()),
                 ("spheres_10000", scene.ten_thousand_scene()),
                 ("spheres_60000", scene.init_spheres(125, "rtiow", 20221015, max_grid=59996))):
    sp = np.ascontiguousarray(sc.objects_gpu())
    rows = []
    for rep in range(7):
        i = 1 + (rep * 7919) % (len(sp) - 4)
        new = sp[[i]].copy()
        new["center"] += np.float32(0.02)
        idx = np.array([i], np.uint32)
        ms = np.zeros(3)
        rc = lib.rt_debug_mf_update(sp.ctypes.data_as(ctypes.c_void_p), len(sp),
                                    idx.ctypes.data_as(ctypes.c_void_p),
                                    new.ctypes.data_as(ctypes.c_void_p), 1,
                                    ms.ctypes.data_as(ctypes.c_void_p))
        rows.append((rc, ms[2], ms[1]))
    rc = [r[0] for r in rows]
    res[name] = {"spheres": len(sp), "in_place_and_byte_identical": all(r == 1 for r in rc),
                 "full_rebuild_ms": round(float(np.median([r[1] for r in rows])), 3),
                 "in_place_ms": round(float(np.median([r[2] for r in rows])), 4)}
    print(name, res[name], flush=True)
res["note"] = ("host ms (this machine) for one moved sphere: the full rebuild (mf_build: scale, "
               "spatial order, rows, bounds) vs the in-place update (mf_update: one O(N) scale pass, "
               "the moved row, its half-block and chunk bound rows); the device upload of the "
               "touched pieces (1.5 KB A block + 2.5 KB bound chunk(s) + 48 B records) is not "
               "included")
if len(sys.argv) > 1:
    json.dump(res, open(sys.argv[1], "w"), indent=1)
