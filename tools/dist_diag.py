"""Diagnostic: config1 row shards (K=2, B=pick_row_block) rendered in 2-frame
launches vs the oracle, frame by frame, and the same through single-frame
renders -- to localise a frame that differs between bench.py N=1 and N=2."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from bevy_raytrace_amd import abi, configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer
from oracle import oracle as O

wl = configs.WORKLOADS["config1"]
sc = wl.make_scene()
sp, mt = sc.objects_gpu(), sc.materials_gpu()
cam = default_camera_block()
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
K = 2
B = configs.pick_row_block(H, K)
r = Renderer(0)
r.set_scene(sp, mt)
NO_REUSE = abi.RT_FLAG_NO_PRIMARY_CACHE


def same(a, b):
    return np.array_equal(a, b, equal_nan=True)


for k in range(K):
    rows = abi.shard_rows(H, B, K, k)
    for F, f0 in ((2, 0), (2, 2), (1, 3)):
        out = torch.full((F, len(rows), W, 4), -1.0, dtype=torch.float32, device="cuda")
        r.render_frames_device(cam, F, out.data_ptr(), W, H, S, D, frame0=f0 * S, row_block=B,
                               shard_count=K, shard_index=k, flags=NO_REUSE)
        st = r.wait()
        got = out.cpu().numpy()
        for i in range(F):
            ref, _ = O.render(cam, sp, mt, W, H, S, D, frame0=(f0 + i) * S, row_block=B,
                              shard_count=K, shard_index=k)
            one, _ = r.render(cam, W, H, S, D, frame0=(f0 + i) * S, row_block=B, shard_count=K,
                              shard_index=k, flags=NO_REUSE)
            bad = np.argwhere(~((got[i] == ref) | (np.isnan(got[i]) & np.isnan(ref))).all(-1))
            print(f"k={k} B={B} F={F} frame {f0 + i}: launch==oracle {same(got[i], ref)} "
                  f"single==oracle {same(one, ref)} bad px {len(bad)} first {bad[:4].tolist()}",
                  flush=True)
