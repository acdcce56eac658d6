"""Predicted strong scaling from one GPU: time every row shard of the headline
frame for N = 2, 4, 8 on one device and compare the slowest shard with the
full frame (development tool; the real N-GPU run is the driver's).

speedup_pred(N) = T_full / max_k T_shard(N, k)   (render kernel only; the
RCCL gather of W*H*16/N bytes per rank and the device re-assembly are
measured separately by bench.py at N>1).
"""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from bevy_raytrace_amd import configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

wl = configs.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else configs.HEADLINE]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
flags = 1  # headline: no primary reuse
buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")


def run(n, k, rb, reps=3):
    ts = []
    for _ in range(reps):
        r.render_device(cam, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                        shard_index=k, flags=flags)
        ts.append(r.wait()["kernel_ms"])
    return min(ts)


run(1, 0, 8, 2)
full = run(1, 0, 8)
out = {"workload": wl.key, "full_ms": full, "shards": {}}
print(f"full frame: {full:.3f} ms", flush=True)
for n in (2, 4, 8):
    rb = configs.pick_row_block(H, n)
    ts = [run(n, k, rb) for k in range(n)]
    pred = full / max(ts)
    out["shards"][n] = {"row_block": rb, "shard_ms": ts, "pred_speedup": pred,
                        "imbalance": max(ts) / (sum(ts) / n)}
    print(f"N={n} rb={rb}: shard ms {['%.3f' % t for t in ts]} max {max(ts):.3f} "
          f"pred speedup {pred:.2f}x imbalance {max(ts) / (sum(ts) / n):.3f}", flush=True)
print(json.dumps(out))
