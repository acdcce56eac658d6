"""Development probe: item order (RT_CHUNK_MAJOR) x tail split (RT_TAIL_SPLIT)
x primary reuse. For each setting: full-frame kernel time, the slowest of
the N=8 row shards (predicted 8-GPU speedup), and bit-identity of the image
with the first setting (the order never changes results)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bevy_raytrace_amd import configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

wl = configs.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0)
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
buf = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")


def run(flags, n=1, k=0, rb=8, reps=3):
    ts, tt = [], []
    for _ in range(reps):
        r.render_device(cam, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                        shard_index=k, flags=flags)
        st = r.wait()
        ts.append(st["kernel_ms"])
        tt.append(st["total_ms"])
    return min(ts), min(tt)


SETTINGS = [tuple(a.split(",")) for a in (sys.argv[2:] or ["0,1,0", "0,1,1", "1,1,0", "1,1,1"])]
ref = {}
for flags in (1, 0):
    for cm, sp, pf in SETTINGS:
        os.environ["RT_CHUNK_MAJOR"] = cm
        os.environ["RT_TAIL_SPLIT"] = sp
        os.environ["RT_PREFETCH"] = pf
        run(flags, reps=1)
        full, tot = run(flags)
        img = buf.clone()
        same = ref.setdefault(flags, img).equal(img) if flags in ref else True
        ref.setdefault(flags, img)
        same = bool(torch.equal(torch.nan_to_num(ref[flags], 7.0), torch.nan_to_num(img, 7.0)))
        rb = configs.pick_row_block(H, 8)
        sh = [run(flags, 8, kk, rb)[1] for kk in range(8)]
        print(f"flags={flags} chunk_major={cm} split={sp} prefetch={pf}: full kernel {full:.3f} total {tot:.3f} ms | "
              f"N=8 shard total max {max(sh):.3f} mean {sum(sh) / 8:.3f} -> pred {tot / max(sh):.2f}x | "
              f"identical={same}", flush=True)
