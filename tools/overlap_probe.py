"""Development probe: per-frame cost when frames are enqueued back-to-back
(no host gap), on one stream vs alternating between two streams (tail of
frame i overlapped with the start of frame i+1)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bevy_raytrace_amd import configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
W, H = 1920, 1080
NF = 8
rs = [Renderer(0) for _ in range(NF)]
for r in rs:
    r.set_scene(sc.objects_gpu(), sc.materials_gpu())
bufs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in range(2)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def batch(S, n, k, rb, nstreams):
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = [torch.cuda.Event(enable_timing=True) for _ in range(nstreams)]
    e0.record(streams[0])
    for s in streams[1:nstreams]:
        s.wait_event(e0)
    for i, r in enumerate(rs):
        st = streams[i % nstreams]
        r.render_device(cam, bufs[i % 2].data_ptr(), W, H, S, 16, row_block=rb, shard_count=n,
                        shard_index=k, flags=1, stream=st.cuda_stream)
    for j in range(nstreams):
        e1[j].record(streams[j])
    for r in rs:
        r.wait()
    torch.cuda.synchronize()
    return max(e0.elapsed_time(e) for e in e1) / NF


def single(S, n, k, rb):
    ts = []
    for r in rs[:3]:
        r.render_device(cam, bufs[0].data_ptr(), W, H, S, 16, row_block=rb, shard_count=n,
                        shard_index=k, flags=1)
        ts.append(r.wait()["kernel_ms"])
    return min(ts)


batch(8, 1, 0, 8, 1)
for (S, n, k, rb) in [(64, 1, 0, 8), (8, 1, 0, 8), (64, 8, 0, 5), (64, 8, 7, 5)]:
    a = single(S, n, k, rb)
    b = batch(S, n, k, rb, 1)
    c = batch(S, n, k, rb, 2)
    print(f"S={S} n={n} k={k}: isolated {a:.3f} ms | back-to-back 1 stream {b:.3f} ms/frame | "
          f"2 streams {c:.3f} ms/frame", flush=True)
