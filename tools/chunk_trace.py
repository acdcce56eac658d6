"""Queue progress over time from the -DRT_CHUNK_TRACE diagnostic build
(tools/librt_hip_chunks.so): the time each 64-item slice of the work queue
is taken, so the item rate of every phase of a launch (start, block items,
single-sample tail, drain) can be compared across launch shapes."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from bevy_raytrace_amd import abi, configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_hip_chunks.so")
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=LIB)
r.lib.rt_debug_chunk_trace.restype = ctypes.c_int
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
buf = torch.empty((8, H, W, 4), dtype=torch.float32, device="cuda:0")
N = 1 << 22


def trace(F, n=1, k=0, tail=None):
    if tail:
        r.tune(tail=tail)
    rb = configs.pick_row_block(H, n)
    for _ in range(2):
        out = np.zeros(N, dtype=np.uint64)
        clk = np.zeros(N, dtype=np.uint64)
        r.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                               shard_index=k, flags=abi.RT_FLAG_NO_PRIMARY_CACHE)
        st = r.wait()
    r.lib.rt_debug_chunk_trace(out.ctypes.data_as(ctypes.c_void_p),
                               clk.ctypes.data_as(ctypes.c_void_p), N)
    rows = len(abi.shard_rows(H, rb, n, k))
    npix = rows * W
    nch = st["paths"]  # upper bound on items
    t = out.astype(np.int64)
    t0 = t[0]
    valid = t >= t0
    last = np.nonzero(valid & (t > 0))[0].max()
    t = (t[: last + 1] - t0) / 100.0  # us (100 MHz realtime)
    span = st["kernel_ms"] * 1e3
    print(f"F={F} n={n} tail={tail}: kernel {st['kernel_ms']:.3f} ms, chunks {last + 1}, "
          f"queue dry at {t.max():.0f} us, drain {span - t.max():.0f} us", flush=True)
    # item rate per decile of the queue
    dec = np.array_split(np.arange(last + 1), 10)
    rates = []
    for d in dec:
        dt = t[d[-1]] - t[d[0]]
        rates.append(len(d) * 64 / max(dt, 1e-3))
    print("   items/us per queue decile: " + " ".join(f"{x:.0f}" for x in rates))
    c = clk.astype(np.int64)[: last + 1]
    rt = out.astype(np.int64)[: last + 1]
    ghz = []
    for d in dec:
        a, b = d[0], d[-1]
        ghz.append((c[b] - c[a]) / max(rt[b] - rt[a], 1) * 0.1)
    print("   shader clock GHz per decile (s_memtime / s_memrealtime): " +
          " ".join(f"{x:.2f}" for x in ghz))
    # time to take the first 1% of the queue
    one = max(1, (last + 1) // 100)
    print(f"   first 1% of queue taken by {t[one]:.0f} us; 50% at {t[(last + 1) // 2]:.0f} us")


CASES = [(1, 1, 0), (4, 1, 0), (8, 1, 0), (4, 8, 7), (8, 8, 7), (4, 8, 0), (8, 8, 0)]
if len(sys.argv) > 1:
    CASES = [tuple(int(v) for v in c.split(",")) for c in sys.argv[1:]]
for F, n, k in CASES:
    for rep in range(2):
        trace(F, n, k)
