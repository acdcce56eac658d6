"""Development probe (combined -DRT_WAVE_TRACE -DRT_PROFILE build,
tools/librt_hip_heavy.so): per wave, iterations, wall time per iteration and
exact sphere tests per iteration -- are the slow waves of a launch slow
because of candidate drains?"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from bevy_raytrace_amd import configs
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_hip_heavy.so")
wl = configs.WORKLOADS["rtiow1080"]
sc = wl.make_scene()
cam = default_camera_block()
r = Renderer(0, lib_path=LIB)
r.lib.rt_debug_wave_trace.restype = ctypes.c_int
r.set_scene(sc.objects_gpu(), sc.materials_gpu())
W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
buf = torch.empty((8, H, W, 4), dtype=torch.float32, device="cuda:0")
F, n, k = 8, 8, 7
rb = configs.pick_row_block(H, n)
for _ in range(2):
    r.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D, row_block=rb, shard_count=n,
                           shard_index=k, flags=1)
    st = r.wait()
out = np.zeros(32768 * 4, dtype=np.uint64)
r.lib.rt_debug_wave_trace(out.ctypes.data_as(ctypes.c_void_p), 32768)
t = out.reshape(-1, 4)[:6144].astype(np.int64)
start, end = t[:, 0], t[:, 1]
span = (end - start) / 100.0
iters = t[:, 3] & 0xFFFF
exact = t[:, 3] >> 32
us_it = span / np.maximum(iters, 1)
ex_it = exact / np.maximum(iters, 1)
order = np.argsort(us_it)
print(f"kernel {st['kernel_ms']:.2f} ms; us/iter median {np.median(us_it):.1f}, p99 {np.percentile(us_it, 99):.1f}")
for name, sel in [("fastest 50%", order[:3072]), ("slowest 5%", order[-307:]), ("slowest 20", order[-20:])]:
    print(f"  {name}: us/iter {us_it[sel].mean():.1f}, exact tests/iter {ex_it[sel].mean():.2f}, "
          f"iters {iters[sel].mean():.0f}, wave ids mean {sel.mean():.0f}")
print("  corr(us/iter, exact/iter) =", np.corrcoef(us_it, ex_it)[0, 1])
# per-SIMD/CU view: waves of one workgroup share a CU
wg = np.arange(6144) // 4
print("  us/iter by workgroup-id decile:", [round(float(us_it[(wg * 10 // 1536) == d].mean()), 1) for d in range(10)])
# where each wave ran: HW_ID (simd [5:4], cu [11:8], sh [12], se [15:13]) + XCC_ID
hw = t[:, 2] & 0xFFFFFFFF
xcc = (t[:, 2] >> 32) & 0xF
simd = (hw >> 4) & 3
cu = (hw >> 8) & 0xF
se = (hw >> 13) & 7
sh = (hw >> 12) & 1
key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
simd_key = key * 4 + simd
print(f"  distinct CUs {len(np.unique(key))}, SIMDs {len(np.unique(simd_key))}, "
      f"waves/SIMD max {np.bincount(simd_key).max()}")
rank = np.zeros(6144, dtype=np.int64)
for kk in np.unique(simd_key):
    idx = np.nonzero(simd_key == kk)[0]
    rank[idx[np.argsort(idx)]] = np.arange(idx.size)   # dispatch order within the SIMD
print("  us/iter by dispatch rank within its SIMD:",
      [round(float(us_it[rank == q].mean()), 1) for q in range(rank.max() + 1)])
print("  us/iter by XCC:", [round(float(us_it[xcc == q].mean()), 1) for q in range(8)])
