"""BASELINE.json configs 4 and 5 at their own sizes on one MI355X, against the
oracle.

Config 4 (7680x4320, 1024 spp, depth 16, row-tiled over 8 GPUs): one GPU
renders the shards exactly as one rank of the 8-GPU job does. This is the size
at which the reference's f32 pixel addressing breaks (generate.wgsl:81,
collect.wgsl:109: pixel = u32(y*W + x) in f32 is inexact for y*W >= 2^24, i.e.
y >= 2185 at W = 7680) and the exact integer addressing of
this build replaces it: rows on both sides of that line are compared bit for
bit with the oracle, whose addressing is exact too.

Config 5 (1920x1080, 10,000 spheres, 128 spp, depth 16): the whole frame, the
sphere list streamed through the scalar cache, sampled rows bit-exact; the
segment count is checked exactly on a 4-row shard (oracle-sized) and as the
shard-union identity on the full frame.
"""
import numpy as np
import pytest

from bevy_raytrace_amd import abi
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.configs import WORKLOADS, pick_row_block
from oracle import oracle as O

pytestmark = pytest.mark.gpu

NO_REUSE = abi.RT_FLAG_NO_PRIMARY_CACHE
CULL = abi.RT_FLAG_CULL


def check_exact(img, ref):
    assert img.shape == ref.shape
    if not np.array_equal(img, ref, equal_nan=True):
        bad = ~((img == ref) | (np.isnan(img) & np.isnan(ref)))
        idx = np.argwhere(bad.any(-1))
        raise AssertionError(f"{len(idx)} pixels differ, first {idx[:5].tolist()}")


def _scene(key):
    wl = WORKLOADS[key]
    sc = wl.make_scene()
    return wl, sc.objects_gpu(), sc.materials_gpu()


def _render_shard_device(renderer, cam, W, H, S, D, B, K, k, flags):
    import torch
    rows = abi.shard_rows(H, B, K, k)
    out = torch.empty((1, len(rows), W, 4), dtype=torch.float32, device="cuda")
    renderer.reserve(1, W, H, S, D, row_block=B, shard_count=K, shard_index=k, flags=flags)
    renderer.render_frames_device(cam, 1, out.data_ptr(), W, H, S, D, row_block=B, shard_count=K,
                                  shard_index=k, flags=flags)
    st = renderer.wait()
    return rows, out[0].cpu().numpy(), st


@pytest.mark.parametrize("k", range(8))
def test_config4_8k_shard_of_8(renderer, k):
    """One rank's part of the 8-GPU 8K frame (row blocks of
    pick_row_block(4320, 8) = 1 row, serpentine deal): the shard's first and
    last rows and rows on both sides of y*W = 2^24, bit-exact."""
    wl, sp, mt = _scene("rtiow8k")
    W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
    K = 8
    B = pick_row_block(H, K)
    assert B == 1 and H % (B * K) == 0
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    rows, img, st = _render_shard_device(renderer, cam, W, H, S, D, B, K, k, NO_REUSE)
    assert len(rows) == H // K and st["traced_segments"] == st["segments"]
    below = max(i for i, y in enumerate(rows) if y * W < 1 << 24)
    above = min(i for i, y in enumerate(rows) if y * W >= 1 << 24)
    pick = [0, below, above, len(rows) - 1]
    assert rows[pick[1]] < 2185 <= rows[pick[2]]
    ref, _ = O.render_rows(cam, sp, mt, W, H, S, D, [rows[i] for i in pick])
    check_exact(img[pick], ref)
    assert (img[..., 3] == 1).all()


def test_config4_8k_shard_walks_identical(renderer):
    """Every row of one rank's part of the 8-GPU 8K frame (shard 7 of 8, 540
    rows x 7680, 1024 spp) through the three walks of the sphere list -- the
    matrix-core filter (default), the packed VALU filter and the culled list:
    bit-identical, segment counts equal."""
    wl, sp, mt = _scene("rtiow8k")
    W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
    K, k = 8, 7
    B = pick_row_block(H, K)
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    _, m, sm = _render_shard_device(renderer, cam, W, H, S, D, B, K, k, NO_REUSE)
    _, v, sv = _render_shard_device(renderer, cam, W, H, S, D, B, K, k,
                                    NO_REUSE | abi.RT_FLAG_VALU_FILTER)
    check_exact(v, m)
    _, c, sc = _render_shard_device(renderer, cam, W, H, S, D, B, K, k, NO_REUSE | CULL)
    check_exact(c, m)
    assert sm["segments"] == sv["segments"] == sc["segments"] == sm["traced_segments"]


def test_config4_8k_segments_exact(renderer):
    """Segment count and pixels of a 4-row shard of the 8K frame (row blocks of
    1, K = 1080: rows 546, 1613, 2706, 3773 -- two of them past 2^24 / W)
    against the oracle's count of the same rows (the C-ABI default mode,
    primary-hit reuse allowed: the count is the algorithmic one either way)."""
    wl, sp, mt = _scene("rtiow8k")
    W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
    B, K, k = 1, 1080, 546
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, W, H, S, D, row_block=B, shard_count=K, shard_index=k)
    assert abi.shard_rows(H, B, K, k) == [546, 1613, 2706, 3773]
    ref, segs = O.render(cam, sp, mt, W, H, S, D, row_block=B, shard_count=K, shard_index=k)
    check_exact(img, ref)
    assert st["segments"] == segs
    assert st["traced_segments"] <= segs


def test_config5_10k_full_frame(renderer):
    """The whole 1080p frame with 10,000 spheres (list streamed, not staged):
    sampled rows bit-exact; the packed VALU filter over every sphere
    (RT_FLAG_VALU_FILTER: no block bounds, nothing skipped) and the culled
    list give the same frame and count as the default matrix-core walk with
    its block bounds (20 bound chunks)."""
    wl, sp, mt = _scene("spheres10k1080")
    W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
    assert len(sp) == 10_000 and (W, H, S, D) == (1920, 1080, 128, 16)
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, W, H, S, D, flags=NO_REUSE)
    assert st["traced_segments"] == st["segments"]
    rows = np.linspace(0, H - 1, 12).round().astype(int).tolist()  # 12 rows spread over the frame
    ref, _ = O.render_rows(cam, sp, mt, W, H, S, D, rows)
    check_exact(img[rows], ref)
    culled, sc = renderer.render(cam, W, H, S, D, flags=NO_REUSE | CULL)
    check_exact(culled, img)
    assert sc["segments"] == st["segments"]
    del culled
    valu, sv = renderer.render(cam, W, H, S, D, flags=NO_REUSE | abi.RT_FLAG_VALU_FILTER)
    check_exact(valu, img)
    assert sv["segments"] == st["segments"]


def test_config5_10k_segments_exact(renderer):
    """Segment count exact against the oracle on a 4-row shard (B = 1,
    K = 270), and on the full frame as the union of the 8 shards of the
    8-GPU layout (pick_row_block(1080, 8) = 1)."""
    wl, sp, mt = _scene("spheres10k1080")
    W, H, S, D = wl.width, wl.height, wl.spp, wl.max_depth
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, W, H, S, D, row_block=1, shard_count=270, shard_index=100,
                              flags=NO_REUSE)
    ref, segs = O.render(cam, sp, mt, W, H, S, D, row_block=1, shard_count=270, shard_index=100)
    check_exact(img, ref)
    assert st["segments"] == segs
    _, full = renderer.render(cam, W, H, S, D, flags=NO_REUSE)
    B = pick_row_block(H, 8)
    parts = [renderer.render(cam, W, H, S, D, row_block=B, shard_count=8, shard_index=k,
                             flags=NO_REUSE)[1]["segments"] for k in range(8)]
    assert sum(parts) == full["segments"]
