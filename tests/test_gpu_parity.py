"""GPU parity: librt_hip.so (the HIP kernel) against the CPU oracle.

The bar is bit-exact: identical f32 images (NaN masks included) and identical
algorithmic segment counts, on the same seeded inputs. At full BASELINE sizes
the oracle checks sampled rows, plus size-independent properties
(determinism, reuse on/off identity, multi-pass identity, shard assembly).
"""
import ctypes
import glob
import os

import numpy as np
import pytest

from bevy_raytrace_amd import abi, scene
from bevy_raytrace_amd.camera import Transform, camera_block, default_camera_block
from oracle import oracle as O

pytestmark = pytest.mark.gpu

NO_REUSE = abi.RT_FLAG_NO_PRIMARY_CACHE
CULL = abi.RT_FLAG_CULL
VALU = abi.RT_FLAG_VALU_FILTER  # the packed-fp32 filter instead of the matrix-core one


def arrays(sc):
    return sc.objects_gpu(), sc.materials_gpu()


def check_exact(img, ref):
    assert img.shape == ref.shape
    same = np.array_equal(img, ref, equal_nan=True)
    if not same:
        bad = ~((img == ref) | (np.isnan(img) & np.isnan(ref)))
        idx = np.argwhere(bad.any(-1))
        raise AssertionError(f"{len(idx)} pixels differ, first {idx[:5].tolist()}")


def glass_scene():
    mats = scene.MaterialCache()
    mats.insert("ground", scene.RayTraceMaterial((0.5, 0.5, 0.5, 1), scene.Reflectance.Lambertian, 1.0, 0))
    mats.insert("glass", scene.RayTraceMaterial((1, 1, 1, 1), scene.Reflectance.Dielectric, 0.0, 1.5))
    mats.insert("diamond", scene.RayTraceMaterial((1, 1, 1, 1), scene.Reflectance.Dielectric, 0.0, 2.4))
    mats.insert("fuzz", scene.RayTraceMaterial((0.9, 0.8, 0.7, 1), scene.Reflectance.Metallic, 0.5, 0))
    sp = [scene.Sphere((0, -1000, -1), 1000, 0), scene.Sphere((0, 1, 0), 1, 1),
          scene.Sphere((0, 1, 0), -0.9, 1), scene.Sphere((-4, 1, 0), 1, 2),
          scene.Sphere((4, 1, 0), 1, 3), scene.Sphere((2, 0.5, 2), 0.5, 2)]
    return scene.Scene(sp, mats, "glass")


CASES = [
    # name, scene, W, H, spp, depth, frame0
    ("config1_full", scene.config1_scene, 400, 225, 16, 8, 0),   # BASELINE configs[0]
    ("reference_sched", scene.reference_scene, 320, 180, 1, 3, 11),  # the reference's own schedule
    ("rtiow", scene.rtiow_final_scene, 192, 108, 12, 16, 0),
    ("glass", glass_scene, 160, 90, 9, 12, 3),
    ("ragged", scene.rtiow_final_scene, 67, 33, 5, 7, 2),
    ("one_pixel", scene.config1_scene, 1, 1, 17, 8, 0),
    ("depth1", scene.rtiow_final_scene, 64, 36, 3, 1, 0),
    ("spheres10k", scene.ten_thousand_scene, 96, 54, 2, 8, 0),
]


WGSL = sorted(p for p in glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                "golden", "wgsl_*.npz"))
              if not os.path.basename(p).startswith("wgsl_isect_"))  # frames only


WGSL_ACCUM = [p for p in WGSL if "_accum" in os.path.basename(p)]


@pytest.mark.parametrize("flags", [0, NO_REUSE, CULL, VALU], ids=["reuse", "noreuse", "cull", "valu"])
@pytest.mark.parametrize("path", WGSL, ids=[os.path.basename(p) for p in WGSL])
def test_matches_interpreted_reference_wgsl(renderer, path, flags):
    """The HIP path against frames of the reference's own WGSL kernels,
    executed by tests/golden/wgsl_exec.py (spp 1; depth 3, or 16 for the
    *_d16 fixtures whose bounce kill is generalised), bit for bit."""
    z = np.load(path, allow_pickle=False)
    sp = z["spheres"].view(abi.SPHERE_DTYPE)
    mt = z["materials"].view(abi.MATERIAL_DTYPE)
    cam = z["camera"].view(abi.CAMERA_DTYPE).reshape(())
    W, H, S, D = (int(v) for v in z["params"])
    renderer.set_scene(sp, mt)
    n = int(z["processed"][0])  # pixels the reference's floor-divided grid traces (D1)
    for f, ref in zip(z["frames"], z["images"]):
        img, _ = renderer.render(cam, W, H, S, D, frame0=int(f), flags=flags)
        check_exact(img.reshape(-1, 4)[:n], ref.reshape(-1, 4)[:n])


@pytest.mark.parametrize("flags", [0, NO_REUSE, CULL, VALU], ids=["reuse", "noreuse", "cull", "valu"])
@pytest.mark.parametrize("path", WGSL_ACCUM, ids=[os.path.basename(p) for p in WGSL_ACCUM])
def test_spp_is_blocked_sum_of_reference_frames(renderer, path, flags):
    """One S-spp render == the blocked f32 sum of the reference's S
    one-sample frames (executed from its WGSL) / S, bit for bit."""
    from test_oracle import blocked_mean
    z = np.load(path, allow_pickle=False)
    sp = z["spheres"].view(abi.SPHERE_DTYPE)
    mt = z["materials"].view(abi.MATERIAL_DTYPE)
    cam = z["camera"].view(abi.CAMERA_DTYPE).reshape(())
    W, H, _, D = (int(v) for v in z["params"])
    frames = [int(f) for f in z["frames"]]
    renderer.set_scene(sp, mt)
    img, _ = renderer.render(cam, W, H, len(frames), D, frame0=frames[0], flags=flags)
    check_exact(img, blocked_mean(list(z["images"])))


@pytest.mark.parametrize("flags", [0, NO_REUSE, CULL, CULL | NO_REUSE, VALU, VALU | NO_REUSE],
                         ids=["reuse", "noreuse", "cull", "cull_noreuse", "valu", "valu_noreuse"])
@pytest.mark.parametrize("name,mk,W,H,S,D,f0", CASES, ids=[c[0] for c in CASES])
def test_bit_exact(renderer, name, mk, W, H, S, D, f0, flags):
    sp, mt = arrays(mk())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, W, H, S, D, frame0=f0, flags=flags)
    ref, segs = O.render(cam, sp, mt, W, H, S, D, frame0=f0)
    check_exact(img, ref)
    assert st["segments"] == segs
    if flags & NO_REUSE:
        assert st["traced_segments"] == segs
    else:
        assert st["traced_segments"] <= segs
    assert (img[..., 3] == 1).all()


def test_empty_scene(renderer):
    from bevy_raytrace_amd.abi import MATERIAL_DTYPE, SPHERE_DTYPE
    sp, mt = np.zeros(0, SPHERE_DTYPE), np.zeros(0, MATERIAL_DTYPE)
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, 33, 17, 3, 4)
    ref, segs = O.render(cam, sp, mt, 33, 17, 3, 4)
    check_exact(img, ref)
    assert st["segments"] == segs == 33 * 17 * 3


def test_other_camera(renderer):
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = camera_block(Transform.from_xyz(-6.0, 3.0, 9.0).looking_at((1.0, 0.5, -1.0)))
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, 120, 80, 6, 10)
    ref, segs = O.render(cam, sp, mt, 120, 80, 6, 10)
    check_exact(img, ref)
    assert st["segments"] == segs


@pytest.mark.parametrize("flags", [0, NO_REUSE], ids=["reuse", "noreuse"])
def test_far_camera_alternates_walks(renderer, flags):
    """The RTIOW scene seen from 400x the default camera distance (|o| ~ 5,500
    > 2^12, the f16 split's range): a wave holding a primary ray walks the
    sphere list with the packed VALU filter, a wave of bounce rays (near the
    scene) with the matrix-core filter, so waves switch walks from one
    iteration to the next (with primary-hit reuse on, most iterations are
    bounces). Bit-exact against the oracle; the oracle confirms both kinds of
    segments occur in quantity."""
    sp, mt = arrays(scene.rtiow_final_scene())
    eye = np.array([13.0, 2.0, 3.0]) * 400.0
    cam = camera_block(Transform.from_xyz(*eye).looking_at((0.0, 0.5, 0.0)), fov=0.0055)
    W, H, S, D = 96, 54, 16, 8
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, W, H, S, D, flags=flags)
    ref, segs = O.render(cam, sp, mt, W, H, S, D)
    check_exact(img, ref)
    assert st["segments"] == segs
    # primary segments (far origin) = W*H*S; the rest are bounces near the
    # scene (the view is filled: most primaries hit and bounce)
    assert 1.5 * W * H * S < segs < 8 * W * H * S


def test_render_async_into_registered_host_buffers(renderer):
    """The Bevy shim's per-frame path: rt_render_async into page-locked host
    buffers (rt_host_register), two frames alternating, bit-exact against the
    oracle; registering twice or unregistering an unknown buffer is refused."""
    sp, mt = arrays(scene.reference_scene())
    cam = default_camera_block()
    W, H, S, D = 96, 54, 1, 3
    renderer.set_scene(sp, mt)
    bufs = [np.empty((H, W, 4), np.float32) for _ in range(2)]
    for b in bufs:
        renderer.host_register(b)
    with pytest.raises(abi.RayTraceError):
        renderer.host_register(bufs[0])
    with pytest.raises(abi.RayTraceError):
        renderer.host_unregister(np.empty(16, np.float32))
    for f in range(4):
        renderer.render_async(cam, bufs[f & 1], W, H, S, D, frame0=f)
        st = renderer.wait()
        ref, segs = O.render(cam, sp, mt, W, H, S, D, frame0=f)
        check_exact(bufs[f & 1], ref)
        assert st["segments"] == segs
    for b in bufs:
        renderer.host_unregister(b)


def test_multi_pass_scratch_identical(renderer):
    """Block sums folded over several passes == one pass (sequential fold)."""
    sp, mt = arrays(scene.config1_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    one, st1 = renderer.render(cam, 80, 45, 40, 6)
    # 16 slots: a small image splits every block into single samples (8 slots
    # per block), so 2 blocks per pass
    renderer.tune(scratch_bytes=80 * 45 * 16 * 16)
    many, st2 = renderer.render(cam, 80, 45, 40, 6)
    assert st2["kernel_launches"] == 3 and st1["kernel_launches"] == 1
    check_exact(many, one)
    ref, segs = O.render(cam, sp, mt, 80, 45, 40, 6)
    check_exact(one, ref)


@pytest.mark.parametrize("wide", ["0", "64"], ids=["never_wide", "always_wide"])
@pytest.mark.parametrize("name,mk", [("rtiow", scene.rtiow_final_scene), ("glass", glass_scene),
                                     ("empty", None)])
def test_sphere_parallel_tail(renderer, wide, name, mk):
    """intersect_wide (the nearly-empty-wave path) and the ray-parallel walk
    give the same image: forced on for every wave, and forced off."""
    from bevy_raytrace_amd.abi import MATERIAL_DTYPE, SPHERE_DTYPE
    sp, mt = arrays(mk()) if mk else (np.zeros(0, SPHERE_DTYPE), np.zeros(0, MATERIAL_DTYPE))
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    renderer.tune(wide_max=wide)
    img, st = renderer.render(cam, 80, 45, 9, 12, frame0=1, flags=NO_REUSE)
    ref, segs = O.render(cam, sp, mt, 80, 45, 9, 12, frame0=1)
    check_exact(img, ref)
    assert st["segments"] == segs


@pytest.mark.parametrize("S", [1, 6, 8, 21, 64])
def test_tail_split_identical(renderer, S):
    """The single-sample tail items (last block of a pass, summed in sample
    order by the collect kernel) give the same image as whole-block items."""
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    on, st_on = renderer.render(cam, 72, 40, S, 10, frame0=5, flags=NO_REUSE)
    renderer.tune(tail_split=0)
    off, st_off = renderer.render(cam, 72, 40, S, 10, frame0=5, flags=NO_REUSE)
    check_exact(on, off)
    assert st_on["segments"] == st_off["segments"]
    renderer.tune(scratch_bytes=72 * 40 * 16 * 8, tail_split=1)  # 1 (split) block per pass
    passes, _ = renderer.render(cam, 72, 40, S, 10, frame0=5)
    check_exact(passes, on)
    ref, segs = O.render(cam, sp, mt, 72, 40, S, 10, frame0=5)
    check_exact(on, ref)
    assert st_on["segments"] == segs


@pytest.mark.parametrize("S,region,tail", [(21, "1000000", "0,0,6"), (64, "1000000", "0,1,1"),
                                           (64, "96", "0.01,0.01,0.01"), (64, "0", "0,1,1")])
def test_item_order_identical(renderer, S, region, tail):
    """Pixel-major items (knob item_order bits: one pixel's pairs / tail
    sample groups, and its frames, back to back in the queue), and grouped
    items (bit 2: 8 pixels' items back to back, frame / pair / sample-group
    major) give the frames of the pair- / sample- / frame-major order -- only
    the work order changes, each item keeps its slot. Three frames in one
    launch, so the regions span frames; the 0.01 tail holds 4-, 2- and
    1-sample items; 72 x 40 = 360 groups of 8 pixels."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    W, H, F = 72, 40, 3
    renderer.set_scene(sp, mt)
    renderer.tune(block_region=region, tail=tail)
    outs = []
    for order in ("0", "1", "2", "3", "4", "7", "7/4"):  # 7/4: groups of 4 pixels
        o, _, g = order.partition("/")
        renderer.tune(item_order=o, pix_group=g or "8")
        buf = torch.empty((F, H, W, 4), dtype=torch.float32, device="cuda")
        renderer.render_frames_device(cam, F, buf.data_ptr(), W, H, S, 10, flags=NO_REUSE)
        st = renderer.wait()
        outs.append((buf.cpu().numpy(), st["segments"]))
    for o in outs[1:]:
        check_exact(o[0], outs[0][0])
        assert o[1] == outs[0][1]
    ref, segs = O.render(cam, sp, mt, W, H, S, 10, frame0=S)  # launch frame 1 = samples S..2S
    check_exact(outs[1][0][1], ref)


def test_schedule_knobs_identical(renderer):
    """The launch-shape rules chosen by the call (round 5: the block region
    by spp / depth and aligned to a frame boundary, the s_setprio rotation by
    samples per lane, lead items -- block_lead, with and without a partial
    pixel-region frame and with several launches per call; the regions made
    to exist at this size by a short tail) and their
    knob overrides change only which lane runs which item and when: the
    frames and segment counts are those of every other setting, and the
    oracle's."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    W, H, F, S = 72, 40, 3, 64
    renderer.set_scene(sp, mt)
    outs = []
    # At this size the default tail covers the whole launch (every pair a tail
    # sample); with a short tail (T) the main part's regions exist, and the
    # block region picks them (tests/test_plan_model.py: 0.3 -> pixel
    # frames 0-1, a lead item in frame 2; 0.55 unaligned -> frame 0 partial,
    # lead items in frames 1-2)
    T = "0,0,0.01"
    for knobs in ({}, {"prio_mode": "0"}, {"prio_mode": "1"}, {"prio_mode": "3"},
                  {"block_region": "128"}, {"block_region": "16", "prio_mode": "0"},
                  {"block_align": "0"}, {"tail": T}, {"tail": T, "block_region": "128"},
                  {"tail": T, "block_region": "0.3"}, {"tail": T, "block_region": "0.3", "prio_mode": "0"},
                  {"tail": T, "block_region": "0.3", "block_lead": "0"},
                  {"tail": T, "block_region": "0.3", "block_lead": "4"},
                  {"tail": T, "block_region": "0.55", "block_align": "0"},
                  {"tail": T, "block_region": "0.55", "block_align": "0", "block_lead": "3"},
                  {"tail": T, "block_lead": "2", "scratch_bytes": str(W * H * 16 * 6)},
                  {"tail": T, "block_region": "0.3", "scratch_bytes": str(W * H * 16 * 12)},
                  {"wave_chunk": "16"}, {"tail": T, "block_region": "0.3", "wave_chunk": "128"}):
        renderer.tune(None)
        if knobs:
            renderer.tune(**knobs)
        buf = torch.empty((F, H, W, 4), dtype=torch.float32, device="cuda")
        renderer.render_frames_device(cam, F, buf.data_ptr(), W, H, S, 10, flags=NO_REUSE)
        st = renderer.wait()
        outs.append((buf.cpu().numpy(), st["segments"]))
    renderer.tune(None)
    for o in outs[1:]:
        check_exact(o[0], outs[0][0])
        assert o[1] == outs[0][1]
    ref, segs = O.render(cam, sp, mt, W, H, S, 10, frame0=2 * S)
    check_exact(outs[0][0][2], ref)


@pytest.mark.parametrize("K,B", [(3, 5), (8, 1)])
def test_image_out_shards_fill_one_image(renderer, K, B):
    """RT_FLAG_IMAGE_OUT: K row shards of a 2-frame launch write their rows
    at their image rows of ONE buffer (what every rank does through rank 0's
    IPC-mapped image, bench.py) -- together the full render; rows a shard
    does not own are left untouched."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    W, H, S, D, F = 96, 61, 8, 8, 2
    renderer.set_scene(sp, mt)
    full = torch.empty((F, H, W, 4), dtype=torch.float32, device="cuda")
    renderer.render_frames_device(cam, F, full.data_ptr(), W, H, S, D, flags=NO_REUSE)
    renderer.wait()
    img = torch.full((F, H, W, 4), -7.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()  # the fill (torch's stream) done before the library's stream writes
    for k in range(K):
        renderer.render_frames_device(cam, F, img.data_ptr(), W, H, S, D, row_block=B,
                                      shard_count=K, shard_index=k,
                                      flags=NO_REUSE | abi.RT_FLAG_IMAGE_OUT)
        renderer.wait()
        if k == 0:  # only shard 0's rows written so far
            got = img.cpu().numpy()
            rows = abi.shard_rows(H, B, K, 0)
            others = np.setdiff1d(np.arange(H), rows)
            assert (got[:, others] == -7.0).all()
            check_exact(got[:, rows], full.cpu().numpy()[:, rows])
    renderer.acquire()  # the owner's system-scope acquire (rt_acquire), as rank 0 does
    check_exact(img.cpu().numpy(), full.cpu().numpy())


def test_image_out_refused_for_host_output(renderer):
    sp, mt = arrays(scene.config1_scene())
    renderer.set_scene(sp, mt)
    with pytest.raises(Exception, match="IMAGE_OUT"):
        renderer.render(default_camera_block(), 32, 18, 4, 4, flags=abi.RT_FLAG_IMAGE_OUT)


@pytest.mark.parametrize("K,B", [(2, 8), (3, 5), (8, 1)])
def test_shards_and_device_assembly(renderer, K, B):
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    W, H, S, D = 96, 61, 4, 8
    renderer.set_scene(sp, mt)
    full, stf = renderer.render(cam, W, H, S, D)
    rows = [len(abi.shard_rows(H, B, K, k)) for k in range(K)]
    mr = max(rows)
    g = torch.zeros((K, mr, W, 4), dtype=torch.float32, device="cuda")
    segs = 0
    for k in range(K):
        part, st = renderer.render(cam, W, H, S, D, row_block=B, shard_count=K, shard_index=k)
        g[k, :rows[k]] = torch.from_numpy(part).cuda()
        segs += st["segments"]
        # device-output path writes the same shard
        buf = torch.empty((rows[k], W, 4), dtype=torch.float32, device="cuda")
        renderer.render_device(cam, buf.data_ptr(), W, H, S, D, 0, B, K, k)
        renderer.wait()
        assert torch.equal(buf.cpu(), torch.from_numpy(part)) or np.array_equal(
            buf.cpu().numpy(), part, equal_nan=True)
    img = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    # the library runs on its own stream: torch's writes of g must be done
    torch.cuda.synchronize()
    renderer.assemble_shards(g.data_ptr(), mr, img.data_ptr(), W, H, B, K)
    torch.cuda.synchronize()
    check_exact(img.cpu().numpy(), full)
    assert segs == stf["segments"]


@pytest.mark.parametrize("K,B,H", [(3, 2, 23), (8, 5, 1080), (1, 8, 17)])
def test_assemble_shard_frames_matches_per_frame(renderer, K, B, H):
    """rt_assemble_shard_frames (one launch over the (shard, frame) slabs one
    gather of multi-frame launches lands) equals rt_assemble_shards frame by
    frame, and the numpy statement of the mapping (distributed.assemble_host)."""
    import torch
    from bevy_raytrace_amd.distributed import ShardLayout, assemble_host
    W, F = 40, 3
    mr = max(len(abi.shard_rows(H, B, K, k)) for k in range(K))
    g = torch.randn((K, F, mr, W, 4), dtype=torch.float32, device="cuda")
    img = torch.full((F, H, W, 4), -7.0, dtype=torch.float32, device="cuda")
    # the library runs on its own stream (no stream argument): torch's writes
    # of its inputs must be complete first (the bench passes its stream)
    torch.cuda.synchronize()
    renderer.assemble_shard_frames(g.data_ptr(), mr, F, img.data_ptr(), W, H, B, K)
    lay = ShardLayout(H, B, K)
    for f in range(F):
        slabs = g[:, f].contiguous()
        one = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        renderer.assemble_shards(slabs.data_ptr(), mr, one.data_ptr(), W, H, B, K)
        torch.cuda.synchronize()
        assert torch.equal(img[f], one)
        assert np.array_equal(img[f].cpu().numpy(), assemble_host(slabs.cpu().numpy(), lay))
    with pytest.raises(abi.RayTraceError):
        renderer.assemble_shard_frames(g.data_ptr(), mr, 0, img.data_ptr(), W, H, B, K)
    if K > 1:
        with pytest.raises(abi.RayTraceError):  # slabs shorter than a shard
            renderer.assemble_shard_frames(g.data_ptr(), mr - 1, F, img.data_ptr(), W, H, B, K)


def test_full_1080p64_properties(renderer):
    """Headline config at full size: sampled-row parity (incl. NaN-path rows),
    determinism, reuse on/off identity."""
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    a, sa = renderer.render(cam, 1920, 1080, 64, 16)
    b, sb = renderer.render(cam, 1920, 1080, 64, 16, flags=NO_REUSE)
    assert sa["segments"] == sb["segments"] == sb["traced_segments"]
    check_exact(a, b)
    c, _ = renderer.render(cam, 1920, 1080, 64, 16)
    check_exact(a, c)
    # 64 rows spread over the frame plus the rows of the NaN paths below
    rows = sorted(set(np.linspace(0, 1079, 64).round().astype(int).tolist()) |
                  {1, 415, 540, 544, 558, 777})
    ref, _ = O.render_rows(cam, sp, mt, 1920, 1080, 64, 16, rows)
    check_exact(a[rows], ref)
    nan_px = np.isnan(a[..., 0])
    assert nan_px[415, 481] and nan_px[544, 866] and nan_px[558, 881]
    assert nan_px.sum() < 200


def test_full_1080p64_lead_items(renderer):
    """Lead items by the call at full size: a 3-frame 1080p/64 launch has a
    pixel region (frame 0) and two frames past it (block region 64 x depth
    samples per lane, rt_api.cpp regions: fp = 1, each later frame's first 2
    blocks one item). Frames and segment counts identical to the plan
    without lead items (block_lead=0) and sampled rows of the lead frames
    bit-exact against the oracle."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    W, H, S, D, F = 1920, 1080, 64, 16, 3
    outs = []
    for knobs in ({}, {"block_lead": "0"}):
        renderer.tune(None)
        if knobs:
            renderer.tune(**knobs)
        buf = torch.empty((F, H, W, 4), dtype=torch.float32, device="cuda")
        renderer.render_frames_device(cam, F, buf.data_ptr(), W, H, S, D)
        st = renderer.wait()
        torch.cuda.synchronize()
        outs.append((buf.cpu().numpy(), st["segments"]))
        del buf
    renderer.tune(None)
    check_exact(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]
    rows = [0, 415, 540, 1079]
    for f in (1, 2):
        ref, _ = O.render_rows(cam, sp, mt, W, H, S, D, rows, frame0=f * S)
        check_exact(outs[0][0][f][rows], ref)


def test_4k_sampled_rows(renderer):
    """BASELINE config 3 (4K, 256 spp, depth 32): 64 rows spread over the
    frame bit-exact against the oracle."""
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, 3840, 2160, 256, 32)
    rows = np.linspace(3, 2157, 64).round().astype(int).tolist()  # 64 rows spread over the frame
    ref, _ = O.render_rows(cam, sp, mt, 3840, 2160, 256, 32, rows)
    check_exact(img[rows], ref)


def test_4k_full_frame_walks_identical(renderer):
    """BASELINE config 3, one whole frame through the three walks of the
    sphere list: the matrix-core filter (default), the packed VALU filter
    (RT_FLAG_VALU_FILTER) and the culled list (RT_FLAG_CULL) -- every pixel
    bit-identical and the segment counts equal, so no filter margin fails
    anywhere in the frame (intersect.wgsl:133-143 is the one answer)."""
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    m, sm = renderer.render(cam, 3840, 2160, 256, 32, flags=NO_REUSE)
    v, sv = renderer.render(cam, 3840, 2160, 256, 32, flags=NO_REUSE | VALU)
    check_exact(v, m)
    del v
    c, sc = renderer.render(cam, 3840, 2160, 256, 32, flags=NO_REUSE | CULL)
    check_exact(c, m)
    assert sm["segments"] == sv["segments"] == sc["segments"] == sm["traced_segments"]


def test_errors(renderer):
    sp, mt = arrays(scene.config1_scene())
    bad = sp.copy()
    bad[2]["material"] = 17
    with pytest.raises(abi.RayTraceError) as e:
        renderer.set_scene(bad, mt)
    assert e.value.status == abi.RT_ERR_BAD_SCENE
    badm = mt.copy()
    badm[1]["reflectance"] = 5
    with pytest.raises(abi.RayTraceError) as e:
        renderer.set_scene(sp, badm)
    assert e.value.status == abi.RT_ERR_BAD_SCENE
    renderer.set_scene(sp, mt)
    cam = default_camera_block()
    for args in [(0, 4, 1, 1), (4, 4, 0, 1), (4, 4, 1, 0)]:
        with pytest.raises(abi.RayTraceError) as e:
            renderer.render(cam, *args)
        assert e.value.status == abi.RT_ERR_INVALID_ARG
    with pytest.raises(abi.RayTraceError):
        renderer.render(cam, 8, 8, 1, 1, shard_count=2, shard_index=2)


def test_frames_in_flight(renderer):
    """RT_MAX_PENDING frames enqueued back to back (each slot on its own
    stream) give the same images and stats as one-at-a-time renders; a third
    enqueue and a synchronous call while frames are pending are refused."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    W, H, S, D = 96, 54, 10, 9
    refs = [renderer.render(cam, W, H, S, D, frame0=f0, flags=NO_REUSE) for f0 in (0, 10)]
    bufs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(2)]
    for rep in range(2):
        for b, f0 in zip(bufs, (0, 10)):
            renderer.render_device(cam, b.data_ptr(), W, H, S, D, frame0=f0, flags=NO_REUSE)
        if rep == 0:
            with pytest.raises(abi.RayTraceError) as e:
                renderer.render_device(cam, bufs[0].data_ptr(), W, H, S, D)
            assert e.value.status == abi.RT_ERR_INVALID_ARG
            with pytest.raises(abi.RayTraceError):
                renderer.render(cam, W, H, S, D)
        stats = [renderer.wait(), renderer.wait()]
        for b, st, (ref, rst) in zip(bufs, stats, refs):
            check_exact(b.cpu().numpy(), ref)
            assert st["segments"] == rst["segments"]
    with pytest.raises(abi.RayTraceError):
        renderer.wait()


def test_render_before_scene():
    from bevy_raytrace_amd.renderer import Renderer
    with Renderer(0) as r:
        with pytest.raises(abi.RayTraceError) as e:
            r.render(default_camera_block(), 8, 8, 1, 1)
        assert e.value.status == abi.RT_ERR_NO_SCENE


def test_native_library_is_in_tree():
    """The product path runs librt_hip.so from the package directory."""
    lib = abi.load()
    assert os.path.dirname(lib._name) == abi.PKG_DIR


def test_plugin_frames_match_oracle():
    """RayTracePlugin/RayTraceNode mirror: the reference's own schedule
    (spp 1, depth 3, frame counter advancing) on a small target."""
    from bevy_raytrace_amd.camera import RayTraceCamera
    from bevy_raytrace_amd.plugin import (FrameCounter, RayTraceOutputImage, RayTracePlugin,
                                          RayTraceSettings, World)
    world = World()
    world.insert_resource(RayTraceCamera(160, 90))
    sc = scene.reference_scene()
    node = RayTracePlugin(RayTraceSettings(), sc).build(world)
    sp, mt = arrays(sc)
    for f in range(3):
        RayTracePlugin.frame(world, node)
        img = world.resource(RayTraceOutputImage).data
        ref, segs = O.render(RayTraceCamera(160, 90).to_gpu(), sp, mt, 160, 90, 1, 3, frame0=f)
        check_exact(img, ref)
        assert node.last_stats["segments"] == segs
    assert world.resource(FrameCounter).frame == 3


def test_update_spheres_and_materials(renderer):
    """rt_update_spheres / rt_update_materials == a full rt_set_scene of the edited scene."""
    sc = scene.rtiow_final_scene()
    sp, mt = arrays(sc)
    renderer.set_scene(sp, mt)
    sp2, mt2 = sp.copy(), mt.copy()
    sp2["center"][10:27] += np.float32(0.3)          # spans three 8-sphere groups
    sp2["radius"][12] = np.float32(0.35)
    sp2["material"][20] = 2                           # now the glass centre sphere's material
    sp2["center"][-1] = (3.5, 1.2, -0.4)              # last group (padding neighbours)
    mt2[5]["color"] = (0.9, 0.1, 0.1, 1.0)
    mt2[7]["reflectance"] = 1
    mt2[7]["fuzziness"] = np.float32(0.25)
    renderer.update_spheres(10, sp2[10:27])
    renderer.update_spheres(len(sp) - 1, sp2[-1:])
    renderer.update_materials(5, mt2[5:8])
    cam = default_camera_block()
    img, st = renderer.render(cam, 128, 72, 4, 8)
    ref, segs = O.render(cam, sp2, mt2, 128, 72, 4, 8)
    check_exact(img, ref)
    assert st["segments"] == segs
    rays = np.array([[13, 2, 3, -1, -0.15, -0.2]], np.float32)
    gi, gt = renderer.intersect(rays)
    ci, ct = O.intersect_batch(sp2, rays)
    assert gi[0] == ci[0] and gt[0] == ct[0]


def mf_rebuilds(renderer):
    out = (ctypes.c_uint64 * 2)()
    assert renderer.lib.rt_debug_mf_rebuilds(renderer.ctx, out) == 0
    return int(out[0]), int(out[1])


@pytest.mark.parametrize("sc_name", ["rtiow", "tenk"])
def test_update_spheres_in_place(renderer, sc_name):
    """Small moves (and a material change) go into the matrix-core layout in
    place (rt_api.cpp mf_update: the moved rows, their half-block and chunk
    bound rows, their records and shading records; no new order), and the
    frames after each edit equal the oracle's of the edited scene -- the
    10,000-sphere list with its chunk-level bounds included. A move that
    leaves the block's box takes the whole rebuild, also exact."""
    sc = scene.rtiow_final_scene() if sc_name == "rtiow" else scene.ten_thousand_scene()
    sp, mt = arrays(sc)
    renderer.set_scene(sp, mt)
    cam = default_camera_block()
    W, H, S, D = (96, 54, 2, 6)
    b0, i0 = mf_rebuilds(renderer)
    rng = np.random.default_rng(11)
    sp2 = sp.copy()
    for step in range(3):
        idx = np.sort(rng.choice(np.arange(len(sp) - 3), 12, replace=False))
        d = rng.uniform(-0.04, 0.04, (12, 3)).astype(np.float32)
        sp2["center"][idx] += d
        sp2["material"][idx[0]] = sp2["material"][idx[-1]]
        for i in idx:
            renderer.update_spheres(int(i), sp2[i:i + 1])
        img, st = renderer.render(cam, W, H, S, D, frame0=step)
        rows = None if sc_name == "rtiow" else list(range(0, H, 9))
        if rows is None:
            ref, segs = O.render(cam, sp2, mt, W, H, S, D, frame0=step)
            check_exact(img, ref)
            assert st["segments"] == segs
        else:
            ref, _ = O.render_rows(cam, sp2, mt, W, H, S, D, rows, frame0=step)
            check_exact(img[rows], ref)
    b1, i1 = mf_rebuilds(renderer)
    assert (b1 - b0, i1 - i0) == (0, 3)  # every edit in place
    sp2["center"][5] += np.float32(40.0)  # far from its block: a new order
    renderer.update_spheres(5, sp2[5:6])
    img, st = renderer.render(cam, W, H, S, D, frame0=7)
    assert mf_rebuilds(renderer)[0] == b1 + 1
    if sc_name == "rtiow":
        ref, segs = O.render(cam, sp2, mt, W, H, S, D, frame0=7)
        check_exact(img, ref)


def test_update_errors(renderer):
    sp, mt = arrays(scene.config1_scene())
    renderer.set_scene(sp, mt)
    with pytest.raises(abi.RayTraceError) as e:
        renderer.update_spheres(3, sp[:2])            # runs past the 4 spheres
    assert e.value.status == abi.RT_ERR_INVALID_ARG
    bad = sp[:1].copy()
    bad["material"] = 9
    with pytest.raises(abi.RayTraceError) as e:
        renderer.update_spheres(0, bad)
    assert e.value.status == abi.RT_ERR_BAD_SCENE
    badm = mt[:1].copy()
    badm["reflectance"] = 3
    with pytest.raises(abi.RayTraceError) as e:
        renderer.update_materials(0, badm)
    assert e.value.status == abi.RT_ERR_BAD_SCENE


def test_plugin_dirty_tracking_animates():
    """Moving one sphere per frame re-uploads that sphere only; frames stay exact."""
    from bevy_raytrace_amd.camera import RayTraceCamera
    from bevy_raytrace_amd.plugin import RayTraceOutputImage, RayTracePlugin, RayTraceSettings, World
    world = World()
    world.insert_resource(RayTraceCamera(96, 54))
    sc = scene.reference_scene()
    world.insert_resource(sc)
    node = RayTracePlugin(RayTraceSettings(samples_per_ray=2, max_depth=4)).build(world)
    for f in range(3):
        sc.spheres[-2].center = (-4.0, 1.0 + 0.25 * f, 0.0)
        RayTracePlugin.frame(world, node)
        sp, mt = arrays(sc)
        ref, segs = O.render(RayTraceCamera(96, 54).to_gpu(), sp, mt, 96, 54, 2, 4, frame0=2 * f)
        check_exact(world.resource(RayTraceOutputImage).data, ref)
    assert node.uploads == {"full": 1, "spheres": 2, "materials": 0}


def test_progressive_accumulation(renderer):
    """Running sum across calls: sum = (s1 + s2) + s3 of the calls' block sums,
    image = sum / total (oracle raw sums folded the same way)."""
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    W, H, D = 80, 45, 8
    acc = None
    f0 = 0
    for k, spp in enumerate([8, 3, 16]):
        img, total = renderer.render_progressive(cam, W, H, spp, D, frame0=f0, reset=(k == 0))
        part, _ = O.render(cam, sp, mt, W, H, spp, D, frame0=f0, raw_sums=True)
        acc = part[..., :3] if acc is None else acc + part[..., :3]
        f0 += spp
        assert total == f0
        exp = np.ones_like(img)
        exp[..., :3] = acc / np.float32(total)
        check_exact(img, exp)
    # reset restarts; a different geometry restarts too
    img, total = renderer.render_progressive(cam, W, H, 4, D, frame0=0, reset=True)
    assert total == 4
    ref, _ = O.render(cam, sp, mt, W, H, 4, D)
    check_exact(img, ref)
    img, total = renderer.render_progressive(cam, W + 1, H, 2, D, frame0=0)
    assert total == 2


def test_srgb8_encode(renderer):
    import torch
    x = np.random.default_rng(3).uniform(-0.2, 1.3, (1000, 4)).astype(np.float32)
    x[:5, 0] = [np.nan, np.inf, -np.inf, 0.0031308, 1.0]
    d_in = torch.from_numpy(x).cuda()
    d_out = torch.empty((1000, 4), dtype=torch.uint8, device="cuda")
    renderer.encode_srgb8(d_in.data_ptr(), d_out.data_ptr(), 1000)
    got = d_out.cpu().numpy().astype(np.int32)
    c = np.nan_to_num(np.clip(x[:, :3].astype(np.float64), 0, 1), nan=0.0)
    c[np.isnan(x[:, :3])] = 0
    s = np.where(c <= 0.0031308, 12.92 * c, 1.055 * c ** (1 / 2.4) - 0.055)
    exp = np.rint(s * 255).astype(np.int32)
    assert np.abs(got[:, :3] - exp).max() <= 1
    assert (got[:, 3] == 255).all()
    assert got[0, 0] == 0 and got[1, 0] == 255 and got[2, 0] == 0


@pytest.mark.parametrize("flags", [0, NO_REUSE], ids=["reuse", "noreuse"])
@pytest.mark.parametrize("K,k,scratch", [(1, 0, None), (3, 2, None), (1, 0, "frame"),
                                         (1, 0, "pass")], ids=["one_launch", "shard",
                                                                "launch_per_frame", "multi_pass"])
def test_frames_batch_identical(renderer, flags, K, k, scratch):
    """rt_render_frames_device: frame i of one launch == rt_render with
    frame0 + i*spp (bit-identical, same total segments), also when the scratch
    limit splits the frames over launches or a frame over passes."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    W, H, S, D, F, f0 = 88, 50, 20, 10, 3, 7
    B = 4
    rows = len(abi.shard_rows(H, B, K, k))
    refs = [renderer.render(cam, W, H, S, D, frame0=f0 + i * S, row_block=B, shard_count=K,
                            shard_index=k, flags=flags) for i in range(F)]
    if scratch == "frame":   # room for one frame's slots per launch
        renderer.tune(scratch_bytes=rows * W * 16 * 3 * 8)
    elif scratch == "pass":  # less than one frame: several passes per frame
        renderer.tune(scratch_bytes=rows * W * 16 * 9)
    out = torch.full((F, rows, W, 4), -1.0, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()  # the fill (torch's stream) done before the library's stream writes
    renderer.render_frames_device(cam, F, out.data_ptr(), W, H, S, D, frame0=f0, row_block=B,
                                  shard_count=K, shard_index=k, flags=flags)
    st = renderer.wait()
    got = out.cpu().numpy()
    for i in range(F):
        check_exact(got[i], refs[i][0])
    assert st["segments"] == sum(r[1]["segments"] for r in refs)
    if scratch is None:
        assert st["kernel_launches"] == 1
    else:
        assert st["kernel_launches"] >= F
    if k == 0 and K == 1:
        ref, segs = O.render(cam, sp, mt, W, H, S, D, frame0=f0 + 2 * S)
        check_exact(got[2], ref)
        assert refs[2][1]["segments"] == segs


def test_frames_batch_errors(renderer):
    import torch
    sp, mt = arrays(scene.config1_scene())
    renderer.set_scene(sp, mt)
    cam = default_camera_block()
    buf = torch.empty((2, 8, 8, 4), dtype=torch.float32, device="cuda")
    with pytest.raises(abi.RayTraceError) as e:
        renderer.render_frames_device(cam, 0, buf.data_ptr(), 8, 8, 1, 1)
    assert e.value.status == abi.RT_ERR_INVALID_ARG
    with pytest.raises(abi.RayTraceError):
        renderer.render_frames_device(cam, 2, 0, 8, 8, 1, 1)


def test_reserve_then_render(renderer):
    """rt_reserve allocates a launch's buffers up front; renders of that size
    (and smaller) then match the oracle; reserve with a call pending fails."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    renderer.set_scene(sp, mt)
    cam = default_camera_block()
    W, H, S, D = 48, 27, 9, 6
    renderer.reserve(3, W, H, S, D)
    buf = torch.empty((3, H, W, 4), dtype=torch.float32, device="cuda")
    renderer.render_frames_device(cam, 3, buf.data_ptr(), W, H, S, D, flags=NO_REUSE)
    with pytest.raises(abi.RayTraceError) as e:
        renderer.reserve(3, W, H, S, D)
    assert e.value.status == abi.RT_ERR_INVALID_ARG
    renderer.wait()
    for i in range(3):
        ref, _ = O.render(cam, sp, mt, W, H, S, D, frame0=i * S)
        check_exact(buf[i].cpu().numpy(), ref)
    img, _ = renderer.render(cam, W, H, 2, D)  # smaller than reserved
    check_exact(img, O.render(cam, sp, mt, W, H, 2, D)[0])
    with pytest.raises(abi.RayTraceError):
        renderer.reserve(1, 0, H, S, D)


@pytest.mark.parametrize("flags", [abi.RT_FLAG_JITTER, abi.RT_FLAG_THIN_LENS,
                                   abi.RT_FLAG_JITTER | abi.RT_FLAG_THIN_LENS,
                                   abi.RT_FLAG_JITTER | abi.RT_FLAG_THIN_LENS | NO_REUSE],
                         ids=["jitter", "thin_lens", "both", "both_noreuse"])
@pytest.mark.parametrize("name,mk", [("rtiow", scene.rtiow_final_scene), ("glass", glass_scene)])
def test_camera_sampling_bit_exact(renderer, flags, name, mk):
    """Opt-in sub-pixel jitter / thin-lens sampling: the
    kernel's per-sample primary rays == the oracle's, bit for bit; the
    primary-hit reuse switches itself off (every segment traced)."""
    sp, mt = arrays(mk())
    cam = camera_block(Transform.from_xyz(13.0, 2.0, 3.0).looking_at((0.0, 0.0, 0.0)),
                       lens_focal_length=0.05, fstop=8.0)
    renderer.set_scene(sp, mt)
    W, H, S, D, f0 = 72, 40, 10, 10, 4
    img, st = renderer.render(cam, W, H, S, D, frame0=f0, flags=flags)
    ref, segs = O.render(cam, sp, mt, W, H, S, D, frame0=f0, flags=flags & ~NO_REUSE)
    check_exact(img, ref)
    assert st["segments"] == segs == st["traced_segments"]
    base, _ = renderer.render(cam, W, H, S, D, frame0=f0)
    assert not np.array_equal(img, base, equal_nan=True)


def test_camera_sampling_frames_and_shards(renderer):
    """Thin lens + jitter through the multi-frame launch and a row shard."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    fl = abi.RT_FLAG_JITTER | abi.RT_FLAG_THIN_LENS
    W, H, S, D, F, K, k, B = 64, 36, 9, 8, 2, 3, 1, 4
    rows = len(abi.shard_rows(H, B, K, k))
    out = torch.empty((F, rows, W, 4), dtype=torch.float32, device="cuda")
    renderer.render_frames_device(cam, F, out.data_ptr(), W, H, S, D, frame0=3, row_block=B,
                                  shard_count=K, shard_index=k, flags=fl)
    renderer.wait()
    got = out.cpu().numpy()
    for i in range(F):
        ref, _ = O.render(cam, sp, mt, W, H, S, D, frame0=3 + i * S, row_block=B, shard_count=K,
                          shard_index=k, flags=fl)
        check_exact(got[i], ref)


@pytest.mark.parametrize("name,mk", [("rtiow", scene.rtiow_final_scene), ("glass", glass_scene)])
def test_short_math_and_ieee_identical(renderer, name, mk):
    """The exact sphere test's short correctly-rounded sqrt/divide (in-domain
    scenes) and the IEEE forms (knob fast_exact=0) render the oracle's bits; a
    zero-radius sphere takes the scene out of the short domain."""
    sp, mt = arrays(mk())
    cam = default_camera_block()
    ref, segs = O.render(cam, sp, mt, 128, 72, 6, 10)
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, 128, 72, 6, 10)
    check_exact(img, ref)
    assert st["segments"] == segs and st["short_math"] == 1
    renderer.tune(fast_exact=0)
    img, st = renderer.render(cam, 128, 72, 6, 10)
    check_exact(img, ref)
    assert st["short_math"] == 0
    renderer.tune(fast_exact=1)
    sp0 = np.concatenate([sp, sp[:1]])
    sp0["radius"][-1] = 0.0
    sp0["center"][-1] = (0.0, 30.0, 0.0)  # out of view; only the domain check changes
    renderer.set_scene(sp0, mt)
    img, st = renderer.render(cam, 128, 72, 6, 10)
    ref0, _ = O.render(cam, sp0, mt, 128, 72, 6, 10)
    check_exact(img, ref0)
    assert st["short_math"] == 0


def stacked_scene():
    """200 coincident spheres (every ray through them has 200 candidates: the
    per-lane queue flushes every 8 groups, and equal roots are broken by list
    order) around a glass and a metal sphere, over the ground."""
    mats = scene.MaterialCache()
    mats.insert("ground", scene.RayTraceMaterial((0.5, 0.5, 0.5, 1), scene.Reflectance.Lambertian, 1.0, 0))
    mats.insert("a", scene.RayTraceMaterial((0.9, 0.2, 0.2, 1), scene.Reflectance.Lambertian, 1.0, 0))
    mats.insert("b", scene.RayTraceMaterial((0.2, 0.9, 0.2, 1), scene.Reflectance.Metallic, 0.2, 0))
    mats.insert("glass", scene.RayTraceMaterial((1, 1, 1, 1), scene.Reflectance.Dielectric, 0.0, 1.5))
    sp = [scene.Sphere((0, -1000, -1), 1000, 0)]
    sp += [scene.Sphere((0, 1, 0), 1, 1 + (i % 2)) for i in range(200)]  # ties: first wins
    sp += [scene.Sphere((-2.2, 1, 0.5), 1, 3), scene.Sphere((2.2, 1, -0.5), 1, 2)]
    return scene.Scene(sp, mats, "stacked")


@pytest.mark.parametrize("flags", [0, NO_REUSE, CULL | NO_REUSE], ids=["reuse", "noreuse", "cull"])
def test_coincident_spheres_queue_flushes(renderer, flags):
    sp, mt = arrays(stacked_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    img, st = renderer.render(cam, 96, 54, 5, 10, frame0=2, flags=flags)
    ref, segs = O.render(cam, sp, mt, 96, 54, 5, 10, frame0=2)
    check_exact(img, ref)
    assert st["segments"] == segs


def test_cull_full_1080p64_identical(renderer):
    """The headline frame through three walks, bit for bit with equal segment
    counts: the default matrix-core walk with block bounds, the packed VALU
    filter over EVERY sphere (RT_FLAG_VALU_FILTER: no bounds, no skipping --
    the unculled reference for the other two) and the culled list
    (RT_FLAG_CULL). (Speeds are bench.py's, not a test's: a shared or
    throttled box says nothing there.)"""
    from bevy_raytrace_amd.abi import RT_FLAG_VALU_FILTER
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    b, sb = renderer.render(cam, 1920, 1080, 64, 16, flags=NO_REUSE)
    v, sv = renderer.render(cam, 1920, 1080, 64, 16, flags=NO_REUSE | RT_FLAG_VALU_FILTER)
    check_exact(b, v)
    c, sc = renderer.render(cam, 1920, 1080, 64, 16, flags=NO_REUSE | CULL)
    check_exact(c, v)
    assert sc["segments"] == sb["segments"] == sv["segments"] == sc["traced_segments"]


@pytest.mark.parametrize("K,k", [(3, 1), (8, 7)])
def test_cull_shards_and_updates(renderer, K, k):
    """Culled list with row shards, and rebuilt after rt_update_spheres."""
    sc_ = scene.rtiow_final_scene()
    sp, mt = arrays(sc_)
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    W, H, S, D = 120, 64, 6, 10
    a, _ = renderer.render(cam, W, H, S, D, row_block=4, shard_count=K, shard_index=k,
                           flags=NO_REUSE)
    c, _ = renderer.render(cam, W, H, S, D, row_block=4, shard_count=K, shard_index=k,
                           flags=NO_REUSE | CULL)
    check_exact(c, a)
    moved = sp[10:30].copy()
    moved["center"][:, 1] += 1.5  # lift 20 spheres: their groups' bounds must follow
    renderer.update_spheres(10, moved)
    sp2 = sp.copy()
    sp2[10:30] = moved
    img, st = renderer.render(cam, 64, 36, 4, 8, flags=CULL)
    ref, segs = O.render(cam, sp2, mt, 64, 36, 4, 8)
    check_exact(img, ref)
    assert st["segments"] == segs


@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_CULL], ids=["brute", "cull"])
def test_reserved_renders_allocate_nothing(renderer, flags):
    """After rt_reserve, rt_render (host output, both in-flight slots) and
    rt_render_frames_device of the reserved size make no device allocation --
    with RT_FLAG_CULL too (rt_reserve builds the culled list), and after a
    sphere update (the lists are rebuilt in place)."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    renderer.set_scene(sp, mt)
    cam = default_camera_block()
    W, H, S, D = 64, 40, 9, 6
    renderer.reserve(2, W, H, S, D, flags=flags)
    before = renderer.alloc_count()
    for f0 in (0, 9, 18):  # rt_render alternates the two slots
        img, _ = renderer.render(cam, W, H, S, D, frame0=f0, flags=flags)
    buf = torch.empty((2, H, W, 4), dtype=torch.float32, device="cuda")
    renderer.render_frames_device(cam, 2, buf.data_ptr(), W, H, S, D, flags=flags)
    renderer.wait()
    assert renderer.alloc_count() == before
    check_exact(img, O.render(cam, sp, mt, W, H, S, D, frame0=18)[0])
    moved = sp[5:7].copy()
    moved["center"] += np.float32(0.25)
    renderer.update_spheres(5, moved)
    img, _ = renderer.render(cam, W, H, S, D, frame0=18, flags=flags)
    assert renderer.alloc_count() == before
    sp2 = sp.copy()
    sp2[5:7] = moved
    check_exact(img, O.render(cam, sp2, mt, W, H, S, D, frame0=18)[0])


def test_failed_scene_upload_leaves_no_scene():
    """A device allocation failing inside rt_set_scene (injected) returns
    RT_ERR_OUT_OF_MEMORY and leaves NO scene -- the next render is refused
    with RT_ERR_NO_SCENE instead of reading freed or half-written buffers; a
    later rt_set_scene recovers. A culled-list build failure is retried."""
    from bevy_raytrace_amd.renderer import Renderer
    small, smt = arrays(scene.config1_scene())
    big, bmt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    with Renderer(0) as r:
        r.set_scene(small, smt)
        r.render(cam, 16, 9, 1, 2)
        r.tune(fail_alloc_after=1)  # the list grows: the 2nd reallocation fails
        with pytest.raises(abi.RayTraceError) as e:
            r.set_scene(big, bmt)
        assert e.value.status == abi.RT_ERR_OUT_OF_MEMORY
        r.tune(None)
        with pytest.raises(abi.RayTraceError) as e:
            r.render(cam, 16, 9, 1, 2)
        assert e.value.status == abi.RT_ERR_NO_SCENE
        r.set_scene(big, bmt)
        for _ in range(2):  # both in-flight slots get their work buffers
            plain, _ = r.render(cam, 32, 18, 2, 4)
        r.tune(fail_alloc_after=0)  # the culled list is built at the first culled call
        with pytest.raises(abi.RayTraceError) as e:
            r.render(cam, 32, 18, 2, 4, flags=CULL)
        assert e.value.status == abi.RT_ERR_OUT_OF_MEMORY
        again, _ = r.render(cam, 32, 18, 2, 4)  # the brute-force list is untouched
        check_exact(again, plain)
        r.tune(None)
        img, _ = r.render(cam, 32, 18, 2, 4, flags=CULL)
        check_exact(img, O.render(cam, big, bmt, 32, 18, 2, 4)[0])


@pytest.mark.parametrize("site", [4, 5, 7, 16])
def test_checked_build_reports_an_out_of_range_index(renderer, site):
    """Positive control of the bounds-checked build (librt_hip_checked.so,
    `--rt-lib`): with one site's bound given as 0 (knob chk_shrink) the render
    fails with RT_ERR_DEVICE naming that site -- so a clean suite under it
    means every checked index stayed in range. The product library checks
    nothing: the same call succeeds, bit-exact."""
    sp, mt = arrays(scene.rtiow_final_scene())
    renderer.set_scene(sp, mt)
    cam = default_camera_block()
    ref, _ = renderer.render(cam, 32, 18, 4, 4)
    renderer.tune("chk_shrink", str(site))
    if hasattr(renderer.lib, "rt_check_bounds_take"):
        with pytest.raises(Exception, match=f"first at site {site}:"):
            renderer.render(cam, 32, 18, 4, 4)
        renderer.tune(None)
        img, _ = renderer.render(cam, 32, 18, 4, 4)  # the record was reset
    else:
        img, _ = renderer.render(cam, 32, 18, 4, 4)
    check_exact(img, ref)


@pytest.mark.parametrize("S,F,flags", [(1, 3, NO_REUSE), (1, 2, 0), (8, 2, NO_REUSE), (21, 3, NO_REUSE),
                                       (64, 5, NO_REUSE), (64, 3, 0), (16, 4, NO_REUSE | CULL)],
                         ids=["spp1", "spp1_reuse", "spp8", "spp21", "spp64", "spp64_reuse",
                              "spp16_cull"])
def test_direct_output_identical(renderer, S, F, flags):
    """Whole items (a pixel item covering its frame's blocks, a block item of a
    one-block frame, a spp-1 tail sample) write their output pixel themselves
    (KParams::dout: fold / spp, rt_collect_kernel's arithmetic) and their
    frames skip the slots and the collect; every frame is bit-identical to the
    all-collect plan (knob direct_out=0), at several frame / sample mixes so
    that direct and collected frames share launches."""
    import torch
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    W, H, D = 96, 54, 8
    outs = []
    for direct in (0, 1):
        renderer.tune("direct_out", str(direct))
        out = torch.full((F, H, W, 4), -3.0, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()  # the fill (torch's stream) done before the library's stream writes
        renderer.render_frames_device(cam, F, out.data_ptr(), W, H, S, D, frame0=7, flags=flags)
        st = renderer.wait()
        outs.append((out.cpu().numpy(), st["segments"]))
    renderer.tune(None)
    check_exact(outs[1][0], outs[0][0])
    assert outs[1][1] == outs[0][1]
    ref, _ = O.render(cam, sp, mt, W, H, S, D, frame0=7 + (F - 1) * S)
    check_exact(outs[1][0][F - 1], ref)


@pytest.mark.parametrize("S", [1, 64])
def test_registered_host_output_two_in_flight(renderer, S):
    """rt_render_async into registered host buffers with two renders in
    flight (the Bevy shim's sequence): every frame bit-identical to a
    synchronous render into a pageable buffer."""
    sp, mt = arrays(scene.rtiow_final_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    W, H, D = 160, 90, 6
    reg = [np.full((H, W, 4), -5.0, np.float32) for _ in range(2)]
    for b in reg:
        renderer.host_register(b)
    try:
        got = []
        for f in range(4):
            if f >= 2:
                renderer.wait()
                got.append(reg[f % 2].copy())
            renderer.render_async(cam, reg[f % 2], W, H, S, D, frame0=f * S)
        for f in (2, 3):
            renderer.wait()
            got.append(reg[f % 2].copy())
    finally:
        for b in reg:
            renderer.host_unregister(b)
    for f in range(4):
        ref, _ = renderer.render(cam, W, H, S, D, frame0=f * S)  # pageable: staged + copied
        check_exact(got[f], ref)


@pytest.mark.parametrize("which", ["rtiow", "reference", "spheres2k"])
def test_block_culled_walk_identical(renderer, which):
    """The matrix-core walk skips, per half-wave, the 32-sphere blocks whose
    bounding sphere no ray of the half passes near (MfScene::B; proof in
    rt_dev_intersect.h "Block bounds"). Frames and segment counts are
    bit-identical with every block walked (knob mf_cull=0) and equal the
    oracle's; spheres2k has 63 blocks, two chunks of bound tiles."""
    import torch
    if which == "spheres2k":
        sc = scene.ten_thousand_scene()
        sp, mt = arrays(sc)
        sp = np.ascontiguousarray(sp[:2000])
    else:
        sp, mt = arrays(scene.rtiow_final_scene() if which == "rtiow" else scene.reference_scene())
    cam = default_camera_block()
    renderer.set_scene(sp, mt)
    W, H, S, D, F = 64, 36, 8, 8, 2
    outs = []
    for cull in (0, 1):
        renderer.tune("mf_cull", str(cull))
        out = torch.full((F, H, W, 4), -3.0, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()  # the fill (torch's stream) done before the library's stream writes
        renderer.render_frames_device(cam, F, out.data_ptr(), W, H, S, D, frame0=3, flags=NO_REUSE)
        st = renderer.wait()
        outs.append((out.cpu().numpy(), st["segments"]))
    renderer.tune(None)
    check_exact(outs[1][0], outs[0][0])
    assert outs[1][1] == outs[0][1]
    ref, segs = O.render(cam, sp, mt, W, H, S, D, frame0=3 + (F - 1) * S)
    check_exact(outs[1][0][F - 1], ref)
