"""Intersection parity: the GPU's filtered closest-hit loop (rt_intersect ->
intersect_world) against the oracle's brute-force reference loop
(intersect.wgsl:94-143), bit-exact index and t, on adversarial rays aimed at
the filter's decision boundary (tests/raygen.py). Each walk is checked: the
default brute-force walk (the matrix-core filter whenever the scene and the
wave's rays fit its f16 split, else the packed VALU filter), the VALU filter
forced (RT_FLAG_VALU_FILTER) and the culled list (RT_FLAG_CULL)."""
import glob
import os
import zlib

import numpy as np
import pytest

from bevy_raytrace_amd import scene
from bevy_raytrace_amd.abi import RT_FLAG_CULL, RT_FLAG_VALU_FILTER
from oracle import oracle as O
from raygen import adversarial_rays

pytestmark = pytest.mark.gpu


def mixed_scene(zero_radius=True):
    """Huge + tiny + negative-radius spheres, overlapping and nested. With the
    zero-radius sphere the scene is outside the short-math domain (r^2 < 2^-40,
    rt_api.cpp scene_fast_ok) and every exact test takes the IEEE forms."""
    mats = scene.MaterialCache()
    mats.insert("a", scene.RayTraceMaterial((0.5, 0.5, 0.5, 1), scene.Reflectance.Lambertian, 1, 0))
    sp = [scene.Sphere((0, -1000, -1), 1000, 0), scene.Sphere((0, 1, 0), 1, 0),
          scene.Sphere((0, 1, 0), -0.9, 0), scene.Sphere((0.5, 1, 0), 0.5, 0),
          scene.Sphere((3, 0.01, 2), 1e-3, 0), scene.Sphere((-3, 2, 1), 2e-5, 0),
          scene.Sphere((1, 1, 1), 0.0, 0), scene.Sphere((2, 3, -4), 50, 0),
          scene.Sphere((0, 1, 0), 1, 0)]  # duplicate: tie broken by list order
    if not zero_radius:
        sp = [x for x in sp if x.radius != 0.0]
    return scene.Scene(sp, mats, "mixed")


FAR = (1e4, -3e3, 2e4)
EDGE_IN = (2.0 ** 30 - 2048.0, 0.0, 0.0)
EDGE_OUT = (2.0 ** 31, 0.0, 0.0)
SCENES = {  # name -> (spheres, translation applied to spheres and rays)
    "rtiow": lambda: (scene.rtiow_final_scene().objects_gpu(), None),
    "spheres10k": lambda: (scene.ten_thousand_scene().objects_gpu(), None),
    "reference": lambda: (scene.reference_scene().objects_gpu(), None),
    "mixed": lambda: (mixed_scene().objects_gpu(), None),
    "mixed_short_math": lambda: (mixed_scene(zero_radius=False).objects_gpu(), None),
    "far_from_origin": lambda: (scene.rtiow_final_scene().objects_gpu(), FAR),
    # centres just inside / outside the short-math scene domain |c| <= 2^30
    # (rt_api.cpp scene_fast_ok): the same rays either way, fast vs IEEE path
    "edge_of_short_domain": lambda: (scene.rtiow_final_scene().objects_gpu(), EDGE_IN),
    "beyond_short_domain": lambda: (scene.rtiow_final_scene().objects_gpu(), EDGE_OUT),
}


WALKS = {"brute": 0, "brute_valu": RT_FLAG_VALU_FILTER, "cull": RT_FLAG_CULL}


@pytest.mark.parametrize("walk", sorted(WALKS))
@pytest.mark.parametrize("fast", [True, False], ids=["short_math", "ieee"])
@pytest.mark.parametrize("name", sorted(SCENES))
def test_intersect_bit_exact(renderer, name, fast, walk):
    """fast=False forces the IEEE exact tests (knob fast_exact=0): both forms
    must give the oracle's bits."""
    if not fast:
        renderer.tune(fast_exact=0)
    sp, off = SCENES[name]()
    from bevy_raytrace_amd.abi import MATERIAL_DTYPE
    mt = np.zeros(int(sp["material"].max()) + 1, dtype=MATERIAL_DTYPE)
    n = 400_000 if len(sp) < 1000 else 60_000
    rays = adversarial_rays(sp, n, seed=zlib.crc32(name.encode()) % 1000)
    if off is not None:
        sp = sp.copy()
        sp["center"] += np.asarray(off, np.float32)
        rays[:, :3] += np.asarray(off, np.float32)
    renderer.set_scene(sp, mt)
    gi, gt = renderer.intersect(rays, flags=WALKS[walk])
    ci, ct = O.intersect_batch(sp, rays)
    bad = np.nonzero((gi != ci) | (gt.view(np.uint32) != ct.view(np.uint32)))[0]
    assert bad.size == 0, f"{bad.size} rays differ, e.g. {bad[:5].tolist()}: gpu {gi[bad[:5]]} {gt[bad[:5]]} cpu {ci[bad[:5]]} {ct[bad[:5]]}"
    assert (ci >= 0).mean() > 0.05  # the set really hits things


def test_cull_tie_goes_to_lower_index(renderer):
    """Two unit spheres touching at (1, 0, 0); the culled list holds index 1
    first (tests/test_cull.py). Rays through the contact point give both the
    same root: the reference's strict `<` keeps sphere 0, and so must the
    culled walk (original-index tie-break)."""
    from test_cull import tangent_pair
    sp = tangent_pair().objects_gpu()
    from bevy_raytrace_amd.abi import MATERIAL_DTYPE
    mt = np.zeros(1, dtype=MATERIAL_DTYPE)
    rng = np.random.default_rng(5)
    k = 4096
    d = rng.normal(size=(k, 3))
    d[:, 0] = 0.0  # perpendicular to the line of centres: tangent to both
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.array([1.0, 0.0, 0.0]) - d * rng.uniform(1, 20, (k, 1))
    rays = np.hstack([o, d]).astype(np.float32)
    renderer.set_scene(sp, mt)
    ci, ct = O.intersect_batch(sp, rays)
    for flags in WALKS.values():
        gi, gt = renderer.intersect(rays, flags=flags)
        assert np.array_equal(gi, ci) and np.array_equal(gt.view(np.uint32), ct.view(np.uint32))
    # the ties really occur: with the order reversed the oracle picks sphere 1
    ri, rt = O.intersect_batch(sp[::-1].copy(), rays)
    assert ((ci == 0) & (ri == 0)).sum() > 100  # reversed list: index 0 = the old sphere 1


WGSL_ISECT = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                           "wgsl_isect_*.npz")))


@pytest.mark.parametrize("flags", list(WALKS.values()), ids=list(WALKS))
@pytest.mark.parametrize("path", WGSL_ISECT, ids=[os.path.basename(p) for p in WGSL_ISECT])
def test_matches_reference_intersect_world(renderer, path, flags):
    """rt_intersect against intersect.wgsl's own intersect_world (executed by
    tests/golden/wgsl_exec.py) on adversarial rays: t bit for bit, misses,
    and the hit sphere's material."""
    from bevy_raytrace_amd.abi import MATERIAL_DTYPE, SPHERE_DTYPE
    z = np.load(path, allow_pickle=False)
    sp = z["spheres"].view(SPHERE_DTYPE)
    renderer.set_scene(sp, z["materials"].view(MATERIAL_DTYPE))
    idx, t = renderer.intersect(z["rays"], flags=flags)
    assert np.array_equal(t, z["t"], equal_nan=True)
    hit = idx >= 0
    assert np.array_equal(~hit, z["t"] == np.float32(1e20))
    assert np.array_equal(sp["material"][idx[hit]], z["material"][hit])


@pytest.mark.parametrize("fast", [True, False], ids=["short_math", "ieee"])
def test_valu_and_matrix_waves_side_by_side(renderer, fast):
    """Round 2 saw VALU-walk waves miss hits only while other waves of the same
    kernel ran the matrix-core walk. Here every other
    wave of 64 rays holds one ray whose origin is outside the f16 split's range
    (|o| > 2^12: that wave takes the packed VALU filter) and the rest are near
    (the matrix-core filter), so the two walks run side by side on every CU;
    four launches, each bit-exact against the oracle."""
    if not fast:
        renderer.tune(fast_exact=0)
    sp, _ = SCENES["mixed"]()
    from bevy_raytrace_amd.abi import MATERIAL_DTYPE
    mt = np.zeros(int(sp["material"].max()) + 1, dtype=MATERIAL_DTYPE)
    rays = adversarial_rays(sp, 400_000, seed=zlib.crc32(b"side_by_side") % 1000)
    o = rays[:, :3]
    near = (np.abs(o).max(1) <= 100.0)
    far = np.abs(o).max(1) > 2.0 ** 12
    nr, fr = rays[near], rays[far]
    nw = len(nr) // 63
    assert nw > 2000 and len(fr) > 0
    waves = []
    for w in range(nw):
        blk = nr[63 * w:63 * w + 63]
        if w & 1:  # one far ray at a varying lane: a VALU-walk wave
            blk = np.insert(blk, w % 64, fr[w % len(fr)], axis=0)
        else:
            blk = np.vstack([blk, nr[(63 * w + 7) % len(nr)]])
        waves.append(blk)
    rays = np.ascontiguousarray(np.vstack(waves), dtype=np.float32)
    renderer.set_scene(sp, mt)
    ci, ct = O.intersect_batch(sp, rays)
    assert (ci >= 0).mean() > 0.05
    for rep in range(4):
        gi, gt = renderer.intersect(rays)
        bad = np.nonzero((gi != ci) | (gt.view(np.uint32) != ct.view(np.uint32)))[0]
        assert bad.size == 0, f"launch {rep}: {bad.size} rays differ, e.g. {bad[:8].tolist()}"



@pytest.mark.parametrize("n", [65_536, 65_537])
def test_largest_matrix_core_list(renderer, n):
    """The matrix-core walk's queue entries hold a 14-bit group index
    (rt_dev_intersect.h mf_spread): 2^16 spheres is the largest list it takes
    (group indices up to 16,382, both index bytes in use), one more sphere
    goes to the VALU filter (rt_api.cpp build_mfma). Rays aimed at spheres
    spread over the whole list, half of them at the last 4,096."""
    from bevy_raytrace_amd.abi import MATERIAL_DTYPE, SPHERE_DTYPE
    rng = np.random.default_rng(n)
    sp = np.zeros(n, dtype=SPHERE_DTYPE)
    sp["center"] = rng.uniform(-400.0, 400.0, (n, 3)).astype(np.float32)
    sp["radius"] = rng.uniform(0.2, 2.0, n).astype(np.float32)
    mt = np.zeros(1, dtype=MATERIAL_DTYPE)
    k = 8192
    tgt = np.where(rng.random(k) < 0.5, rng.integers(n - 4096, n, k), rng.integers(0, n, k))
    o = rng.uniform(-500.0, 500.0, (k, 3)).astype(np.float32)
    aim = sp["center"][tgt] + rng.normal(0.0, 1.0, (k, 3)) * sp["radius"][tgt, None]
    d = (aim - o).astype(np.float32)
    rays = np.ascontiguousarray(np.hstack([o, d]), dtype=np.float32)
    renderer.set_scene(sp, mt)
    gi, gt = renderer.intersect(rays)
    ci, ct = O.intersect_batch(sp, rays)
    bad = np.nonzero((gi != ci) | (gt.view(np.uint32) != ct.view(np.uint32)))[0]
    assert bad.size == 0, f"{bad.size} rays differ, e.g. {bad[:5].tolist()}"
    assert (ci >= n - 4096).sum() > 600 and (ci >= 0).mean() > 0.5


def _box_scene(n, lo, hi, rmin, rmax, seed):
    from bevy_raytrace_amd.abi import SPHERE_DTYPE
    rng = np.random.default_rng(seed)
    sp = np.zeros(n, dtype=SPHERE_DTYPE)
    sp["center"] = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    sp["radius"] = rng.uniform(rmin, rmax, n).astype(np.float32)
    return sp


COHERENT = {  # name -> (spheres, half-waves of rays)
    # the headline's list: 16 blocks, one bound chunk
    "rtiow": lambda: (scene.rtiow_final_scene().objects_gpu(), 4096),
    # 2,000 spheres at |c| ~ 140..176: sphere rows near the f16 split's
    # range (|S'| <= 2^15, rt_api.cpp build_mfma), 63 blocks, 4 bound chunks
    "cluster_at_range_edge": lambda: (_box_scene(2000, (95, -5, 95), (125, 25, 125), 0.1, 0.8, 11), 2048),
    # 2,000 spheres in a 80-unit box: 4 bound chunks
    "random2k": lambda: (_box_scene(2000, (-40, 0, -40), (40, 20, 40), 0.2, 1.0, 12), 2048),
    # config 5's list: 313 blocks, 20 bound chunks
    "spheres10k": lambda: (scene.ten_thousand_scene().objects_gpu(), 1024),
}


@pytest.mark.parametrize("name", sorted(COHERENT))
def test_block_bounds_at_their_decision_boundary(renderer, name):
    """Block-bound culling on the GPU where it decides (rt_dev_intersect.h
    "Block bounds" / "Forward bounds"): every 32-ray half-wave is coherent and
    aimed at ONE 16-sphere half-block -- rays tangent to the member whose far
    side sets the bound's radius (so their lines pass at the bound's own
    radius), the same ray replicated 32 times, fans from one origin grazing a
    member at r (1 +- 1e-8..1e-4), and origins at |o|^2 just below 2^15, the
    largest the matrix-core walk takes (tests/raygen.py coherent_halves).
    Such halves skip most blocks: the walk must skip > 30 % of the tiles a
    walk without bounds visits (rt_debug_intersect_tiles) while index and t
    stay bit-exact against the oracle; the same rays through every block
    (knob mf_cull=0) and through the unculled packed VALU filter
    (RT_FLAG_VALU_FILTER) give the same bits."""
    from bevy_raytrace_amd import abi
    from bevy_raytrace_amd.abi import MATERIAL_DTYPE
    from raygen import coherent_halves
    sp, halves = COHERENT[name]()
    perm = abi.cull_layout(sp)[0]
    rays = coherent_halves(sp, perm, halves, seed=zlib.crc32(name.encode()) % 1000)
    mt = np.zeros(int(sp["material"].max()) + 1, dtype=MATERIAL_DTYPE)
    renderer.set_scene(sp, mt)
    ci, ct = O.intersect_batch(sp, rays)
    assert (ci >= 0).mean() > 0.2

    def exact(gi, gt, what):
        bad = np.nonzero((gi != ci) | (gt.view(np.uint32) != ct.view(np.uint32)))[0]
        assert bad.size == 0, (f"{what}: {bad.size} rays differ, e.g. {bad[:5].tolist()}: gpu "
                               f"{gi[bad[:5]]} {gt[bad[:5]]} cpu {ci[bad[:5]]} {ct[bad[:5]]}")

    gi, gt = renderer.intersect(rays)
    walked, total = renderer.intersect_tiles()
    exact(gi, gt, "block-bound walk")
    # every wave took the matrix-core walk (|o|^2 <= 2^15, |c| in range): 2
    # halves x nblk 32 x 32 tiles each without bounds (8 nblk 16 x 16 tiles
    # in an RT_MF16 build) -- and skipped
    nblk = (int(np.nonzero(perm >= 0)[0].max()) + 1 + 31) // 32
    waves = -(-len(rays) // 64)
    assert total in (2 * nblk * waves, 8 * nblk * waves), (total, nblk)
    assert walked <= 0.7 * total, (walked, total)
    # the chunk-level bounds (lists of 2..32 bound chunks) only remove tiles
    renderer.tune(mf_top=0)
    ni, nt = renderer.intersect(rays)
    w_nt, t_nt = renderer.intersect_tiles()
    exact(ni, nt, "block bounds without chunk bounds (mf_top=0)")
    assert t_nt == total and w_nt >= walked
    renderer.tune(None)
    renderer.tune(mf_cull=0)
    ai, at = renderer.intersect(rays)
    w_all, t_all = renderer.intersect_tiles()
    exact(ai, at, "every block (mf_cull=0)")
    assert w_all == t_all == total
    renderer.tune(None)
    vi, vt = renderer.intersect(rays, flags=RT_FLAG_VALU_FILTER)
    exact(vi, vt, "unculled VALU filter")
    assert renderer.intersect_tiles() == (0, 0)
