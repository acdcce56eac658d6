"""Oracle pinning (CPU): known-answer values, C vs numpy restatements, golden fixtures.

The reference ships no tests or golden data and its WGSL has no runtime here
(SURVEY.md §8c). The oracle is pinned by (1) the reference's own six compute
shaders executed by a WGSL interpreter (tests/golden/wgsl_exec.py, fixtures
tests/golden/wgsl_*.npz made by tests/golden/make_wgsl_golden.py in the build
container) -- bit-exact per frame at the reference's depth 3, spp 1; the
builtins the WGSL spec leaves to the driver (normalize, length, pow, tan) take
the oracle's documented op forms in both; (2) the hand-derived values of
SURVEY Appendix C; (3) two independent restatements agreeing bit for bit.
"""
import glob
import os

import numpy as np
import pytest

from bevy_raytrace_amd import scene
from bevy_raytrace_amd.abi import MATERIAL_DTYPE, SPHERE_DTYPE
from bevy_raytrace_amd.camera import Transform, camera_block, default_camera_block
from oracle import oracle as O
from oracle import rt_oracle_np as N

F = np.float32
HERE = os.path.dirname(os.path.abspath(__file__))


def camf(cam):
    return np.frombuffer(cam.tobytes(), np.float32)


# ------------------------------------------------------------ Appendix C KATs
HASH_KAT = {  # shade.wgsl:105-116
    0: (0.77879172563552856, 0.15285363793373108, 0.056309748440980911),
    1: (0.15154574811458588, 0.029333777725696564, 0.26464989781379700),
    2: (0.27796033024787903, 0.67902785539627075, 0.42240458726882935),
    12345: (0.91660130023956299, 0.31799834966659546, 0.26120650768280029),
    2073600: (0.61315089464187622, 0.22740712761878967, 0.40775686502456665),
}


@pytest.mark.parametrize("n", sorted(HASH_KAT))
def test_hash3_kat(n):
    exp = np.array(HASH_KAT[n], dtype=np.float32)
    assert np.array_equal(O.hash3(n), exp)
    assert np.array_equal(N.hash3(np.array([n], np.uint32))[0], exp)


def test_hash3_never_zero():
    # n is always odd after the mixing step => no all-zero seed => no NaN from normalize
    ns = np.random.default_rng(1).integers(0, 2**32, 200000, dtype=np.uint64).astype(np.uint32)
    h = N.hash3(ns)
    assert (h > 0).all() and (h <= 1).all()
    assert F(0x7FFFFFFF) == F(2147483648.0)


def test_camera_constants_kat():
    assert O.tan_half(F(1.5708)) == F(1.0000036)
    cam = default_camera_block()
    ipd, lfl = cam["image_plane_distance"], cam["lens_focal_length"]
    assert F((ipd * lfl) / (ipd - lfl)) == F(0.10101011)
    T = cam["transform"].reshape(4, 4)  # rows = columns of the column-major matrix
    assert np.array_equal(T[0, :3], np.array([0.2248595, 0, -0.97439116], np.float32))
    assert np.array_equal(T[1, :3], np.array([-0.14445336, 0.9889499, -0.03333539], np.float32))
    assert np.array_equal(T[2, :3], np.array([0.96362406, 0.14824986, 0.22237478], np.float32))
    assert np.array_equal(T[3], np.array([13, 2, 3, 1], np.float32))


@pytest.mark.parametrize("xy,d", [((960, 540), (-0.96362406, -0.14824986, -0.22237478)),
                                  ((0, 0), (-0.9686123, 0.11266974, 0.22157523)),
                                  ((1919, 1079), (-0.7034691, -0.36952055, -0.60711265))])
def test_primary_ray_kat(xy, d):
    cam = default_camera_block()
    o, dd = O.primary_ray(cam, 1920, 1080, *xy)
    assert np.array_equal(o, np.array([13, 2, 3], np.float32))
    # Appendix C prints 8 significant digits: equal within 1 ulp
    np.testing.assert_array_max_ulp(dd, np.array(d, np.float32), maxulp=1)
    cc = N.camera_consts(camf(cam), 1920, 1080)
    o2, d2 = N.primary_rays(cc, np.array([xy[0]]), np.array([xy[1]]))
    assert np.array_equal(o2[0], o) and np.array_equal(d2[0], dd)


@pytest.mark.parametrize("d,exp", [((0, 1, 0), (0.25, 0.55, 1.0)), ((1, 0, 0), (0.5, 0.7, 1.0)),
                                   ((0, -1, 0), (0.75, 0.85, 1.0))])
def test_sky_kat(d, exp):
    s = O.sky(d)
    np.testing.assert_allclose(s, exp, rtol=0, atol=6e-8)
    assert np.array_equal(N.sky(np.array([d], np.float32))[0], s)


# ------------------------------------------------------- C vs numpy restatement
def _scene_arrays(sc):
    return sc.objects_gpu(), sc.materials_gpu()


def glass_scene():
    """Dielectric-heavy scene exercising TIR, Schlick and refraction (shade.wgsl:163-187)."""
    mats = scene.MaterialCache()
    mats.insert("ground", scene.RayTraceMaterial((0.5, 0.5, 0.5, 1), scene.Reflectance.Lambertian, 1.0, 0))
    mats.insert("glass", scene.RayTraceMaterial((1, 1, 1, 1), scene.Reflectance.Dielectric, 0.0, 1.5))
    mats.insert("diamond", scene.RayTraceMaterial((1, 1, 1, 1), scene.Reflectance.Dielectric, 0.0, 2.4))
    mats.insert("fuzz", scene.RayTraceMaterial((0.9, 0.8, 0.7, 1), scene.Reflectance.Metallic, 0.5, 0))
    sp = [scene.Sphere((0, -1000, -1), 1000, 0), scene.Sphere((0, 1, 0), 1, 1),
          scene.Sphere((0, 1, 0), -0.9, 1), scene.Sphere((-4, 1, 0), 1, 2),
          scene.Sphere((4, 1, 0), 1, 3), scene.Sphere((2, 0.5, 2), 0.5, 2)]
    return scene.Scene(sp, mats, "glass")


CROSS = [
    ("config1", scene.config1_scene, 48, 27, 4, 8, 0),
    ("reference", scene.reference_scene, 40, 24, 2, 3, 3),
    ("rtiow", scene.rtiow_final_scene, 32, 18, 2, 16, 0),
    ("glass", glass_scene, 40, 24, 3, 12, 5),
    ("tiny", scene.config1_scene, 1, 1, 9, 4, 0),
    ("depth1", scene.config1_scene, 17, 9, 3, 1, 0),
]


@pytest.mark.parametrize("name,mk,W,H,S,D,f0", CROSS, ids=[c[0] for c in CROSS])
def test_c_vs_numpy(name, mk, W, H, S, D, f0):
    sp, mt = _scene_arrays(mk())
    cam = default_camera_block()
    a, sa = O.render(cam, sp, mt, W, H, S, D, frame0=f0, nthreads=4)
    b, sb = N.render(camf(cam), sp, mt, W, H, S, D, frame0=f0)
    assert sa == sb
    assert np.array_equal(a, b, equal_nan=True)


def test_empty_scene_is_sky():
    cam = default_camera_block()
    sp = np.zeros(0, SPHERE_DTYPE)
    mt = np.zeros(0, MATERIAL_DTYPE)
    img, segs = O.render(cam, sp, mt, 16, 9, 3, 4)
    assert segs == 16 * 9 * 3  # one segment per path, all misses
    o, d = O.primary_ray(cam, 16, 9, 5, 4)
    assert np.array_equal(img[4, 5, :3], O.sky(d))
    assert (img[..., 3] == 1).all()


def test_oracle_rejects_bad_scene():
    sc = scene.config1_scene()
    sp, mt = _scene_arrays(sc)
    sp = sp.copy()
    sp[1]["material"] = 99
    with pytest.raises(ValueError):
        O.render(default_camera_block(), sp, mt, 4, 4, 1, 2)


def test_shard_union_equals_full():
    """Row tiling is exact: the union of shard renders is the full render."""
    from bevy_raytrace_amd.distributed import ShardLayout, assemble_host
    sp, mt = _scene_arrays(scene.config1_scene())
    cam = default_camera_block()
    W, H, S, D = 24, 23, 2, 6
    full, segs = O.render(cam, sp, mt, W, H, S, D, nthreads=4)
    for world, B in [(2, 3), (3, 5), (4, 1)]:
        lay = ShardLayout(H, B, world)
        g = np.zeros((world, lay.max_rows, W, 4), np.float32)
        tot = 0
        for k in range(world):
            part, s = O.render(cam, sp, mt, W, H, S, D, row_block=B, shard_count=world,
                               shard_index=k, nthreads=2)
            g[k, :part.shape[0]] = part
            tot += s
        assert tot == segs
        assert np.array_equal(assemble_host(g, lay), full, equal_nan=True)


def test_nan_paths_are_reference_behaviour():
    """A Lambertian ray re-hitting its own sphere from inside (no origin offset,
    shade.wgsl:123) with the per-(pixel,frame) seed reused every bounce
    (shade.wgsl:216-218) converges to n == -normalize(seed): normalize(0) = NaN.
    Both restatements agree on these NaN paths."""
    sc = scene.rtiow_final_scene()
    sp, mt = _scene_arrays(sc)
    cam = default_camera_block()
    c, segs = O.trace_path(cam, sp, mt, 1920, 1080, 481, 415, 7, 16)
    assert np.isnan(c).all() and segs == 6
    cc = N.camera_consts(camf(cam), 1920, 1080)
    mats = dict(index=sp.view(np.uint32).reshape(-1, 8)[:, 4].astype(np.int64),
                color=mt.view(np.float32).reshape(-1, 8)[:, 0:3], refl=mt.view(np.int32).reshape(-1, 8)[:, 4],
                fuzz=mt.view(np.float32).reshape(-1, 8)[:, 5], ior=mt.view(np.float32).reshape(-1, 8)[:, 6])
    sph = sp.view(np.float32).reshape(-1, 8)[:, 0:4].copy()
    c2, s2 = N.trace(sph, mats, cc, 1920, 1080, np.array([481]), np.array([415]), 7, 16)
    assert np.isnan(c2).all() and s2 == 6


# ------------------------------------------------------------ golden fixtures
GOLDEN = sorted(p for p in glob.glob(os.path.join(HERE, "golden", "*.npz"))
                if not os.path.basename(p).startswith("wgsl_"))
WGSL = sorted(p for p in glob.glob(os.path.join(HERE, "golden", "wgsl_*.npz"))
              if not os.path.basename(p).startswith("wgsl_isect_"))
WGSL_ISECT = sorted(glob.glob(os.path.join(HERE, "golden", "wgsl_isect_*.npz")))


def check_against_reference_intersect(sp, z, idx, t):
    """(index, t) of a closest-hit loop vs the record the reference's own
    intersect_world returned: t bit for bit, misses at VERY_FAR, and the hit
    sphere's material."""
    assert np.array_equal(t, z["t"], equal_nan=True)
    hit = idx >= 0
    assert np.array_equal(~hit, z["t"] == np.float32(1e20))
    assert np.array_equal(sp["material"][idx[hit]], z["material"][hit])


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_golden_fixture(path):
    z = np.load(path, allow_pickle=False)
    sp = z["spheres"].view(SPHERE_DTYPE)
    mt = z["materials"].view(MATERIAL_DTYPE)
    cam = z["camera"].view(np.float32)
    W, H, S, D, f0 = (int(v) for v in z["params"])
    img, segs = O.render(cam, sp, mt, W, H, S, D, frame0=f0, nthreads=4)
    assert segs == int(z["segments"][0])
    assert np.array_equal(img, z["image"], equal_nan=True)


def test_golden_fixtures_present():
    assert len(GOLDEN) >= 4
    assert len(WGSL) >= 4 and len(WGSL_ISECT) >= 3


@pytest.mark.parametrize("path", WGSL_ISECT, ids=[os.path.basename(p) for p in WGSL_ISECT])
def test_oracle_intersect_matches_reference_intersect_world(path):
    """Adversarial rays (grazing, on/inside surfaces, far origins, NaN/inf and
    unnormalised directions; tests/raygen.py) through intersect.wgsl's own
    intersect_world, executed by the WGSL interpreter."""
    z = np.load(path, allow_pickle=False)
    sp = z["spheres"].view(SPHERE_DTYPE)
    idx, t = O.intersect_batch(sp, z["rays"])
    check_against_reference_intersect(sp, z, idx, t)
    assert 0 < (idx >= 0).sum() < len(idx)


@pytest.mark.parametrize("path", WGSL, ids=[os.path.basename(p) for p in WGSL])
def test_oracle_matches_interpreted_reference_wgsl(path):
    """Each frame of RayTraceNode::run (clear, generate, 3 x {prepass,
    intersect, shade}, collect; ray_trace_node.rs:195-224) executed from the
    reference's WGSL == the oracle's frame (spp 1, frame0 = that frame,
    depth 3), bit for bit."""
    z = np.load(path, allow_pickle=False)
    sp = z["spheres"].view(SPHERE_DTYPE)
    mt = z["materials"].view(MATERIAL_DTYPE)
    cam = z["camera"].view(np.float32)
    W, H, S, D = (int(v) for v in z["params"])
    # depth 3 = the reference's own schedule; the *_d16 fixtures run its
    # shaders with the bounce-kill constant generalised (make_wgsl_golden.py)
    assert S == 1 and (D == 3 or os.path.basename(path).endswith("_d16.npz"))
    n = int(z["processed"][0])  # pixels the reference's floor-divided grid traces (D1)
    for f, ref in zip(z["frames"], z["images"]):
        img, _ = O.render(cam, sp, mt, W, H, S, D, frame0=int(f), nthreads=4)
        assert np.array_equal(img.reshape(-1, 4)[:n], ref.reshape(-1, 4)[:n],
                              equal_nan=True), f"frame {int(f)}"
    # the fixture is not trivially sky: hits and misses, several materials
    assert len(np.unique(z["images"][0].reshape(-1, 4), axis=0)) > W * H // 4


WGSL_ACCUM = [p for p in WGSL if "_accum" in os.path.basename(p)]
WGSL_DEEP = [p for p in WGSL if os.path.basename(p).endswith("_d16.npz")]


def blocked_mean(frames_rgb):
    """The result definition of an S-spp pixel (rt_hip.h RT_SAMPLE_BLOCK): the
    per-sample colours summed in f32 inside blocks of 8 consecutive samples
    (0 + c0 + c1 ...), the block sums folded in block order, / f32(S), alpha 1."""
    S = len(frames_rgb)
    acc = None
    for b in range(0, S, 8):
        bs = np.zeros_like(frames_rgb[0][..., :3])
        for c in frames_rgb[b:b + 8]:
            bs = bs + c[..., :3]
        acc = bs if acc is None else acc + bs
    out = np.ones(frames_rgb[0].shape, np.float32)
    out[..., :3] = acc / np.float32(S)
    return out


def test_wgsl_accumulation_and_depth_fixtures_present():
    assert WGSL_ACCUM and len(WGSL_DEEP) >= 2


@pytest.mark.parametrize("path", WGSL_ACCUM, ids=[os.path.basename(p) for p in WGSL_ACCUM])
def test_oracle_spp_is_blocked_sum_of_reference_frames(path):
    """An S-spp frame == the blocked f32 sum of the reference's S one-sample
    frames (its SAMPLES_PER_RAY = 1 frames 0..S-1, executed from its WGSL) /
    S: pins this build's sample accumulation against the reference's
    per-frame output, not only against itself."""
    z = np.load(path, allow_pickle=False)
    sp = z["spheres"].view(SPHERE_DTYPE)
    mt = z["materials"].view(MATERIAL_DTYPE)
    cam = z["camera"].view(np.float32)
    W, H, _, D = (int(v) for v in z["params"])
    frames = [int(f) for f in z["frames"]]
    assert frames == list(range(frames[0], frames[0] + len(frames)))
    img, _ = O.render(cam, sp, mt, W, H, len(frames), D, frame0=frames[0], nthreads=4)
    assert np.array_equal(img, blocked_mean(list(z["images"])), equal_nan=True)


# ------------------------------------------- opt-in camera sampling (§8f row 4)
def test_sincos_accuracy_and_restatements():
    """rt_sincos (include/rt_hip.h): C == numpy bit for bit, |err| < 2e-7
    against the double-precision sin/cos of the same f32 angle."""
    two_pi = np.float32(2.0) * np.float32(3.14159265358979)
    th = np.concatenate([np.linspace(two_pi, 2 * two_pi, 4001, dtype=np.float32),
                         np.linspace(-7.0, 7.0, 2001, dtype=np.float32),
                         np.float32([0.0, two_pi, 2 * two_pi, 1e-30])])
    ns, nc = N.sincos(th)
    for i in range(0, th.size, 7):
        cs, cc = O.sincos(th[i])
        assert cs == ns[i] and cc == nc[i], th[i]
    assert np.abs(ns.astype(np.float64) - np.sin(th.astype(np.float64))).max() < 2e-7
    assert np.abs(nc.astype(np.float64) - np.cos(th.astype(np.float64))).max() < 2e-7


SAMPLING = [("jitter", 0x2), ("thin_lens", 0x4), ("both", 0x6)]


@pytest.mark.parametrize("fname,flags", SAMPLING, ids=[s[0] for s in SAMPLING])
@pytest.mark.parametrize("name,mk", [("config1", scene.config1_scene), ("glass", glass_scene)])
def test_c_vs_numpy_camera_sampling(fname, flags, name, mk):
    """Jitter / thin-lens camera sampling: the two restatements agree bit for
    bit, and the flags change the image (they are not the reference default)."""
    sp, mt = _scene_arrays(mk())
    cam = camera_block(Transform.from_xyz(13.0, 2.0, 3.0).looking_at((0.0, 0.0, 0.0)),
                       lens_focal_length=0.05, fstop=8.0)
    W, H, S, D, f0 = 36, 20, 3, 8, 2
    a, sa = O.render(cam, sp, mt, W, H, S, D, frame0=f0, nthreads=4, flags=flags)
    b, sb = N.render(camf(cam), sp, mt, W, H, S, D, frame0=f0, flags=flags)
    assert sa == sb
    assert np.array_equal(a, b, equal_nan=True)
    base, _ = O.render(cam, sp, mt, W, H, S, D, frame0=f0, nthreads=4)
    assert not np.array_equal(a, base, equal_nan=True)
