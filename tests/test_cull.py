"""Culled list (RT_FLAG_CULL), host side, CPU only: the layout rt_api.cpp
build_cull makes (a permutation of the spheres into groups, clusters of 8
groups, a bounding record per group) and the property the kernel relies on --
a lane with a filter candidate in a group passes that group's bound
(rt_api.cpp cull_layout, proof in its comment) -- checked with an f32
emulation of the kernel's filter (rt_dev_intersect.h ray_filter_consts,
filter8) on the adversarial ray sets of tests/raygen.py. The GPU results of
the culled path are compared with the oracle in test_gpu_parity.py /
test_gpu_intersect.py."""
import numpy as np
import pytest

from bevy_raytrace_amd import abi, scene
from raygen import adversarial_rays

F = np.float32
M, MU, MUB = 2.0 ** -16, 2.0 ** -17, 2.0 ** -7


def fma(a, b, c):
    """f32 fma emulated in f64 (exact product; the sum rounds twice, which can
    move a result by one f32 ulp -- far inside the bound's margin)."""
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(F)


def ray_consts(rays):
    o = rays[:, :3].astype(F)
    d = rays[:, 3:].astype(F)
    dd = fma(d[:, 2], d[:, 2], fma(d[:, 1], d[:, 1], d[:, 0] * d[:, 0]))
    with np.errstate(all="ignore"):
        rs = (F(1.0) / np.sqrt(dd)).astype(F)
        dn = (d * rs[:, None]).astype(F)
        oo = fma(o[:, 2], o[:, 2], fma(o[:, 1], o[:, 1], o[:, 0] * o[:, 0]))
        k1 = fma(dn[:, 2], o[:, 2], fma(dn[:, 1], o[:, 1], dn[:, 0] * o[:, 0]))
        o2 = (F(2.0 * (1.0 - M)) * o).astype(F)
        T = (F(1.0 - M - MU) * oo).astype(F)
        TB = (F(1.0 - M - MUB) * oo).astype(F)
        a = dd  # |d|^2 (the kernel's a = sqr(length(d)) differs by an ulp at most)
        om = np.abs(o).max(1)
        ok = (om <= 2.0 ** 30) & (a >= 2.0 ** -100) & (a <= 2.0 ** 100)
    return dict(ndn=-dn, k1=k1, o2=o2, T=T, TB=TB, ok=ok)


def filt(R, c, S):
    """H for rays R (n) x spheres c (g, 3), S (g) -> (n, g), filter8's op order."""
    with np.errstate(all="ignore"):
        ndn, k1, o2 = R["ndn"][:, None, :], R["k1"][:, None], R["o2"][:, None, :]
        cx, cy, cz = (np.broadcast_to(c[None, :, k], (len(k1), len(c))) for k in range(3))
        hb = fma(np.broadcast_to(ndn[..., 0], cx.shape), cx, np.broadcast_to(k1, cx.shape))
        hb = fma(np.broadcast_to(ndn[..., 1], cy.shape), cy, hb)
        hb = fma(np.broadcast_to(ndn[..., 2], cz.shape), cz, hb)
        H = fma(hb, hb, np.broadcast_to(S[None, :], hb.shape))
        H = fma(np.broadcast_to(o2[..., 2], cz.shape), cz, H)
        H = fma(np.broadcast_to(o2[..., 1], cy.shape), cy, H)
        H = fma(np.broadcast_to(o2[..., 0], cx.shape), cx, H)
    return H


def member_S(sp):
    c = sp["center"].astype(np.float64)
    r2 = (sp["radius"] * sp["radius"]).astype(F)
    return (r2.astype(np.float64) - (1.0 - M - MU) * (c * c).sum(1)).astype(F)


def check_layout(sp):
    perm, bnd, cbnd, ng, nc = abi.cull_layout(sp)
    n = len(sp)
    real = perm[perm >= 0]
    assert sorted(real.tolist()) == list(range(n))
    assert nc == (ng + 7) // 8 and len(bnd) == nc * 8 and len(cbnd) == (nc + 7) // 8 * 8
    assert (perm[ng * 8:] < 0).all()
    for g in range(nc * 8):  # empty groups never pass, non-empty ones may
        members = perm[g * 8:(g + 1) * 8] if g < ng else np.array([-1])
        if (members < 0).all():
            assert bnd[g, 3] == -np.inf
    assert (cbnd[nc:, 3] == -np.inf).all()  # pad clusters of the last super
    return perm, bnd, cbnd, ng, nc


def dominance(sp, rays, chunk=4000):
    """Count (ray, group) pairs where a member is a candidate but the bound
    fails, over the rays the kernel culls for; and the bound pass rate."""
    perm, bnd, cbnd, ng, nc = check_layout(sp)
    S = member_S(sp)
    c = sp["center"].astype(F)
    viol = tested = passed = 0
    for s0 in range(0, len(rays), chunk):
        R = ray_consts(rays[s0:s0 + chunk])
        HB = filt(R, bnd[:, :3].astype(F), bnd[:, 3].astype(F))  # (n, nc*8)
        HC = filt(R, cbnd[:, :3].astype(F), cbnd[:, 3].astype(F))  # (n, supers*8)
        with np.errstate(invalid="ignore"):
            bpass = HB >= R["TB"][:, None]
            cpass = HC >= R["TB"][:, None]
        for g in range(ng):
            mem = perm[g * 8:(g + 1) * 8]
            mem = mem[mem >= 0]
            if mem.size == 0:
                continue
            H = filt(R, c[mem], S[mem])
            with np.errstate(invalid="ignore"):
                cand = (H >= R["T"][:, None]).any(1)
            bad = cand & ~(bpass[:, g] & cpass[:, g // 8]) & R["ok"]
            viol += int(bad.sum())
            tested += int(R["ok"].sum())
            passed += int((bpass[:, g] & R["ok"]).sum())
    return viol, passed / max(1, tested)


def tangent_pair():
    """Two unit spheres touching at (1, 0, 0), the later one (index 1) first in the
    culled order: rays through the contact point tie exactly."""
    mats = scene.MaterialCache()
    mats.insert("a", scene.RayTraceMaterial((0.5, 0.5, 0.5, 1), scene.Reflectance.Lambertian, 1, 0))
    sp = [scene.Sphere((2, 0, 0), 1, 0), scene.Sphere((0, 0, 0), 1, 0)]
    return scene.Scene(sp, mats, "tangent")


SCENES = {
    "rtiow": lambda: scene.rtiow_final_scene().objects_gpu(),
    "spheres10k": lambda: scene.ten_thousand_scene().objects_gpu()[::7].copy(),
    "reference": lambda: scene.reference_scene().objects_gpu(),
    "config1": lambda: scene.config1_scene().objects_gpu(),
    "tangent": lambda: tangent_pair().objects_gpu(),
}


@pytest.mark.parametrize("name", sorted(SCENES))
def test_bounds_dominate_members(name):
    sp = SCENES[name]()
    rays = adversarial_rays(sp, 24_000, seed=7)
    viol, rate = dominance(sp, rays)
    assert viol == 0


def test_bounds_dominate_far_scene():
    sp = scene.rtiow_final_scene().objects_gpu().copy()
    sp["center"] += np.asarray((1e4, -3e3, 2e4), F)
    rays = adversarial_rays(scene.rtiow_final_scene().objects_gpu(), 16_000, seed=3)
    rays[:, :3] += np.asarray((1e4, -3e3, 2e4), F)
    viol, _ = dominance(sp, rays)
    assert viol == 0


def test_bounds_cull_rtiow():
    """The point of the layout: on camera-like rays into the RTIOW scene most
    groups' bounds fail for most rays."""
    sp = scene.rtiow_final_scene().objects_gpu()
    rng = np.random.default_rng(0)  # (pass rate of the group bounds alone)
    o = np.tile([13.0, 2.0, 3.0], (4000, 1))
    tgt = rng.uniform([-11, 0, -11], [11, 1, 11], (4000, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    viol, rate = dominance(sp, np.hstack([o, d]).astype(F))
    assert viol == 0
    assert rate < 0.4


def test_layout_edge_cases():
    # empty, one sphere, huge / non-finite members (always-pass bounds)
    perm, bnd, cbnd, ng, nc = abi.cull_layout(scene.Scene([], scene.MaterialCache(), "e").objects_gpu())
    assert ng == 0 and nc == 0 and len(cbnd) == 0
    sp = scene.rtiow_final_scene().objects_gpu()[:9].copy()
    sp["center"][3] = (2.0 ** 31, 0, 0)
    sp["radius"][5] = np.inf
    perm, bnd, cbnd, ng, nc = check_layout(sp)
    for bad in (3, 5):
        g = int(np.nonzero(perm == bad)[0][0]) // 8
        assert bnd[g, 3] == np.inf and (bnd[g, :3] == 0).all()
        assert cbnd[g // 8, 3] == np.inf
    one = sp[:1].copy()
    perm, bnd, cbnd, ng, nc = check_layout(one)
    assert ng == 1 and nc == 1


def test_tangent_pair_order():
    """The tie-break test's premise: the later sphere comes first in the
    culled list (so the kernel must compare original indices)."""
    perm = abi.cull_layout(tangent_pair().objects_gpu())[0]
    assert perm[0] == 1 and perm[1] == 0
