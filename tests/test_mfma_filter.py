"""The matrix-core filter's margin proof, checked numerically on the CPU.

rt_dev_intersect.h intersect_world_mfma decides which spheres get the
reference's exact test (intersect.wgsl:97-115) from two f16 hi/lo MFMA tiles:
hb' = k1 - dn.c and v' = S' + o2.c, then H' = fma(hb', hb', v') against
T' = (1 - m - mu')|o|^2 - 2^-20. The product is bit-exact only if that test
is conservative: every sphere whose exact test accepts a root must have
H' >= T'. This file restates the kernel's arithmetic in numpy -- the ray
constants, the f16 splits, the A rows of rt_api.cpp build_mfma, the MFMA's
16-product f32 sums in three summation orders (the hardware's is not
documented) -- and checks that property on the adversarial ray sets of the
GPU intersection tests (tests/raygen.py), for every (ray, sphere) pair whose
ray lies inside the filter's range (|o_i| <= 2^12, the kernel's
mfma_wave_ok). It also checks the error bound the proof states against the
exact value of H.
"""
import zlib

import numpy as np
import pytest

from bevy_raytrace_amd import scene
from raygen import adversarial_rays

F, H16, D = np.float32, np.float16, np.float64
M, MU, ABS = 2.0 ** -16, 2.0 ** -16, 2.0 ** -20  # rt_dev_intersect.h RT_MF_MU, RT_MF_ABS
EPSILON, VERY_FAR = F(0.001), F(1e20)


def fma32(a, b, c):
    """f32 fma: the f64 product of two f32 is exact, one rounding to f32
    after the add (double rounding cannot flip a comparison here by more than
    the f64 ulp, far inside the margins)."""
    return (D(a) * D(b) + D(c)).astype(F)


def split(x):
    """split_h: hi = RN_f16(x), lo = RN_f16(x - hi) (x - hi exact in f32)."""
    x = np.asarray(x, F)
    hi = x.astype(H16).astype(F)
    lo = (x - hi).astype(H16).astype(F)
    return hi, lo


def ray_columns(rays):
    """The B columns u (hb) and v (v + S) of each ray, as the kernel builds
    them; returns u, v (n, 16) f32 and T' (n,)."""
    o, d = rays[:, :3].astype(F), rays[:, 3:].astype(F)
    dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        rs = (1.0 / np.sqrt(D(dd))).astype(F)  # v_rsq_f32 (<= 1 ulp; covered by m)
    dn = d * rs[:, None]
    oo = fma32(o[:, 2], o[:, 2], fma32(o[:, 1], o[:, 1], o[:, 0] * o[:, 0]))
    k1 = fma32(dn[:, 2], o[:, 2], fma32(dn[:, 1], o[:, 1], dn[:, 0] * o[:, 0]))
    two = F(2.0) * (F(1.0) - F(M))
    T = F(1.0 - M - MU) * oo - F(ABS)
    z = np.zeros(len(rays), F)
    one = np.ones(len(rays), F)
    xh, xl = split(-dn[:, 0])
    yh, yl = split(-dn[:, 1])
    zh, zl = split(-dn[:, 2])
    kh, kl = split(k1)
    ph, pl = split(two * o[:, 0])
    qh, ql = split(two * o[:, 1])
    rh, rl = split(two * o[:, 2])
    u = np.stack([xh, xh, xl, yh, yh, yl, zh, zh, zl, kh, kl, z, z, z, z, z], 1)
    v = np.stack([ph, ph, pl, qh, qh, ql, rh, rh, rl, z, z, one, one, z, z, z], 1)
    return u, v, T


def sphere_rows(sp):
    """rt_api.cpp build_mfma: A row of sphere j (f32 values of the f16 parts)."""
    c = sp["center"].astype(F)
    r2 = (sp["radius"] * sp["radius"]).astype(F)  # the stored s.w = RN(r*r)
    rows = []
    for a in range(3):
        hi = c[:, a].astype(H16)
        lo = (D(c[:, a]) - D(hi)).astype(H16)
        rows += [hi, lo, hi]
    cc = (D(c) ** 2).sum(1)
    S = D(r2) - (1.0 - 2.0 ** -16 - 2.0 ** -16) * cc
    assert np.all(np.abs(S) <= 2.0 ** 15) and np.all(np.abs(c) <= 2.0 ** 12)  # mf_ok
    sh = S.astype(H16)
    sl = (S - D(sh)).astype(H16)
    n = len(sp)
    rows += [np.ones(n, H16), np.ones(n, H16), sh, sl] + [np.zeros(n, H16)] * 3
    return np.stack(rows, 1).astype(F)  # (n, 16)


def mfma_sum(A, B, order):
    """sum_k A[j,k] B[i,k] -> (rays, spheres) f32. Each product is exact in
    f32 (two f16); the 16-term sum is rounded per the order."""
    P = A[None, :, :].astype(D) * B[:, None, :].astype(D)  # (rays, spheres, 16) exact
    if order == "exact":
        return P.sum(-1).astype(F)
    if order == "pairwise":
        P = P.astype(F)
        while P.shape[-1] > 1:
            P = (P[..., 0::2] + P[..., 1::2]).astype(F)
        return P[..., 0]
    ks = range(16) if order == "forward" else range(15, -1, -1)
    acc = np.zeros(P.shape[:2], F)
    for k in ks:
        acc = (acc + P[..., k].astype(F)).astype(F)
    return acc


def exact_hits(sp, rays):
    """Per (ray, sphere): the reference's exact test yields a root that can
    become the closest hit (intersect.wgsl:97-115 and :137, the oracle's f32
    op forms)."""
    o, d = rays[:, :3].astype(F), rays[:, 3:].astype(F)
    l = np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2])
    a = (l * l)[:, None]
    c = sp["center"].astype(F)[None, :, :]
    r = sp["radius"].astype(F)[None, :]
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        oc = o[:, None, :] - c
        hb = (oc[..., 0] * d[:, None, 0] + oc[..., 1] * d[:, None, 1]) + oc[..., 2] * d[:, None, 2]
        qq = (oc[..., 0] * oc[..., 0] + oc[..., 1] * oc[..., 1]) + oc[..., 2] * oc[..., 2]
        lo = np.sqrt(qq)
        cq = lo * lo - r * r
        dis = hb * hb - a * cq
        ok = ~(dis < F(0.0))
        sq = np.sqrt(np.where(ok, dis, F(0.0)))
        r1 = (-hb - sq) / a
        r2 = (-hb + sq) / a
        bad1 = (r1 < EPSILON) | (VERY_FAR < r1)
        bad2 = (r2 < EPSILON) | (VERY_FAR < r2)
        root = np.where(bad1, r2, r1)
    # a NaN root never wins the strict `<` against best_t (intersect.wgsl:137)
    return ok & ~(bad1 & bad2) & (root < VERY_FAR)


SCENES = {
    "rtiow": lambda: scene.rtiow_final_scene().objects_gpu(),
    "reference": lambda: scene.reference_scene().objects_gpu(),
    "config1": lambda: scene.config1_scene().objects_gpu(),
    "spheres10k": lambda: scene.ten_thousand_scene().objects_gpu()[:2048],
}


@pytest.mark.parametrize("name", sorted(SCENES))
def test_matrix_core_filter_is_conservative(name):
    sp = SCENES[name]()
    n = 16_000 if len(sp) < 1000 else 4_000
    rays = adversarial_rays(sp, n, seed=zlib.crc32(name.encode()) % 1000)
    inside = np.abs(rays[:, :3]).max(1) <= 2.0 ** 12  # mfma_wave_ok
    rays = rays[inside]
    u, v, T = ray_columns(rays)
    A = sphere_rows(sp)
    hits = exact_hits(sp, rays)
    assert hits.sum() > 1000  # the set really has hits to lose
    checked = 0
    for order in ("exact", "pairwise", "forward", "backward"):
        for j0 in range(0, len(sp), 256):
            Aj = A[j0:j0 + 256]
            hb = mfma_sum(Aj, u, order)
            vs = mfma_sum(Aj, v, order)
            with np.errstate(invalid="ignore", over="ignore"):
                Hp = fma32(hb, hb, vs)
                cand = Hp >= T[:, None]
            lost = hits[:, j0:j0 + 256] & ~cand
            assert not lost.any(), (
                f"{order}: {int(lost.sum())} exact hits filtered out, e.g. ray "
                f"{np.argwhere(lost)[0].tolist()}")
            checked += int(hits[:, j0:j0 + 256].sum())
    assert checked > 4000


@pytest.mark.parametrize("name", ["rtiow", "spheres10k"])
def test_split_error_within_stated_bound(name):
    """|H' - H~| <= 2^-17 (|o|^2 + |c|^2) + 2^-20.3 r^2 + 2^-21, the bound the
    kernel's margins are built from (rt_dev_intersect.h), where H~ is the
    exact value of hb~^2 + S' + o2.c with the kernel's f32 ray constants."""
    sp = SCENES[name]()
    rays = adversarial_rays(sp, 4_000, seed=7)
    rays = rays[np.abs(rays[:, :3]).max(1) <= 2.0 ** 12]
    rays = rays[np.isfinite(rays).all(1) & (np.abs(rays[:, 3:]).max(1) > 0)]
    u, v, _ = ray_columns(rays)
    # exact operands: the unsplit f32 ray constants and the f32 sphere values
    xs = u[:, 0] + u[:, 2], u[:, 3] + u[:, 5], u[:, 6] + u[:, 8]
    o2 = v[:, 0] + v[:, 2], v[:, 3] + v[:, 5], v[:, 6] + v[:, 8]
    o = rays[:, :3].astype(D)
    c = sp["center"].astype(D)
    r2 = (sp["radius"] * sp["radius"]).astype(F).astype(D)
    S = r2 - (1.0 - 2.0 ** -15) * (c ** 2).sum(1)
    k1 = D(u[:, 9]) + D(u[:, 10])
    hb_x = k1[:, None] + sum(D(xs[a])[:, None] * c[None, :, a] for a in range(3))
    v_x = S[None, :] + sum(D(o2[a])[:, None] * c[None, :, a] for a in range(3))
    H_x = hb_x * hb_x + v_x
    A = sphere_rows(sp)
    worst = 0.0
    for order in ("exact", "pairwise", "forward", "backward"):
        hb = mfma_sum(A, u, order)
        vs = mfma_sum(A, v, order)
        Hp = fma32(hb, hb, vs).astype(D)
        bound = (2.0 ** -17 * ((o ** 2).sum(1)[:, None] + (c ** 2).sum(1)[None, :])
                 + 2.0 ** -20.3 * r2[None, :] + 2.0 ** -21)
        worst = max(worst, float(np.max(np.abs(Hp - H_x) / bound)))
    assert worst < 1.0, worst
