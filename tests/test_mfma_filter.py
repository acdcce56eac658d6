"""The matrix-core filter's margin proof, checked numerically on the CPU.

rt_dev_intersect.h intersect_world_mfma decides which spheres get the
reference's exact test (intersect.wgsl:97-115) from one 32-term dot product
per (sphere, ray) pair on the matrix cores: V = T0 - H0, H0 = S' + L.c +
sum_ab Q_ab c_a c_b (the VALU filter's hb^2 + S + o2.c less the ray's k1^2),
T0 = (1 - m - mu')|o|^2 - k1^2 - abs' one more term of the dot product, every
feature and T0 split into f16 hi/lo parts; a sphere is a candidate iff V < 0.
The product is bit-exact only if that test is conservative: every sphere
whose exact test yields a root that can win must have V < 0. This file restates
the kernel's arithmetic in numpy -- the ray constants and features, the f16
splits, the A rows of rt_api.cpp build_mfma (with its scale 2^sq of the
quadratic features), the two chained MFMAs' 32-product f32 sums in four
summation orders (the hardware's is not documented) -- and checks that
property on the adversarial ray sets of the GPU intersection tests
(tests/raygen.py), for every (ray, sphere) pair whose ray lies inside the
filter's range (|o_i| <= 2^12, |o|^2 <= 2^15, the kernel's mfma_wave_ok). It also checks the
error bound the kernel's margins are built from against the exact value.
"""
import zlib

import numpy as np
import pytest

from bevy_raytrace_amd import scene
from raygen import adversarial_rays

F, H16, D = np.float32, np.float16, np.float64
M, MU = 2.0 ** -16, 2.0 ** -16  # rt_dev_intersect.h m_, RT_MF_MU
EPSILON, VERY_FAR = F(0.001), F(1e20)
QUAD = [(0, 0), (1, 1), (2, 2), (0, 1), (0, 2), (1, 2)]


def fma32(a, b, c):
    """f32 fma: the f64 product of two f32 is exact, one rounding to f32
    after the add (the double rounding is far inside the margins)."""
    return (D(a) * D(b) + D(c)).astype(F)


def split(x):
    """The kernel's ray-side split: hi = RN_f16(x), lo = RN_f16(x - hi)
    (x - hi exact in f32)."""
    x = np.asarray(x, F)
    hi = x.astype(H16).astype(F)
    lo = (x - hi).astype(H16).astype(F)
    return hi, lo


def qscale(sp):
    """build_mfma's sq: max |c_a c_b| 2^-sq <= 2^14."""
    c = sp["center"].astype(F).astype(D)
    mx = max(1.0, float(np.max(np.abs(c[:, :, None] * c[:, None, :]))))
    sq = 0
    while mx * 2.0 ** -sq > 2.0 ** 14:
        sq += 1
    return sq


def sphere_rows(sp, sq):
    """rt_api.cpp build_mfma: A row of each sphere (f32 values of the f16
    parts), K = 32."""
    c = sp["center"].astype(F).astype(D)
    r2 = (sp["radius"] * sp["radius"]).astype(F).astype(D)  # the stored s.w = RN(r*r)
    assert np.all(np.abs(c) <= 2.0 ** 12)  # mf_ok
    S = r2 - (1.0 - M - MU) * (c ** 2).sum(1)
    assert np.all(np.abs(S) <= 2.0 ** 15)  # mf_ok
    return rows_of(c, S, sq)


def rows_of(c, S, sq, bound=False, k31=1.0):
    """A rows (f32 values of the f16 parts, K = 32) of centres c (n, 3) and
    constants S' (n,); an infinite S' is its hi part alone (build_mfma)."""
    def hl(x):
        hi = x.astype(H16)
        with np.errstate(invalid="ignore"):
            lo = np.where(np.isinf(x), 0.0, x - hi.astype(D)).astype(H16)
        return hi, lo

    his, los = [], []
    for a in range(3):
        hi, lo = hl(c[:, a])
        his.append(hi)
        los.append(lo)
    for a, b in QUAD:
        hi, lo = hl(c[:, a] * c[:, b] * 2.0 ** -sq)
        his.append(hi)
        los.append(lo)
    shi, slo = hl(S)
    n = len(c)
    one = np.ones(n, H16)
    # K group 0: hi y0..y7, lo y0..y7; group 1: hi y0..y7, hi y8, hi y8, lo y8,
    # 1, 1, S' hi, S' lo, 0 (build_mfma's words w0..w15)
    cols = his[:8] + los[:8] + his[:8] + [his[8], his[8], los[8], one, one, shi, slo,
                                          (one * H16(k31)) if bound else np.zeros(n, H16)]
    return np.stack(cols, 1).astype(F)


def ray_constants(rays):
    """ray_filter_consts' values as the kernel computes them: e = -dn, k1, o2,
    |o|^2 (f32; v_rsq_f32 modelled as the correctly rounded 1/sqrt)."""
    o, d = rays[:, :3].astype(F), rays[:, 3:].astype(F)
    dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        rs = (1.0 / np.sqrt(D(dd))).astype(F)
        e = -(d * rs[:, None])
        oo = fma32(o[:, 2], o[:, 2], fma32(o[:, 1], o[:, 1], o[:, 0] * o[:, 0]))
        k1 = fma32(-e[:, 2], o[:, 2], fma32(-e[:, 1], o[:, 1], -e[:, 0] * o[:, 0]))
    two = F(2.0) * (F(1.0) - F(M))
    return o, e, k1, oo, two * o


def ray_columns(rays, sq, abs_margin):
    """The ray column (n, 32) and threshold T0 (n,), as the kernel builds them:
    the negated features, -1, -1 against S', T0's hi, lo against 1, 1, and
    K 31 = -RN_f16(muB |o|^2) (against 0 in a sphere row, 1 in a block-bound
    row: T0_B's margin)."""
    o, e, k1, oo, o2 = ray_constants(rays)
    sc = F(2.0 ** sq)
    with np.errstate(invalid="ignore", over="ignore"):
        feats = [fma32(F(2.0) * k1, e[:, a], o2[:, a]) for a in range(3)]
        feats += [((F(2.0) * e[:, a] if a != b else e[:, a]) * e[:, b]) * sc for a, b in QUAD]
        T0 = (fma32(-k1, k1, F(1.0 - M - MU) * oo) - F(abs_margin)).astype(F)
        k31 = (-(F(MUB) * oo)).astype(H16).astype(F)
    his, los = [], []
    for x in feats:
        hi, lo = split(-x)
        his.append(hi)
        los.append(lo)
    m1, z = -np.ones(len(rays), F), np.zeros(len(rays), F)
    with np.errstate(invalid="ignore", over="ignore"):
        thi, tlo = split(T0)
    # the kernel's words w0..w15: hi x0..x7 twice, lo x0..x7, (hi x8, lo x8),
    # (hi x8, T0 hi), (T0 lo, -1), (-1, 0)
    cols = his[:8] + his[:8] + los[:8] + [his[8], los[8], his[8], thi, tlo, m1, m1, k31]
    return np.stack(cols, 1), T0


def mfma_sum(A, B, order):
    """sum_k A[j,k] B[i,k] -> (rays, spheres) f32. Each product is exact in
    f32 (two f16); the 32-term sum is rounded per the order ("chained": two
    16-term sums, the second accumulating onto the first, as two MFMAs)."""
    P = A[None, :, :].astype(D) * B[:, None, :].astype(D)
    if order == "exact":
        return P.sum(-1).astype(F)
    if order == "chained":
        return (P[..., :16].sum(-1).astype(F).astype(D) + P[..., 16:].sum(-1)).astype(F)
    if order == "pairwise":
        P = P.astype(F)
        while P.shape[-1] > 1:
            P = (P[..., 0::2] + P[..., 1::2]).astype(F)
        return P[..., 0]
    ks = range(32) if order == "forward" else range(31, -1, -1)
    acc = np.zeros(P.shape[:2], F)
    for k in ks:
        acc = (acc + P[..., k].astype(F)).astype(F)
    return acc


ORDERS = ("exact", "chained", "pairwise", "forward", "backward")


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
    "spheres10k": lambda: scene.ten_thousand_scene().objects_gpu(),
}
# spheres checked per scene (the pair count of the full 10 k list is too large
# for the four summation orders); sq -- hence the f16 rows and abs' -- always
# comes from the WHOLE scene, as build_mfma computes it
SUBSET = {"spheres10k": 2048}


def scene_rows(name):
    full = SCENES[name]()
    return full[:SUBSET.get(name, len(full))], qscale(full)


def _rays(sp, name, n):
    rays = adversarial_rays(sp, n, seed=zlib.crc32(name.encode()) % 1000)
    o = rays[:, :3].astype(F)
    oo = fma32(o[:, 2], o[:, 2], fma32(o[:, 1], o[:, 1], o[:, 0] * o[:, 0]))
    return rays[(np.abs(o).max(1) <= 2.0 ** 12) & (oo <= 2.0 ** 15)]  # mfma_wave_ok


@pytest.mark.parametrize("name", sorted(SCENES))
def test_matrix_core_filter_is_conservative(name):
    sp, sq = scene_rows(name)
    rays = _rays(sp, name, 12_000 if len(sp) < 1000 else 3_000)
    B, T0 = ray_columns(rays, sq, 2.0 ** (sq - 20))
    A = sphere_rows(sp, sq)
    hits = exact_hits(sp, rays)
    assert hits.sum() > 1000  # the set really has hits to lose
    for order in ORDERS:
        for j0 in range(0, len(sp), 256):
            with np.errstate(invalid="ignore", over="ignore"):
                cand = mfma_sum(A[j0:j0 + 256], B, order) < 0  # V = T0 - H0 < 0
            lost = hits[:, j0:j0 + 256] & ~cand
            assert not lost.any(), (
                f"{order}: {int(lost.sum())} exact hits filtered out, e.g. ray "
                f"{np.argwhere(lost)[0].tolist()}")


@pytest.mark.parametrize("name", ["rtiow", "spheres10k"])
def test_error_within_stated_bound(name):
    """|-V' - (H~ - T~)| <= 2^-16.02 (|o|^2 + |c|^2) + 2^-19 |S'| + abs',
    the bound of rt_dev_intersect.h's margin comment, where H~ - T~ is the
    exact value of hb^2 + S' + o2.c - (1 - m - mu')|o|^2 with the kernel's f32
    ray constants e, k1, o2 (hb = k1 + e.c)."""
    sp, sq = scene_rows(name)
    rays = _rays(sp, "bound" + name, 3_000)
    rays = rays[np.isfinite(rays).all(1) & (np.abs(rays[:, 3:]).max(1) > 0)]
    absm = 2.0 ** (sq - 20)
    B, T0 = ray_columns(rays, sq, absm)
    o, e, k1, _, o2 = ray_constants(rays)
    c = sp["center"].astype(F).astype(D)
    r2 = (sp["radius"] * sp["radius"]).astype(F).astype(D)
    S = r2 - (1.0 - M - MU) * (c ** 2).sum(1)
    oo = (o.astype(D) ** 2).sum(1)
    hb = k1.astype(D)[:, None] + e.astype(D) @ c.T
    exact = hb * hb + S[None, :] + o2.astype(D) @ c.T - (1.0 - M - MU) * oo[:, None]
    bound = (2.0 ** -16.02 * (oo[:, None] + (c ** 2).sum(1)[None, :]) + 2.0 ** -19 * np.abs(S)[None, :]
             + absm)
    A = sphere_rows(sp, sq)
    worst = 0.0
    for order in ORDERS:
        got = -mfma_sum(A, B, order).astype(D)  # H0' - T0'
        worst = max(worst, float(np.max(np.abs(got - exact) / bound)))
    assert worst < 1.0, worst


def test_scale_is_the_whole_scenes():
    """sq of every checked scene as build_mfma computes it, from all spheres
    (6 for each: the ground sphere's |c|^2 ~ 2^20 sets it)."""
    assert scene_rows("rtiow")[1] == qscale(SCENES["rtiow"]())
    full = SCENES["spheres10k"]()
    assert scene_rows("spheres10k")[1] == qscale(full)


MUB = 2.0 ** -12  # rt_dev_intersect.h RT_MF_MUB (2^-8 through round 5)


def round_up_f32(v):
    f = np.float32(v)
    return float(np.nextafter(f, np.float32(np.inf))) if float(f) < v else float(f)


def block_bounds(sp, perm, nblk, size=16, return_forward=False):
    """rt_api.cpp build_mfma's bounds: per `size` walk positions (half a
    32-sphere block) the box centre C (f32) of the members, L = max(|c - C|
    (1 + 2^-40) + r (1 + 2^-18)), R^2 = (1 + 2^-5 + 2^-10) L^2 (1 + 2^-40) + 2^-60 and
    S'_B = R^2 - (1 - m - mu' - muB)|C|^2 rounded up (+inf beyond 2^15, -inf
    for an empty one); nblk counts bounds."""
    c_all = sp["center"].astype(F).astype(D)
    r2_all = (sp["radius"] * sp["radius"]).astype(F).astype(D)
    # chunk-level rows (size 512) split the proof's slack with t = 2^-7: R^2 =
    # (1 + 2^-7 + 2^-9) L^2 and 4 muB (their K 31 = 4, rows_of)
    chunk = size == 512
    kB = 1.0 - M - MU - (4 * MUB if chunk else MUB)
    fac = (1 + 2.0 ** -7 + 2.0 ** -9) if chunk else (1 + 2.0 ** -5 + 2.0 ** -10)
    C = np.zeros((nblk, 3))
    S = np.full(nblk, -np.inf)
    Lf = np.zeros(nblk)  # the forward rows' L' (0 for an empty bound)
    for b in range(nblk):
        idx = perm[size * b:size * b + size]
        idx = idx[idx >= 0]
        if len(idx) == 0:
            continue
        c = c_all[idx]
        C[b] = ((c.min(0) + c.max(0)) * 0.5).astype(F).astype(D)
        Lm = np.max(np.linalg.norm(c - C[b], axis=1) * (1 + 2.0 ** -40) + np.sqrt(r2_all[idx]) * (1 + 2.0 ** -18))
        R2 = fac * Lm * Lm * (1 + 2.0 ** -40) + 2.0 ** -60
        SB = round_up_f32((R2 - kB * (C[b] ** 2).sum()) * (1 + 2.0 ** -40) + 2.0 ** -60)
        S[b] = SB if abs(SB) <= 2.0 ** 15 else np.inf
        lf = (1 + 2.0 ** -12) * Lm + 2.0 ** -8 * np.abs(C[b]).sum() + 2.0 ** -14
        if np.isinf(S[b]) or not lf <= 2.0 ** 15:
            Lf[b] = np.inf
        else:  # rounded up to f16
            h = np.float16(lf)
            Lf[b] = float(np.nextafter(h, np.float16(np.inf))) if float(h) < lf else float(h)
    if return_forward:
        return C, S, Lf
    return C, S


def forward_rows(C, Lf):
    """rt_api.cpp build_mfma's forward rows (K 0..7 of v_mfma_f32_32x32x8_f16,
    zero-padded to 32): C hi x3, 1, L' (f16, rounded up)."""
    n = len(C)
    cols = [np.zeros(n)] * 32
    for a in range(3):
        cols[a] = C[:, a].astype(H16).astype(D)
    cols[3] = np.ones(n)
    cols[4] = Lf.astype(H16).astype(D)
    assert np.all(cols[4] >= Lf)
    return np.stack(cols, 1).astype(F)


def forward_columns(rays):
    """The kernel's forward column (intersect_world_mfma): dn = -e hi x3, c0 =
    fma(2^-9, |o|_1, -k1) hi, 1 (zero-padded to 32)."""
    o, e, k1, _, _ = ray_constants(rays)
    with np.errstate(invalid="ignore", over="ignore"):
        o1 = ((np.abs(o[:, 0]) + np.abs(o[:, 1])).astype(F) + np.abs(o[:, 2])).astype(F)
        c0 = fma32(F(2.0 ** -9), o1, -k1)
    n = len(rays)
    cols = [np.zeros(n, F)] * 32
    for a in range(3):
        cols[a] = split(-e[:, a])[0]
    cols[3] = split(c0)[0]
    cols[4] = np.ones(n, F)
    return np.stack(cols, 1)


BOUND_CASES = [(n, 16) for n in sorted(SCENES)] + [("spheres10k", 512)]


@pytest.mark.parametrize("name,size", BOUND_CASES,
                         ids=[f"{n}-{s}" for n, s in BOUND_CASES])
def test_block_bounds_are_conservative(name, size):
    """The walk skips a 32-sphere block for a half-wave when no ray of the
    half has V_B < 0 on either of the block's two half-block bound rows (rt_dev_intersect.h "Block
    bounds"): every exact hit of a member sphere must have V_B < 0, in every
    summation order, on the adversarial ray sets (rays in the walk's domain:
    mfma_wave_ok and |d|^2 in [2^-100, 2^100]). size 512: the chunk-level
    bounds of a list of 2..32 bound chunks ("Chunk bounds": 10,000 spheres,
    20 chunks of 512 walk positions), built the same way."""
    from bevy_raytrace_amd import abi
    full = SCENES[name]()
    sq = qscale(full)
    perm = abi.cull_layout(full)[0]
    nblk = -(-(len(perm) - 8) // size)  # bounds over whole clusters (+ one pad group)
    C, S = block_bounds(full, perm, nblk, size=size)
    A = rows_of(C, S, sq, bound=True, k31=4.0 if size == 512 else 1.0)
    sp = full[:SUBSET.get(name, len(full))]
    rays = _rays(sp, "blk" + name, 6_000 if len(sp) < 1000 else 2_000)
    d = rays[:, 3:].astype(F)
    dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    rays = rays[(dd >= 2.0 ** -100) & (dd <= 2.0 ** 100)]
    Bc, _ = ray_columns(rays, sq, 2.0 ** (sq - 20))
    hits = exact_hits(sp, rays)  # (rays, spheres of the subset)
    pos = np.full(len(full), -1)
    pos[perm[perm >= 0]] = np.nonzero(perm >= 0)[0]
    blk = pos[:len(sp)] // size  # the bound of each checked sphere
    assert hits.sum() > 500
    for order in ORDERS:
        with np.errstate(invalid="ignore", over="ignore"):
            passed = mfma_sum(A, Bc, order) < 0  # (rays, blocks)
        lost = hits & ~passed[:, blk]
        assert not lost.any(), (f"{order}: {int(lost.sum())} exact hits in skipped blocks, e.g. "
                                f"{np.argwhere(lost)[0].tolist()}")


@pytest.mark.parametrize("name,size", BOUND_CASES,
                         ids=[f"{n}-{s}" for n, s in BOUND_CASES])
def test_forward_bounds_are_conservative(name, size):
    """The bound tile passes a (ray, half-block bound) pair only when its line
    row passes (V_B < 0) AND its forward row does (U >= +0: the bound is not
    wholly behind the ray's origin, rt_dev_intersect.h "Forward bounds"): every
    exact hit of a member sphere must pass both, in every summation order
    (size 512: the chunk-level bounds)."""
    from bevy_raytrace_amd import abi
    full = SCENES[name]()
    sq = qscale(full)
    perm = abi.cull_layout(full)[0]
    nblk = -(-(len(perm) - 8) // size)
    C, S, Lf = block_bounds(full, perm, nblk, size=size, return_forward=True)
    A = rows_of(C, S, sq, bound=True, k31=4.0 if size == 512 else 1.0)
    Af = forward_rows(C, Lf)
    sp = full[:SUBSET.get(name, len(full))]
    rays = _rays(sp, "fwd" + name, 6_000 if len(sp) < 1000 else 2_000)
    d = rays[:, 3:].astype(F)
    dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    rays = rays[(dd >= 2.0 ** -100) & (dd <= 2.0 ** 100)]
    Bc, _ = ray_columns(rays, sq, 2.0 ** (sq - 20))
    Uc = forward_columns(rays)
    hits = exact_hits(sp, rays)
    pos = np.full(len(full), -1)
    pos[perm[perm >= 0]] = np.nonzero(perm >= 0)[0]
    blk = pos[:len(sp)] // size
    assert hits.sum() > 500
    cut = 0
    for order in ORDERS:
        with np.errstate(invalid="ignore", over="ignore"):
            line = mfma_sum(A, Bc, order) < 0
            U = mfma_sum(Af, Uc, order)
        assert not np.isnan(U).any()
        passed = line & ~np.signbit(U)
        cut = max(cut, int((line & ~passed).sum()))
        lost = hits & ~passed[:, blk]
        assert not lost.any(), (f"{order}: {int(lost.sum())} exact hits in skipped bounds, e.g. "
                                f"{np.argwhere(lost)[0].tolist()}")
    assert cut > 0  # the forward rows do cut pairs the line rows pass
