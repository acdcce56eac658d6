"""Independent numpy restatement of the reference WGSL path.

TEST INFRASTRUCTURE ONLY: imported by tests/ to cross-check the C oracle
(oracle/rt_oracle.c). Never imported by the product package.

Written separately from the C oracle, vectorised over pixels instead of scalar
per path, following the same fixed op forms (see rt_oracle.c header). numpy
float32 arithmetic is one IEEE round-to-nearest operation per ufunc call
(no FMA), so the two restatements must agree bit for bit.

Reference lines: generate.wgsl:66-129, intersect.wgsl:94-163,
shade.wgsl:105-258, collect.wgsl:99-125, src/ray_trace_node.rs:195-224.
"""
from __future__ import annotations

import math

import numpy as np

F = np.float32
VERY_FAR = F(1e20)
EPSILON = F(0.001)
SAMPLE_BLOCK = 8


def hash3(n):
    """shade.wgsl:105-116 on a uint32 array -> (..., 3) float32."""
    n = np.asarray(n, dtype=np.uint32)
    with np.errstate(over="ignore"):
        n = (n << np.uint32(13)) ^ n
        n = n * (n * n * np.uint32(15731) + np.uint32(789221)) + np.uint32(1376312589)
        k = np.stack([n * n, n * (n * np.uint32(16807)), n * (n * np.uint32(48271))], -1)
    m = (k & np.uint32(0x7FFFFFFF)).astype(np.float32)
    return m / F(2147483648.0)


def _dot(a, b):
    r = a[..., 0] * b[..., 0]
    r = r + a[..., 1] * b[..., 1]
    return r + a[..., 2] * b[..., 2]


def _normalize(v):
    l = np.sqrt(_dot(v, v))
    return v / l[..., None]


def tan_half(fov):
    return F(math.tan(float(F(fov) / F(2.0))))


RT_FLAG_JITTER, RT_FLAG_THIN_LENS = 0x2, 0x4
JITTER_MUL, LENS_MUL = np.uint32(0x9E3779B1), np.uint32(0x85EBCA77)
PI2 = F(F(2.0) * F(3.14159265358979))


def sincos(theta):
    """rt_sincos of the opt-in thin-lens sampling (include/rt_hip.h): the same
    f32 op sequence as the C oracle and the kernel, written independently."""
    theta = np.asarray(theta, dtype=np.float32)
    h = float.fromhex
    q = np.rint(theta * F(h("0x1.45f306p-1")))
    r = theta - q * F(h("0x1.92p+0"))
    r = r - q * F(h("0x1.fb5444p-12"))
    r = r - q * F(h("0x1.68cp-39"))
    r2 = r * r
    sr = r + r * (r2 * (F(h("-0x1.555556p-3")) + r2 * (F(h("0x1.111112p-7")) + r2 * (
        F(h("-0x1.a01a02p-13")) + r2 * F(h("0x1.71de3ap-19"))))))
    cr = F(1.0) + r2 * (F(-0.5) + r2 * (F(h("0x1.555556p-5")) + r2 * (F(h("-0x1.6c16c2p-10")) + r2 * (
        F(h("0x1.a01a02p-16")) + r2 * F(h("-0x1.27e4fcp-22"))))))
    quad = q.astype(np.int64) & 3
    s = np.select([quad == 0, quad == 1, quad == 2], [sr, cr, -sr], -cr).astype(np.float32)
    c = np.select([quad == 0, quad == 1, quad == 2], [cr, -sr, -cr], sr).astype(np.float32)
    return s, c


def camera_consts(cam_floats, width, height, flags=0):
    """cam_floats: the 32 f32 of the 128-B CameraGPU block."""
    c = np.asarray(cam_floats, dtype=np.float32)
    T = c[0:16]
    fov, ipd, lfl, fstop = c[19], c[23], c[27], c[31]
    return dict(
        T=T,
        tan=tan_half(fov),
        fp=F((ipd * lfl) / (ipd - lfl)),
        aspect=F(width),
        hw=F(F(width) / F(2.0)),
        hh=F(F(height) / F(2.0)),
        coc=F(lfl / (F(2.0) * fstop)),
        flags=flags, W=width, H=height,
    )


def primary_rays(cc, xs, ys, frame=0):
    """generate.wgsl:66-129 for integer pixel arrays -> origins, dirs (N,3).
    `frame` (the seed frame) only matters with the opt-in jitter / lens flags."""
    px = xs.astype(np.float32)
    py = ys.astype(np.float32)
    flags = cc.get("flags", 0)
    if flags & (RT_FLAG_JITTER | RT_FLAG_THIN_LENS):
        with np.errstate(over="ignore"):
            idx = (xs.astype(np.uint32) + np.uint32(cc["W"]) * ys.astype(np.uint32)
                   + np.uint32(cc["W"] * cc["H"] % (1 << 32)) * np.uint32(frame))
    if flags & RT_FLAG_JITTER:
        with np.errstate(over="ignore"):
            j = hash3(idx * JITTER_MUL)
        px = px + (j[:, 0] - F(0.5))
        py = py + (j[:, 1] - F(0.5))
    dx = ((px - cc["hw"]) * cc["tan"]) / cc["aspect"]
    dy = ((-py + cc["hh"]) * cc["tan"]) / cc["aspect"]
    d = np.stack([dx, dy, np.full_like(dx, F(-1.0))], -1)
    d = _normalize(d)
    denom = _dot(d, np.array([0.0, 0.0, -1.0], dtype=np.float32))
    fp = d * (cc["fp"] / denom)[..., None]
    origin = np.zeros_like(d)
    if flags & RT_FLAG_THIN_LENS:
        with np.errstate(over="ignore"):
            l = hash3(idx * LENS_MUL)
        theta = PI2 * l[:, 0] + PI2
        sr = np.sqrt(l[:, 1])
        sn, cs = sincos(theta)
        a, b = (cs * sr) * cc["coc"], (sn * sr) * cc["coc"]
        origin = np.stack([F(1.0) * a + F(0.0) * b, F(0.0) * a + F(1.0) * b,
                           F(0.0) * a + F(0.0) * b], -1)
    d = _normalize(fp - origin)
    T = cc["T"]
    o = origin + T[12:15]
    td = np.empty_like(d)
    for r in range(3):
        td[:, r] = ((T[0 + r] * d[:, 0] + T[4 + r] * d[:, 1]) + T[8 + r] * d[:, 2]) + T[12 + r] * F(0.0)
    return o, td


def sky(d):
    u = _normalize(d)
    t = F(0.5) * u[..., 1] + F(1.0)
    omt = (F(1.0) - t) * F(1.0)
    return np.stack([omt + t * F(0.5), omt + t * F(0.7), omt + t * F(1.0)], -1)


def intersect(spheres, o, d):
    """Closest hit, intersect.wgsl:94-143. spheres: (N,4) center+radius."""
    n = o.shape[0]
    l = np.sqrt(_dot(d, d))
    a = l * l
    best_t = np.full(n, VERY_FAR, dtype=np.float32)
    best = np.full(n, -1, dtype=np.int64)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        for i in range(spheres.shape[0]):
            c = spheres[i, 0:3]
            r = spheres[i, 3]
            oc = o - c
            hb = _dot(oc, d)
            lo = np.sqrt(_dot(oc, oc))
            cc = lo * lo - r * r
            dis = hb * hb - a * cc
            ok = ~(dis < F(0.0))
            sq = np.sqrt(np.where(ok, dis, F(0.0)))
            root = (-hb - sq) / a
            bad = (root < EPSILON) | (VERY_FAR < root)
            root2 = (-hb + sq) / a
            bad2 = (root2 < EPSILON) | (VERY_FAR < root2)
            root = np.where(bad, root2, root)
            ok &= ~(bad & bad2)
            upd = ok & (root < best_t)
            best_t = np.where(upd, root, best_t)
            best = np.where(upd, i, best)
    return best, best_t


def trace(spheres, mats, cc, width, height, xs, ys, frame, D):
    """One sample (frame) for pixel arrays -> colours (N,3), segment count."""
    o, d = primary_rays(cc, xs, ys, frame)
    n = o.shape[0]
    color = np.ones((n, 3), dtype=np.float32)
    with np.errstate(over="ignore"):
        seed_in = (xs.astype(np.uint32) + np.uint32(width) * ys.astype(np.uint32)
                   + np.uint32(width * height % (1 << 32)) * np.uint32(frame))
    seed = hash3(seed_in)
    nseed = _normalize(seed)
    alive = np.ones(n, dtype=bool)
    segs = 0
    for b in range(D):
        idx = np.nonzero(alive)[0]
        if idx.size == 0:
            break
        segs += idx.size
        oo, dd = o[idx], d[idx]
        best, t = intersect(spheres, oo, dd)
        miss = best < 0
        mi = idx[miss]
        color[mi] = color[mi] * sky(dd[miss])
        alive[mi] = False
        hit = ~miss
        hi = idx[hit]
        if b == D - 1:
            color[hi] = F(0.0)
            alive[hi] = False
            break
        if hi.size == 0:
            continue
        ho, hd, ht, hs = oo[hit], dd[hit], t[hit], best[hit]
        cen = spheres[hs, 0:3]
        rad = spheres[hs, 3]
        pos = ho + hd * ht[:, None]
        nrm = _normalize((pos - cen) / rad[:, None])
        front = ~(_dot(hd, nrm) > F(0.0))
        nrm = np.where(front[:, None], nrm, -nrm)
        mid = mats["index"][hs]
        refl = mats["refl"][mid]
        mcol = mats["color"][mid]
        new_o = np.empty_like(ho)
        new_d = np.empty_like(hd)
        # Lambertian, shade.wgsl:118-130
        L = refl == 0
        if L.any():
            dest = (pos[L] + nrm[L]) + nseed[hi[L]]
            new_d[L] = _normalize(dest - pos[L])
            new_o[L] = pos[L]
        # Metallic, shade.wgsl:136-146
        M = refl == 1
        if M.any():
            v, nm = hd[M], nrm[M]
            refl_v = v - nm * (F(2.0) * _dot(v, nm))[:, None]
            refl_v = _normalize(refl_v)
            noise = nseed[hi[M]] * mats["fuzz"][mid[M]][:, None]
            new_d[M] = _normalize(refl_v + noise)
            new_o[M] = pos[M] + nm * EPSILON
        # Dielectric, shade.wgsl:163-187
        G = refl == 2
        if G.any():
            v, nm, ff = hd[G], nrm[G], front[G]
            ior = mats["ior"][mid[G]]
            ratio = np.where(ff, F(1.0) / ior, ior)
            u = _normalize(v)
            cos_t = np.minimum(_dot(-u, nm), F(1.0))
            sin_t = np.sqrt(F(1.0) - cos_t * cos_t)
            cannot = ratio * sin_t > F(1.0)
            r0 = (F(1.0) - ratio) / (F(1.0) + ratio)
            r0 = r0 * r0
            x = F(1.0) - cos_t
            x2 = x * x
            p5 = (x2 * x2) * x
            refl_p = r0 + (F(1.0) - r0) * p5
            do_refl = cannot | (refl_p > seed[hi[G], 0])
            rv = v - nm * (F(2.0) * _dot(v, nm))[:, None]
            # refract(u, n, ratio), shade.wgsl:148-154
            ct = np.minimum(_dot(-u, nm), F(1.0))
            perp = (u + nm * ct[:, None]) * ratio[:, None]
            lp = np.sqrt(_dot(perp, perp))
            with np.errstate(invalid="ignore"):
                par = -np.sqrt(np.abs(F(1.0) - (lp * lp)))
            rr = _normalize(perp + nm * par[:, None])
            new_d[G] = np.where(do_refl[:, None], rv, rr)
            new_o[G] = pos[G] + nm * EPSILON
        color[hi] = color[hi] * np.where(G[:, None], F(1.0), mcol)
        o[hi] = new_o
        d[hi] = new_d
    return color, segs


def render(cam_floats, spheres_arr, mats_arr, width, height, spp, D, frame0=0, rows=None, flags=0):
    """Render rows (default all) -> (len(rows), W, 4) float32, segments.

    spheres_arr: structured array / (N,8) float32 view of the 32-B SphereGPU
    records; mats_arr: (M,8) view of the 32-B MaterialGPU records.
    """
    sp = np.asarray(spheres_arr)
    sph = sp.view(np.float32).reshape(-1, 8)[:, 0:4].copy() if sp.size else np.zeros((0, 4), np.float32)
    sph_mat = sp.view(np.uint32).reshape(-1, 8)[:, 4].astype(np.int64) if sp.size else np.zeros(0, np.int64)
    mt = np.asarray(mats_arr)
    mf = mt.view(np.float32).reshape(-1, 8) if mt.size else np.zeros((0, 8), np.float32)
    mi = mt.view(np.int32).reshape(-1, 8) if mt.size else np.zeros((0, 8), np.int32)
    mats = dict(index=sph_mat, color=mf[:, 0:3].copy(), refl=mi[:, 4].copy(), fuzz=mf[:, 5].copy(),
                ior=mf[:, 6].copy())
    cc = camera_consts(cam_floats, width, height, flags)
    rows = list(range(height)) if rows is None else list(rows)
    ys = np.repeat(np.asarray(rows, dtype=np.int64), width)
    xs = np.tile(np.arange(width, dtype=np.int64), len(rows))
    acc = np.zeros((xs.size, 3), dtype=np.float32)
    segs = 0
    for s0 in range(0, spp, SAMPLE_BLOCK):
        bs = np.zeros((xs.size, 3), dtype=np.float32)
        for s in range(s0, min(spp, s0 + SAMPLE_BLOCK)):
            c, sg = trace(sph, mats, cc, width, height, xs, ys, frame0 + s, D)
            segs += sg
            bs = bs + c
        acc = acc + bs
    out = np.ones((xs.size, 4), dtype=np.float32)
    out[:, 0:3] = acc / F(spp)
    return out.reshape(len(rows), width, 4), segs
