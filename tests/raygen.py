"""Adversarial ray sets for intersection parity tests (test support, numpy only).

Grazing rays pass at distance r(1 + k eps) from sphere centres (the filter's
decision boundary), surface rays start on / just off a sphere (the t ~ EPSILON
boundary and self-hits, intersect.wgsl:110), plus far origins, rays from
inside spheres (some exactly at the centre), unnormalised and degenerate
directions."""
from __future__ import annotations

import numpy as np

F = np.float32


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def adversarial_rays(spheres: np.ndarray, n: int, seed: int = 0) -> np.ndarray:
    rng = np.random.default_rng(seed)
    c = spheres["center"].astype(np.float64)
    r = spheres["radius"].astype(np.float64)
    lo, hi = c.min(0) - 5, c.max(0) + 5
    lo = np.maximum(lo, -60)
    hi = np.minimum(hi, 60)
    k = n // 8
    out = []
    # 1 random origins in the scene box, random directions
    o = rng.uniform(lo, hi, (k, 3))
    d = _unit(rng.normal(size=(k, 3)))
    out.append(np.hstack([o, d]))
    # 2 grazing: distance r(1 + e) from a random sphere's centre, e ~ +-1e-6
    i = rng.integers(0, len(r), k)
    d = _unit(rng.normal(size=(k, 3)))
    perp = _unit(np.cross(d, rng.normal(size=(k, 3))))
    e = rng.choice([-1, 1], k) * 10.0 ** rng.uniform(-8, -4, k)
    p = c[i] + perp * (r[i] * (1 + e))[:, None]
    o = p - d * rng.uniform(0.5, 30, k)[:, None]
    out.append(np.hstack([o, d]))
    # 3 surface origins (+ tiny offsets), random directions
    i = rng.integers(0, len(r), k)
    nrm = _unit(rng.normal(size=(k, 3)))
    off = rng.choice([0.0, 0.001, -0.001, 1e-6], k)
    o = c[i] + nrm * (np.abs(r[i]) + off)[:, None]
    d = _unit(rng.normal(size=(k, 3)))
    out.append(np.hstack([o, d]))
    # 4 reflected-like: surface origin, direction near the tangent plane
    i = rng.integers(0, len(r), k)
    nrm = _unit(rng.normal(size=(k, 3)))
    o = c[i] + nrm * np.abs(r[i])[:, None]
    t = _unit(np.cross(nrm, rng.normal(size=(k, 3))))
    d = _unit(t + nrm * rng.uniform(-1e-3, 1e-3, k)[:, None])
    out.append(np.hstack([o, d]))
    # 5 far origins looking at the scene
    # (1e10 > 2^32: those lanes' waves take the IEEE exact test, rt_dev_intersect.h ray_fast)
    o = rng.normal(size=(k, 3)) * rng.choice([1e3, 1e4, 1e5, 1e10], k)[:, None]
    tgt = rng.uniform(lo, hi, (k, 3))
    d = _unit(tgt - o)
    out.append(np.hstack([o, d]))
    # 6 inside spheres
    i = rng.integers(0, len(r), k)
    frac = rng.uniform(0, 0.999, k)
    frac[rng.random(k) < 0.1] = 0.0  # exactly at the centre: |oc|^2 = 0
    o = c[i] + _unit(rng.normal(size=(k, 3))) * (np.abs(r[i]) * frac)[:, None]
    d = _unit(rng.normal(size=(k, 3)))
    out.append(np.hstack([o, d]))
    # 7 unnormalised directions (|d| 1e-3 .. 1e3)
    o = rng.uniform(lo, hi, (k, 3))
    d = rng.normal(size=(k, 3)) * (10.0 ** rng.uniform(-3, 3, k))[:, None]
    out.append(np.hstack([o, d]))
    # 8 camera rays with degenerate / special directions
    m = n - 7 * k
    o = np.tile([13.0, 2.0, 3.0], (m, 1))
    d = _unit(rng.normal(size=(m, 3)))
    special = rng.integers(0, 5, m)
    d[special == 0] = [0.0, 0.0, 0.0]
    d[special == 1] = [np.nan, 0.0, 1.0]
    d[special == 2] = [np.inf, 1.0, 0.0]
    out.append(np.hstack([o, d]))
    return np.vstack(out).astype(F)


def half_blocks(spheres, perm):
    """The matrix-core walk's 16-sphere half-blocks (rt_api.cpp build_mfma:
    walk position p of spatial order `perm`, half-block p // 16) with the
    bound each gets on the host: centre C = the midpoint of the members'
    centre box, rounded to f32, L = max |C - c_i| + r_i. Returns a list of
    (member indices, C, L) for the non-empty half-blocks."""
    c = spheres["center"].astype(np.float64)
    r = np.abs(spheres["radius"].astype(np.float64))
    out = []
    for h in range(len(perm) // 16):
        idx = np.asarray(perm[16 * h:16 * h + 16])
        idx = idx[idx >= 0]
        if len(idx) == 0:
            continue
        C = ((c[idx].min(0) + c[idx].max(0)) * 0.5).astype(F).astype(np.float64)
        L = float(np.max(np.linalg.norm(c[idx] - C, axis=1) + r[idx]))
        out.append((idx, C, L))
    return out


def coherent_halves(spheres, perm, n_halves, seed=0, o_max=None):
    """Rays for the block-bound tiles' decision boundary: `n_halves` groups of
    32 rays (one 32-lane half of a wave each, in order), every group aimed at
    ONE half-block, so its rays' lines pass near few blocks and the half skips
    the rest. For each group a half-block and its extremal member i (the
    member whose far side is the bound's radius L from C) are picked; the
    point P of sphere i farthest from C lies at distance L from C, so rays
    tangent to sphere i at P (passing r_i (1 +- 1e-8..1e-4) from its centre)
    are the rays whose lines pass at the bound's own radius. Kinds, cycling:
      0  one such ray, replicated 32 times;
      1  a fan of 32 tangent rays at P (directions around the tangent plane,
         origins 0.5..30 back along each ray);
      2  32 rays from one origin grazing one (random) member of the block;
      3  as 1, with origins at |o| in [0.965, 0.9995] x o_max (the largest
         origin the matrix-core walk takes, |o|^2 <= 2^15: mfma_wave_ok),
         where the threshold T0 and the bound margin muB |o|^2 are largest.
    Every origin stays within 0.9995 o_max, so every wave takes the
    matrix-core walk.
    Returns (n_halves * 32, 6) float32."""
    rng = np.random.default_rng(seed)
    c = spheres["center"].astype(np.float64)
    r = np.abs(spheres["radius"].astype(np.float64))
    hb = [h for h in half_blocks(spheres, perm) if h[2] < 50.0]  # not the ground's block
    o_max = o_max if o_max is not None else np.sqrt(2.0 ** 15)
    lim = o_max * 0.9995
    out = []
    for w in range(n_halves):
        kind = w % 4
        idx, C, L = hb[rng.integers(len(hb))]
        i = idx[np.argmax(np.linalg.norm(c[idx] - C, axis=1) + r[idx])]
        u = c[i] - C
        u = _unit(u) if np.linalg.norm(u) > 0 else _unit(rng.normal(size=3))
        if kind == 2:  # one origin, 32 rays grazing one member
            j = idx[rng.integers(len(idx))]
            o0 = c[j] + _unit(rng.normal(size=3)) * (r[j] + rng.uniform(5, 40))
            while np.linalg.norm(o0) > lim:  # pulled in towards the sphere (|o| <= o_max)
                o0 = c[j] + (o0 - c[j]) * 0.7
            a = _unit(np.cross(c[j] - o0, rng.normal(size=(32, 3))))
            e = rng.choice([-1, 1], 32) * 10.0 ** rng.uniform(-8, -4, 32)
            # aim at a point beside the centre at r (1 + e) perpendicular to the sight line
            tgt = c[j] + a * (r[j] * (1 + e))[:, None]
            d = _unit(tgt - o0)
            o = np.tile(o0, (32, 1))
        else:
            m = 1 if kind == 0 else 32
            t = _unit(np.cross(u, rng.normal(size=(m, 3))))  # tangent directions at P
            t = _unit(t + u * rng.uniform(-1e-3, 1e-3, (m, 1)))
            e = rng.choice([-1, 1], m) * 10.0 ** rng.uniform(-8, -4, m)
            p = c[i] + u * (r[i] * (1 + e))[:, None]  # the line's closest point to c_i
            if kind == 3:
                # s > 0 with |p - t s| = target: s = t.p + sqrt((t.p)^2 - |p|^2 + target^2)
                target = o_max * rng.uniform(0.965, 0.9995, m)
                tp = (t * p).sum(1)
                disc = tp * tp - (p * p).sum(1) + target * target
                s = np.where(disc > 0, tp + np.sqrt(np.maximum(disc, 0)), 1e-3)
            else:
                s = rng.uniform(0.5, 30, m)
                # origins past o_max moved in along the ray (to |o| in [0.9, 0.999] lim)
                far = np.linalg.norm(p - t * s[:, None], axis=1) > lim
                if far.any():
                    target = lim * rng.uniform(0.9, 0.999, m)
                    tp = (t * p).sum(1)
                    disc = tp * tp - (p * p).sum(1) + target * target
                    s_in = tp - np.sqrt(np.maximum(disc, 0))  # the root nearer the tangent point
                    s_in = np.where(s_in > 1e-3, s_in, tp + np.sqrt(np.maximum(disc, 0)))
                    s = np.where(far & (disc > 0) & (s_in > 1e-3), s_in, np.where(far, 1e-3, s))
            o = p - t * s[:, None]
            d = t
            if m == 1:
                o, d = np.tile(o, (32, 1)), np.tile(d, (32, 1))
        out.append(np.hstack([o, d]))
    return np.vstack(out).astype(F)
