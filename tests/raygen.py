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
