"""Research probe (CPU, uses the numpy oracle as a ray source): how many
(32-sphere block, 32-ray half-wave) tiles of the matrix-core walk could a
per-block bounding-sphere test skip at the headline workload?

Rays: the headline frame's paths (RTIOW, 1920x1080, depth 16) for pixel
pairs (P, P+1) at random samples, recorded per segment. A half-wave holds
pixel-major lanes as the render kernel's queue deals them (20 lanes of one
pixel's frames, 12 of the next), each lane at a uniformly random segment of
a random sample's path. Blocks: the sphere list in list order (the current
walk) or in 3-D Morton order of the centres, 32 per block, bound = centre of
the block's box and the radius covering its spheres. A tile is skippable when
no ray of the half passes within the bound (t >= 0).

usage: python tools/sim_block_cull.py [pairs] [samples]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bevy_raytrace_amd import scene  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
import oracle.rt_oracle_np as O  # noqa: E402

W, H, D = 1920, 1080, 16
pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 300
nsamp = int(sys.argv[2]) if len(sys.argv) > 2 else 24
rng = np.random.default_rng(7)

sc = scene.rtiow_final_scene()
sp = np.asarray(sc.objects_gpu())
sph = sp.view(np.float32).reshape(-1, 8)[:, 0:4].copy()
sph_mat = sp.view(np.uint32).reshape(-1, 8)[:, 4].astype(np.int64)
mt = np.asarray(sc.materials_gpu())
mf = mt.view(np.float32).reshape(-1, 8)
mi = mt.view(np.int32).reshape(-1, 8)
mats = dict(index=sph_mat, color=mf[:, 0:3].copy(), refl=mi[:, 4].copy(), fuzz=mf[:, 5].copy(),
            ior=mf[:, 6].copy())
cc = O.camera_consts(np.ascontiguousarray(default_camera_block()).view(np.float32).reshape(-1)[:32], W, H, 0)

# record every intersect call's rays and results
rec = []
_orig = O.intersect


def _rec(spheres, o, d):
    best, t = _orig(spheres, o, d)
    rec.append((o.copy(), d.copy(), best.copy()))
    return best, t


O.intersect = _rec
px = rng.integers(0, W - 1, pairs)
py = rng.integers(0, H, pairs)
xs = np.concatenate([px, px + 1]).astype(np.int64)
ys = np.concatenate([py, py]).astype(np.int64)
n = xs.size
samples = rng.integers(0, 64 * 20, nsamp)
paths = [[None] * nsamp for _ in range(n)]  # paths[pixel][sample] = (segs, 6)
for si, s in enumerate(samples):
    rec.clear()
    O.trace(sph, mats, cc, W, H, xs, ys, int(s), D)
    alive = np.arange(n)
    segs = [[] for _ in range(n)]
    for o, d, best in rec:
        for k, p in enumerate(alive):
            segs[p].append(np.concatenate([o[k], d[k]]))
        alive = alive[best >= 0]
    for p in range(n):
        paths[p][si] = np.array(segs[p], dtype=np.float64)
    print(f"sample {si + 1}/{nsamp}", file=sys.stderr, flush=True)
O.intersect = _orig


def morton_order(c):
    q = ((c - c.min(0)) / (np.ptp(c, 0) + 1e-9) * 1023).astype(np.int64)

    def spread(v):
        out = np.zeros_like(v)
        for b in range(10):
            out |= ((v >> b) & 1) << (3 * b)
        return out
    return np.argsort(spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2), kind="stable")


def bounds(order):
    out = []
    for b in range(0, len(order), 32):
        idx = order[b:b + 32]
        idx = idx[idx >= 0]
        c, r = sph[idx, :3].astype(np.float64), np.abs(sph[idx, 3]).astype(np.float64)
        C = (c.min(0) + c.max(0)) / 2
        R = np.max(np.linalg.norm(c - C, axis=1) + r)
        out.append((C, R))
    return out


def passes(C, R, rays):
    o, d = rays[:, :3], rays[:, 3:]
    dn = d / np.linalg.norm(d, axis=1, keepdims=True)
    oc = C - o
    tc = np.einsum("ij,ij->i", oc, dn)
    d2 = np.einsum("ij,ij->i", oc, oc) - np.maximum(tc, 0) ** 2
    if MARGIN:  # the bound row's margins: R^2 (1 + 2^-3) + muB (|o|^2 + |C|^2)
        R2 = R * R * (1 + 2.0 ** -3) + 2.0 ** -7 * (np.einsum("ij,ij->i", o, o) + C @ C)
        R = np.sqrt(R2)
    inside = np.einsum("ij,ij->i", oc, oc) <= R * R
    if LINE:  # the filter's test: the infinite line, either direction
        return (np.einsum("ij,ij->i", oc, oc) - tc ** 2) <= R * R * (1 + 1e-6)
    return inside | ((tc >= 0) & (d2 <= R * R * (1 + 1e-6)))


allsegs = [np.concatenate(paths[q]) for q in range(n)]
orders = {"list": np.arange(len(sph)), "morton": morton_order(sph[:, :3].astype(np.float64))}
# the big spheres (r > 0.5) in blocks of their own at the front, rest Morton
big = np.nonzero(np.abs(sph[:, 3]) > 0.5)[0]
small = np.nonzero(~(np.abs(sph[:, 3]) > 0.5))[0]
orders["big_first+morton"] = np.concatenate([big, small[morton_order(sph[small, :3].astype(np.float64))]])
# the culled list's layout (rt_api.cpp cull_layout): spheres above 4x the
# median radius first, padded to a whole block (pads never pass), the rest in
# Morton order
orders["big_block+morton"] = np.concatenate([big, -np.ones((-len(big)) % 32, np.int64),
                                             small[morton_order(sph[small, :3].astype(np.float64))]])


def kd_order(idx, c):
    """Recursive split along the longest axis of the box, at a multiple of
    64 / 32 / 8 positions near the median (clusters, blocks and groups
    aligned): compact blocks."""
    n = len(idx)
    if n <= 8:
        return list(idx)
    pts = c[idx]
    ax = int(np.argmax(pts.max(0) - pts.min(0)))
    srt = idx[np.argsort(pts[:, ax], kind="stable")]
    unit = 64 if n > 64 else (32 if n > 32 else 8)
    cut = max(unit, int(round(n / 2 / unit)) * unit)
    if cut >= n:
        cut = (n // 2 + 7) // 8 * 8
    return kd_order(srt[:cut], c) + kd_order(srt[cut:], c)


orders["big_block+kd"] = np.concatenate([big, -np.ones((-len(big)) % 32, np.int64),
                                         np.array(kd_order(small, sph[:, :3].astype(np.float64)))])
trials = 4000
MIX = int(os.environ.get("MIX", "0"))
MARGIN = os.environ.get("MARGIN", "0") == "1"
WEIGHT = os.environ.get("WEIGHT", "1") == "1"  # pairs weighted by their iterations
LINE = os.environ.get("LINE", "0") == "1"  # line test (what the bound tile computes)
for name, order in orders.items():
    bnd = bounds(order)
    skip = np.zeros(len(bnd))
    skip_seg1 = np.zeros(len(bnd))
    # a half-wave spends iterations in proportion to its pixels' path
    # lengths: draw pairs weighted by their mean segments per path
    seg_w = np.array([np.mean([len(paths[q][k]) + len(paths[q + pairs][k]) for k in range(nsamp)])
                      for q in range(pairs)])
    seg_w = seg_w / seg_w.sum()
    for t in range(trials):
        p = rng.choice(pairs, p=seg_w) if WEIGHT else rng.integers(0, pairs)
        if MIX:  # lanes from MIX random pixels (the queue's chunk mixing)
            lanes = list(rng.integers(0, 2 * pairs, MIX).repeat(32 // MIX))
        else:
            lanes = [p] * 20 + [p + pairs] * 12
        rays = []
        for q in lanes:
            # a lane's state at a random iteration: uniform over ALL segments
            # of the pixel's paths (long paths hold the lane longer)
            allseg = allsegs[q]
            rays.append(allseg[rng.integers(0, len(allseg))])
        rays = np.array(rays)
        for b, (C, R) in enumerate(bnd):
            if not passes(C, R, rays).any():
                skip[b] += 1
    skip /= trials
    print(f"{name:18s} blocks {len(bnd)}: skippable tiles {skip.mean():.3f}  per block "
          + " ".join(f"{x:.2f}" for x in skip) + "  radii " + " ".join(f"{R:.1f}" for _, R in bnd))
segl = np.mean([len(paths[q][s]) for q in range(n) for s in range(nsamp)])
print(f"mean segments per path {segl:.2f}")
