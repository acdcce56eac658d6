"""Research probe (CPU, the numpy oracle as a ray source): at the
spheres10k1080 workload, how many of the 20 bound chunks (512 walk positions
each) does a 32-ray half-wave pass with the chunk-level test the kernel runs
(the ray's line within the bound, the bound not wholly behind the origin),
and how many would also pass a SEGMENT limit -- the bound not wholly beyond
the ray's exact hit on the large spheres (tested directly first)?

Rays: paths of random pixels at random samples (depth 16), recorded per
segment; a half-wave's lanes are drawn from MIX random pixels (the queue's
mixing, ~5 pixels per half-wave in the headline's ray dump), each at a
uniformly random segment of its paths. Chunks: the big spheres (r > 0.5) in a
block of their own, the rest in k-d order (tools/sim_block_cull.py), 16
blocks per chunk; bound = box centre, radius over the members.
usage: python tools/sim_segment_10k.py [pixels] [samples]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bevy_raytrace_amd import scene  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
import oracle.rt_oracle_np as O  # noqa: E402

W, H, D = 1920, 1080, 16
npx = int(sys.argv[1]) if len(sys.argv) > 1 else 400
nsamp = int(sys.argv[2]) if len(sys.argv) > 2 else 6
MIX = int(os.environ.get("MIX", "5"))
rng = np.random.default_rng(11)

sc = scene.ten_thousand_scene()
sp = np.asarray(sc.objects_gpu())
sph = sp.view(np.float32).reshape(-1, 8)[:, 0:4].copy()
sph_mat = sp.view(np.uint32).reshape(-1, 8)[:, 4].astype(np.int64)
mt = np.asarray(sc.materials_gpu())
mf = mt.view(np.float32).reshape(-1, 8)
mi = mt.view(np.int32).reshape(-1, 8)
mats = dict(index=sph_mat, color=mf[:, 0:3].copy(), refl=mi[:, 4].copy(), fuzz=mf[:, 5].copy(),
            ior=mf[:, 6].copy())
cc = O.camera_consts(np.ascontiguousarray(default_camera_block()).view(np.float32).reshape(-1)[:32], W, H, 0)

rec = []
_orig = O.intersect


def _rec(spheres, o, d):
    best, t = _orig(spheres, o, d)
    rec.append((o.copy(), d.copy(), best.copy(), t.copy()))
    return best, t


O.intersect = _rec
xs = rng.integers(0, W, npx).astype(np.int64)
ys = rng.integers(0, H, npx).astype(np.int64)
segs = [[] for _ in range(npx)]  # per pixel: rows (o, d, t_hit)
for si in range(nsamp):
    rec.clear()
    O.trace(sph, mats, cc, W, H, xs, ys, int(rng.integers(0, 256)), D)
    alive = np.arange(npx)
    for o, d, best, t in rec:
        for k, p in enumerate(alive):
            segs[p].append(np.concatenate([o[k], d[k], [t[k] if best[k] >= 0 else np.inf]]))
        alive = alive[best >= 0]
    print(f"sample {si + 1}/{nsamp}", file=sys.stderr, flush=True)
O.intersect = _orig
segs = [np.array(s, dtype=np.float64) for s in segs]

big = np.nonzero(np.abs(sph[:, 3]) > 0.5)[0]
small = np.nonzero(~(np.abs(sph[:, 3]) > 0.5))[0]
allr = np.concatenate(segs)
bo, tb = O.intersect(sph[big], allr[:, :3].astype(np.float32), allr[:, 3:6].astype(np.float32))
t_large_all = np.where(bo >= 0, tb.astype(np.float64), np.inf)
off = np.cumsum([0] + [len(s) for s in segs])
t_large = [t_large_all[off[i]:off[i + 1]] for i in range(npx)]


def kd_order(idx, c):
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


order = np.concatenate([big, -np.ones((-len(big)) % 32, np.int64),
                        np.array(kd_order(small, sph[:, :3].astype(np.float64)))])
CH = int(os.environ.get("CH", "512"))  # walk positions per chunk bound (SUB: bounds per chunk)
SUB = int(os.environ.get("SUB", "1"))
bnd = []
for b in range(0, len(order), CH):
    sub = []
    for q in range(SUB):
        idx = order[b + q * CH // SUB:b + (q + 1) * CH // SUB]
        idx = idx[idx >= 0]
        if len(idx) == 0:
            continue
        c, r = sph[idx, :3].astype(np.float64), np.abs(sph[idx, 3]).astype(np.float64)
        C = (c.min(0) + c.max(0)) / 2
        sub.append((C, np.max(np.linalg.norm(c - C, axis=1) + r)))
    bnd.append(sub)


def tests(C, R, rays, tl):
    o, d = rays[:, :3], rays[:, 3:6]
    ln = np.linalg.norm(d, axis=1)
    dn = d / ln[:, None]
    oc = C - o
    tc = oc @ np.zeros(3) + np.einsum("ij,ij->i", oc, dn)
    R2 = R * R * (1 + 2.0 ** -4)
    line = (np.einsum("ij,ij->i", oc, oc) - tc ** 2) <= R2
    fwd = tc >= -R
    seg = tc - R <= tl * ln
    return line & fwd, line & fwd & seg


trials = 3000
seg_w = np.array([len(s) for s in segs], dtype=np.float64)
seg_w /= seg_w.sum()
cur = np.zeros(len(bnd))
new = np.zeros(len(bnd))
for _t in range(trials):
    pix = rng.choice(npx, MIX, p=seg_w)
    rays, tl = [], []
    for q in pix.repeat(32 // MIX + 1)[:32]:
        k = rng.integers(0, len(segs[q]))
        rays.append(segs[q][k])
        tl.append(t_large[q][k])
    rays, tl = np.array(rays), np.array(tl)
    for b, sub in enumerate(bnd):
        anyc = anys = False
        for (C, R) in sub:
            a, s_ = tests(C, R, rays, tl)
            anyc |= a.any()
            anys |= s_.any()
        cur[b] += anyc
        new[b] += anys
print(f"chunks {len(bnd)}; passed per half-wave: line+forward {cur.sum() / trials:.2f}, "
      f"+ segment limit {new.sum() / trials:.2f}")
print("per chunk (cur/new): " + " ".join(f"{c / trials:.2f}/{n / trials:.2f}" for c, n in zip(cur, new)))
print(f"segments per path {np.mean([len(s) for s in segs]) / nsamp:.2f}; rays with a finite "
      f"large-sphere hit {np.isfinite(t_large_all).mean():.3f}")
