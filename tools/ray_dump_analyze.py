"""CPU analysis of tools/ray_dump.py's dump: per half-wave, the distinct
pixels, the bounce mix, and the 32-sphere blocks of the matrix-core walk
(k-d order, the library's own layout) some ray of the half passes near
(the bound row's line test with its margins) -- against the walk's measured
tiles per iteration.
usage: python tools/ray_dump_analyze.py <ray_dump.npy>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bevy_raytrace_amd import abi, scene  # noqa: E402

dump = np.load(sys.argv[1])  # (waves, 64, 2, 4)
o = dump[:, :, 0, :3].astype(np.float64)
pix = dump[:, :, 0, 3].copy().view(np.uint32)
d = dump[:, :, 1, :3].astype(np.float64)
bounce = dump[:, :, 1, 3].copy().view(np.uint32)
live = pix != 0xFFFFFFFF
sp = scene.rtiow_final_scene().objects_gpu()
sph = np.asarray(sp).view(np.float32).reshape(-1, 8)[:, :4].astype(np.float64)
perm = abi.cull_layout(sp)[0]
nblk = (len(perm) - 8) // 32
bnd = []
for b in range(nblk):
    idx = perm[32 * b:32 * b + 32]
    idx = idx[idx >= 0]
    if len(idx) == 0:
        bnd.append(None)
        continue
    c = sph[idx, :3]
    C = (c.min(0) + c.max(0)) / 2
    L = np.max(np.linalg.norm(c - C, axis=1) + np.abs(sph[idx, 3]))
    bnd.append((C, L))
need, npix, b0 = [], [], []
for w in range(dump.shape[0]):
    for h in range(2):
        sl = slice(32 * h, 32 * h + 32)
        lv = live[w, sl]
        if not lv.any():
            continue
        oo, dd = o[w, sl][lv], d[w, sl][lv]
        dn = dd / np.linalg.norm(dd, axis=1, keepdims=True)
        cnt = 0
        for bb in bnd:
            if bb is None:
                continue
            C, L = bb
            R2 = 1.125 * L * L + 2.0 ** -7 * ((oo * oo).sum(1) + C @ C)
            oc = C - oo
            tc = (oc * dn).sum(1)
            if (((oc * oc).sum(1) - tc * tc) <= R2).any():
                cnt += 1
        need.append(cnt)
        npix.append(len(set(pix[w, sl][lv].tolist())))
        b0.append(np.mean(bounce[w, sl][lv] == 0))
need = np.array(need)
print(f"halves {len(need)}: blocks needed per half {need.mean():.2f} of {sum(b is not None for b in bnd)} "
      f"(tiles per iteration {2 * need.mean():.2f}); distinct pixels per half {np.mean(npix):.2f}; "
      f"bounce-0 share {np.mean(b0):.2f}")
for k in range(1, 8):
    sel = np.array(npix) == k
    if sel.any():
        print(f"  halves with {k} pixels: {sel.sum():5d}, blocks needed {need[sel].mean():.2f}")
