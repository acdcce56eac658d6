"""CPU model of the matrix-core walk's tiles on the real rays of the headline
launch (tools/ray_dump.py's dump: every lane's ray in 1,024 waves at one
loop iteration): how many (sphere, ray) pairs the walk filters per wave
iteration with the current tile shape -- 32 spheres x 32 rays per
v_mfma_f32_32x32x16_f16 pair, a block walked for a half-wave when either of
its two 16-sphere half-block bounds passes a ray of the half -- against
finer shapes the bounds could select with: 16 spheres x 32 rays (a
half-block per half-wave) and 16 x 16 (v_mfma_f32_16x16x32_f16: a
half-block per 16-ray quarter). The bound test is the kernel's (rt_api.cpp
build_mfma, rt_dev_intersect.h "Block bounds" / "Forward bounds"): the line
passes within R^2 = (1 + 2^-4) L^2 + muB (|o|^2 + |C|^2) of the bound's centre
C, and the bound is not wholly behind the origin
(dn.(C - o) + 2^-7 (|o|_1 + |C|_1) + (1 + 2^-3) L >= 0).
usage: python tools/tile_shape_model.py <ray_dump.npy>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from bevy_raytrace_amd import abi, scene  # noqa: E402


def bounds(sp, perm):
    c = sp["center"].astype(np.float64)
    r = np.abs(sp["radius"].astype(np.float64))
    last = int(np.nonzero(perm >= 0)[0].max()) + 1
    nblk = (last + 31) // 32
    out = []
    for h in range(2 * nblk):
        idx = perm[16 * h:16 * h + 16]
        idx = idx[idx >= 0]
        if len(idx) == 0:
            out.append(None)
            continue
        C = ((c[idx].min(0) + c[idx].max(0)) * 0.5).astype(np.float32).astype(np.float64)
        L = float(np.max(np.linalg.norm(c[idx] - C, axis=1) + r[idx]))
        out.append((C, L))
    return nblk, out


def passes(o, dn, C, L):
    """(rays,) bool: the half-block bound (C, L) passes the ray (o, dn)."""
    R2 = (1 + 2.0 ** -4) * L * L
    oc = C - o
    tc = (oc * dn).sum(1)
    line = ((oc * oc).sum(1) - tc * tc) <= R2 + 2.0 ** -8 * ((o * o).sum(1) + C @ C)
    fwd = tc + 2.0 ** -7 * (np.abs(o).sum(1) + np.abs(C).sum()) + (1 + 2.0 ** -3) * L >= 0
    return line & fwd


def main():
    dump = np.load(sys.argv[1])  # (waves, 64, 2, 4)
    o = dump[:, :, 0, :3].astype(np.float64)
    pix = dump[:, :, 0, 3].copy().view(np.uint32)
    d = dump[:, :, 1, :3].astype(np.float64)
    live = pix != 0xFFFFFFFF
    sp = scene.rtiow_final_scene().objects_gpu()
    perm = abi.cull_layout(sp)[0]
    nblk, bnd = bounds(sp, perm)
    nh = len(bnd)
    waves = dump.shape[0]
    t32 = t16x32 = t16x16 = 0
    pass_any = 0
    for w in range(waves):
        lv = live[w]
        if not lv.any():
            continue
        dn = d[w] / np.maximum(np.linalg.norm(d[w], axis=1, keepdims=True), 1e-30)
        P = np.zeros((64, nh), bool)  # ray x half-block
        for h, b in enumerate(bnd):
            if b is not None:
                P[:, h] = passes(o[w], dn, *b) & lv
        for half in range(2):
            ph = P[32 * half:32 * half + 32].any(0)  # half-blocks some ray of the half passes
            blk = ph.reshape(nblk, 2).any(1)
            t32 += int(blk.sum())          # 32x32 tiles (current)
            t16x32 += int(ph.sum())        # 16 spheres x 32 rays
        for q in range(4):
            t16x16 += int(P[16 * q:16 * q + 16].any(0).sum())
        pass_any += int(P.any(0).sum())
    n = waves
    print(f"{n} waves, {nblk} blocks, {nh} half-blocks")
    print(f"32x32 tiles per wave iteration (2 halves): {t32 / n:.2f}  -> pairs {t32 / n * 1024:.0f}")
    print(f"16-sphere x 32-ray tiles per iteration: {t16x32 / n:.2f} -> pairs {t16x32 / n * 512:.0f}")
    print(f"16x16 tiles per iteration (4 quarters): {t16x16 / n:.2f} -> pairs {t16x16 / n * 256:.0f}")
    print(f"half-blocks some ray of the wave passes: {pass_any / n:.2f} of {nh}")


if __name__ == "__main__":
    main()
