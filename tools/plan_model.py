"""Host-side model of one launch's item -> (frame, blocks, slot) map and of the
collect's slot reads (rt_dev_path.h start_item / fold_frame, rt_api.cpp
regions / launch_slots), checked for exact cover: every (frame, block) pair of
the main part traced by exactly one item, every slot written once and read by
the collect of its own frame, in block order.  Pure Python, no GPU; used to
check a work-plan change before it goes to the box.

usage: python tools/plan_model.py   (runs the sweep below)
"""
import itertools


def plan(nframes, nb, qpix, qmain, lead):
    fp = (qpix + nb - 1) // nb
    fl, nreg = fp, qmain - qpix
    if lead and lead < nb:
        f = fp
        while f * nb < qmain:
            nreg -= min(lead, qmain - f * nb)
            f += 1
            fl += 1
    else:
        lead = 0
    c0 = fp * nb - qpix
    return fp, fl, lead, nreg, c0


def items(nframes, nb, qpix, qmain, lead, npix=3):
    fp, fl, lead, nreg, c0 = plan(nframes, nb, qpix, qmain, lead)
    main_pix = fl * npix
    out = []  # (frame, b0, b1, slot, k)
    for item in range(main_pix):  # frame-major order
        f, k = divmod(item, npix)
        b1 = min(nb, qpix - f * nb) if f < fp else min(lead, qmain - f * nb)
        out.append((f, 0, b1, f * npix + k, k))
    for j in range(nreg * npix):
        r, k = divmod(j, npix)
        if r < c0:
            f = fp - 1
            b0 = qpix + r - f * nb
        else:
            r1 = r - c0
            fr = r1 // (nb - lead)
            f = fp + fr
            b0 = lead + (r1 - fr * (nb - lead))
        out.append((f, b0, b0 + 1, main_pix + r * npix + k, k))
    return out, (fp, fl, lead, nreg, c0, main_pix)


def collect_reads(f, k, nb, qpix, qmain, regs, npix=3):
    fp, fl, lead, nreg, c0, main_pix = regs
    q0 = f * nb

    def below(q):
        return min(nb, q - q0) if q > q0 else 0

    lf = f >= fp
    bm = below(qmain)
    bp = min(lead, bm) if lf else below(qpix)
    reads = []
    if bp:
        reads.append(((0, bp), f * npix + k))
    for b in range(bp, bm):
        r = c0 + (f - fp) * (nb - lead) + (b - lead) if lf else q0 + b - qpix
        reads.append(((b, b + 1), main_pix + r * npix + k))
    return reads


def check(nframes, nb, qpix, qmain, lead, npix=3):
    its, regs = items(nframes, nb, qpix, qmain, lead, npix)
    slots = {}
    cover = {}
    for f, b0, b1, slot, k in its:
        assert b1 > b0, (f, b0, b1)
        assert slot not in slots, ("slot twice", slot)
        slots[slot] = (f, b0, b1, k)
        for b in range(b0, b1):
            key = (f, b, k)
            assert key not in cover, ("pair twice", key)
            cover[key] = slot
    want = {(q // nb, q % nb, k) for q in range(qmain) for k in range(npix)}
    assert set(cover) == want, "cover"
    for f in range(nframes):
        for k in range(npix):
            nxt = 0
            for (b0, b1), slot in collect_reads(f, k, nb, qpix, qmain, regs, npix):
                assert slots[slot] == (f, b0, b1, k), (f, k, slot, slots.get(slot), b0, b1)
                assert b0 == nxt
                nxt = b1
            assert nxt == min(nb, max(0, qmain - f * nb)), (f, k, nxt)
    return regs


def main():
    n = 0
    for nframes, nb in itertools.product((1, 2, 3, 5, 20), (1, 2, 3, 8)):
        pairs = nframes * nb
        for L in (0, 1, nb, min(pairs, nb + 1)):
            qmain = pairs - L
            for qpix in range(0, qmain + 1):
                for lead in (0, 1, 2, 3, 4, 7, 8):
                    check(nframes, nb, qpix, qmain, lead)
                    n += 1
    print("plan_model: %d plans exact" % n)


if __name__ == "__main__":
    main()


def host_plan(npix, spp, depth, nframes, lanes, tail=(0.0, 1.0, 0.5), block_region=None,
              block_align=True, block_lead=-1, sample_block=8):
    """rt_api.cpp enqueue's plan for a one-pass launch (no scratch limit):
    -> dict(qmain, qpix, fp, fl, lead, nreg, c0)."""
    import math
    nb = (spp + sample_block - 1) // sample_block

    def per_px(a, mult):
        if a <= 0:
            return 0
        v = math.ceil(a * depth * lanes / npix)
        return (v + mult - 1) // mult * mult

    A4, A2, A1 = per_px(tail[0], 4), per_px(tail[1], 2), per_px(tail[2], 1)
    pairs = nframes * nb
    L = (A4 + A2 + A1 + sample_block - 1) // sample_block
    L = 1 if L < 1 else min(L, pairs)
    qmain = pairs - L
    a8 = block_region if block_region is not None else min(128.0, max(64.0, 16.0 * spp / depth))
    Q = (per_px(a8, 1) + sample_block - 1) // sample_block
    if Q >= qmain:
        Q = qmain
    elif block_align and nb > 1:
        qa = (qmain - Q + nb - 1) // nb * nb
        if qa < qmain and 4 * (qmain - qa) >= 3 * Q:
            Q = qmain - qa
    qpix = qmain - Q
    fp = (qpix + nb - 1) // nb
    m = block_lead if block_lead >= 0 else (2 if fp else 0)
    fp_, fl, lead, nreg, c0 = plan(nframes, nb, qpix, qmain, m)
    return dict(qmain=qmain, qpix=qpix, fp=fp_, fl=fl, lead=lead, nreg=nreg, c0=c0)
