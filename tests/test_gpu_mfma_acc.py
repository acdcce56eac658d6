"""The matrix-core filter's one measured hardware premise, re-checked on every
GPU box (DESIGN.md §4.2 "Assumption").

The filter's margin proof (rt_dev_intersect.h, above RT_MF_MU) bounds the
f32 accumulation of its 31 exact f16 x f16 products in the walk's chain of two
`v_mfma_f32_32x32x16_f16` by 33 roundings of at most 2^-24 of the running
|sum|: |D - exact| <= 33 * 2^-24 * sum|p|. AMD documents no summation order or
rounding for the instruction, so the premise is measured: rt_debug_mfma_acc
runs the product's own chain (same source file, same flags) on random and
adversarial operand tiles and this test asserts the worst element inside the
allowance, reporting the measured worst case.

"Exact" is the float64 sum of the products (each exact in float64: 11 x 11
significand bits); its own error is <= 32 * 2^-53 * sum|p|, 2^-24 of the
allowance."""
import json
import os

import numpy as np
import pytest

from bevy_raytrace_amd import abi

pytestmark = pytest.mark.gpu

ALLOWANCE = 33.0  # roundings of <= 2^-24 sum|p| (the proof's budget)
T = 1024  # tiles per operand family


def run_tiles(A, B):
    """D = the walk's chained MFMAs per tile: A (t, 32, 32) rows x K, B (t, 32, 32) K x cols."""
    import torch
    lib = abi.load()
    assert hasattr(lib, "rt_debug_mfma_acc"), "library built without the matrix-core filter"
    a = torch.from_numpy(np.ascontiguousarray(A, np.float16).view(np.int16)).cuda()
    b = torch.from_numpy(np.ascontiguousarray(B, np.float16).view(np.int16)).cuda()
    d = torch.empty(A.shape, dtype=torch.float32, device="cuda")
    assert lib.rt_debug_mfma_acc(a.data_ptr(), b.data_ptr(), d.data_ptr(), A.shape[0]) == 0
    return d.cpu().numpy()


def ratio(A, B, D):
    """|D - exact| / (2^-24 sum|p|) per element (0 where every product is 0)."""
    a, b = A.astype(np.float64), B.astype(np.float64)
    exact = a @ b
    mag = np.abs(a) @ np.abs(b)
    err = np.abs(D.astype(np.float64) - exact)
    with np.errstate(invalid="ignore", divide="ignore"):
        r = np.where(mag > 0, err / (mag * 2.0 ** -24), np.where(err > 0, np.inf, 0.0))
    return r, exact


def f16(x):
    return np.asarray(x, np.float64).astype(np.float16)


def split(x):
    """x -> (hi, lo) f16 parts, as the host's feature split (rt_api.cpp build_mfma)."""
    hi = f16(x)
    return hi, f16(np.asarray(x, np.float64) - hi.astype(np.float64))


def families(rng):
    """Operand tile families (A, B), each (T, 32, 32) f16."""
    out = {}
    # 1. random mixed signs, exponents in [-6, 6]: cancellation-heavy
    def rnd(shape, lo=-6, hi=6):
        return f16(rng.choice([-1.0, 1.0], shape) * np.ldexp(rng.uniform(1, 2, shape),
                                                             rng.integers(lo, hi + 1, shape)))
    out["random"] = (rnd((T, 32, 32)), rnd((T, 32, 32)))
    # 2. one large product then 31 products each just under half an ulp of it:
    #    a sequential f32 sum would round every one of them away
    A = np.zeros((T, 32, 32)); B = np.zeros((T, 32, 32))
    A[:, :, 0] = 1.0
    B[:, 0, :] = f16(np.ldexp(rng.uniform(1, 2, (T, 32)), 0))
    A[:, :, 1:] = f16(np.ldexp(rng.uniform(1.0, 1.99, (T, 32, 31)), -12))
    B[:, 1:, :] = f16(np.ldexp(rng.uniform(1.0, 1.0 + 2 ** -10, (T, 31, 32)), -14)) * \
        rng.choice([-1.0, 1.0], (T, 31, 32))
    out["absorbed_tail"] = (f16(A), f16(B))
    # 3. large terms that cancel pairwise, the residue made of small terms
    A = rnd((T, 32, 32), 4, 7); B = rnd((T, 32, 32), 4, 7)
    A[:, :, 1:16:2] = A[:, :, 0:16:2]
    B[:, 1:16:2, :] = -B[:, 0:16:2, :]
    A[:, :, 16:] = rnd((T, 32, 16), -10, -6)
    out["cancelling"] = (f16(A), f16(B))
    # 4. the filter's own shape: ten features split hi + lo on both sides
    #    (hi*hi + hi*lo + lo*hi, 30 terms), + the threshold's hi and lo against
    #    exact ones (K 30, 31), features from RTIOW-range centres / rays
    sph = rng.uniform(-11, 11, (T, 32, 10)) * rng.choice([1.0, 1e-2, 10.0], (T, 32, 10))
    ray = rng.uniform(-1, 1, (T, 10, 32)) * rng.choice([1.0, 1e-3, 8.0], (T, 10, 32))
    thr = -np.einsum("tik,tkj->tij", sph, ray)[:, :1, :] * rng.uniform(0.999, 1.001, (T, 1, 32))
    sh, sl = split(sph)
    rh, rl = split(ray)
    th, tl = split(thr[:, 0, :])
    A = np.zeros((T, 32, 32), np.float16); B = np.zeros((T, 32, 32), np.float16)
    for k in range(10):
        A[:, :, 3 * k], B[:, 3 * k, :] = sh[:, :, k], rh[:, k, :]
        A[:, :, 3 * k + 1], B[:, 3 * k + 1, :] = sh[:, :, k], rl[:, k, :]
        A[:, :, 3 * k + 2], B[:, 3 * k + 2, :] = sl[:, :, k], rh[:, k, :]
    A[:, :, 30] = 1.0; B[:, 30, :] = th
    A[:, :, 31] = 1.0; B[:, 31, :] = tl
    out["filter_shaped"] = (A, B)
    # 5. sums landing on f32 rounding ties: 2^24 + 1 style (1 + 2^-24 + 2^-24 ...)
    A = np.zeros((T, 32, 32)); B = np.zeros((T, 32, 32))
    A[:, :, 0] = 1.0; B[:, 0, :] = 1.0
    A[:, :, 1:] = 2.0 ** -12
    B[:, 1:, :] = 2.0 ** -12 * rng.choice([0.5, 1.0, -0.5, -1.0, 1.5], (T, 31, 32))
    out["ties"] = (f16(A), f16(B))
    return out


def test_mfma_chain_layout_is_the_products():
    """A tile with one non-zero product per element returns that product
    exactly: the operand layout the test (and the walk) assumes is the
    instruction's."""
    rng = np.random.default_rng(7)
    A = np.zeros((4, 32, 32), np.float16); B = np.zeros((4, 32, 32), np.float16)
    for t in range(4):
        ks = rng.permutation(32)
        for r in range(32):
            A[t, r, ks[r]] = f16(rng.uniform(1, 2) * (r + 1))
        B[t] = f16(rng.uniform(-2, 2, (32, 32)))
    D = run_tiles(A, B)
    exact = A.astype(np.float64) @ B.astype(np.float64)
    assert np.array_equal(D, exact.astype(np.float32))


def test_mfma_accumulation_within_the_proofs_allowance():
    rng = np.random.default_rng(20221015)
    report = {}
    for name, (A, B) in families(rng).items():
        D = run_tiles(A, B)
        r, exact = ratio(A, B, D)
        assert np.isfinite(D).all(), name
        report[name] = {"worst_ratio": float(r.max()),
                        "share_equal_rn_exact": float(np.mean(D == exact.astype(np.float32))),
                        "elements": int(r.size)}
    worst = max(v["worst_ratio"] for v in report.values())
    line = {"allowance": ALLOWANCE, "worst_ratio": worst, "families": report,
            "unit": "|D - exact| / (2^-24 sum|p|), two chained v_mfma_f32_32x32x16_f16"}
    print("mfma accumulation:", json.dumps(line))
    out = os.environ.get("RT_MFMA_ACC_REPORT")
    if out:
        with open(out, "w") as f:
            json.dump(line, f, indent=1)
    assert worst <= ALLOWANCE, line
