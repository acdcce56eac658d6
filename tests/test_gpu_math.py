"""The kernel's short correctly rounded forms (bevy_raytrace_amd/csrc/rt_math.h,
guarded in rt_dev_math.h) against the IEEE operations, on the operands their
guards exist for: signed zeros, denormals, tiny / huge values, inf, NaN, and a
random bulk. numpy's float32 sqrt and division are IEEE correctly rounded, so
the bar is bit equality (NaN == NaN)."""
import numpy as np
import pytest

from bevy_raytrace_amd import abi

pytestmark = pytest.mark.gpu

SPECIAL = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-40, 1e-38, 1.2e-38, 1e-30, 1e-19, 2.0 ** -40,
                    2.0 ** -41, 2.0 ** -60, 2.0 ** -61, 2.0 ** -100, 1e-7, 0.2, 1.0, 1.5, 3.0,
                    1e7, 2.0 ** 40, 2.0 ** 41, 2.0 ** 60, 2.0 ** 61, 1e30, 3e38, np.inf, -np.inf,
                    np.nan, -1.0, -0.2, -1e-30, -2.0 ** -40], dtype=np.float32)


def run(mode, x, nout):
    import torch
    lib = abi.load()
    d_in = torch.from_numpy(np.ascontiguousarray(x, np.float32).ravel()).cuda()
    n = nout
    d_out = torch.empty(n * (3 if mode in (1, 2) else 1), dtype=torch.float32, device="cuda")
    assert lib.rt_debug_math(mode, d_in.data_ptr(), n, d_out.data_ptr()) == 0
    return d_out.cpu().numpy()


def same(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    eq = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    return eq


def bulk(rng, n, lo=-45, hi=45):
    sign = rng.choice([-1.0, 1.0], n)
    return (sign * 2.0 ** rng.uniform(lo, hi, n) * rng.uniform(1, 2, n)).astype(np.float32)


def test_sqrt_guarded():
    rng = np.random.default_rng(1)
    x = np.concatenate([SPECIAL, np.abs(bulk(rng, 200000, -130, 120)), bulk(rng, 1000)])
    got = run(0, x, x.size)
    with np.errstate(invalid="ignore"):
        exp = np.sqrt(x)
    assert same(got, exp).all(), x[~same(got, exp)][:8]


def test_normalize_guarded():
    rng = np.random.default_rng(2)
    comb = np.array(np.meshgrid(SPECIAL, SPECIAL[::3], SPECIAL[::5])).reshape(3, -1).T
    v = np.concatenate([comb, bulk(rng, 3 * 100000, -50, 50).reshape(-1, 3),
                        rng.normal(size=(100000, 3)).astype(np.float32)]).astype(np.float32)
    got = run(1, v, v.shape[0]).reshape(-1, 3)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        l = np.sqrt((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2])
        exp = v / l[:, None]
    ok = same(got, exp)
    assert ok.all(), v[~ok.all(1)][:5]


def test_div3_guarded():
    rng = np.random.default_rng(3)
    comb = np.array(np.meshgrid(SPECIAL, SPECIAL[::4], SPECIAL[::6], SPECIAL)).reshape(4, -1).T
    q = np.concatenate([comb, bulk(rng, 4 * 100000, -50, 50).reshape(-1, 4)]).astype(np.float32)
    got = run(2, q, q.shape[0]).reshape(-1, 3)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore", under="ignore"):
        exp = q[:, :3] / q[:, 3:4]
    ok = same(got, exp)
    assert ok.all(), q[~ok.all(1)][:5]


def test_div_guarded():
    rng = np.random.default_rng(4)
    comb = np.array(np.meshgrid(SPECIAL, SPECIAL)).reshape(2, -1).T
    p = np.concatenate([comb, bulk(rng, 2 * 300000, -70, 70).reshape(-1, 2)]).astype(np.float32)
    got = run(3, p, p.shape[0])
    with np.errstate(invalid="ignore", divide="ignore", over="ignore", under="ignore"):
        exp = p[:, 0] / p[:, 1]
    ok = same(got, exp)
    assert ok.all(), p[~ok][:8]
