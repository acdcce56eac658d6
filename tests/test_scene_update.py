"""Scene edits on the host (the reference re-uploads the whole
list every frame, /root/reference/src/sphere.rs:166-197): rt_update_spheres
marks the moved spheres, and the next render moves them into the matrix-core
walk's layout in place (rt_api.cpp mf_update) -- their rows, their
half-block's bound row and their chunk's chunk-level row -- instead of a new
spatial order and a whole rebuild, when every moved sphere keeps its radius,
stays near its block's box and the feature scale does not change.

CPU only, through the host-only entry rt_debug_mf_update: the in-place layout
must be, byte for byte, the layout filled from scratch in the same walk order
(A fragments, bound chunks, records, permutations), and the fallbacks must be
taken where the conditions fail. The GPU side (frames after in-place edits
equal the oracle's) is tests/test_gpu_parity.py::test_update_spheres_in_place.
Timings are printed for DESIGN.md §9 (tools/scene_update_times.py records
them)."""
import ctypes

import numpy as np
import pytest

from bevy_raytrace_amd import abi, scene


def mf_update(sp, idx, new):
    lib = abi.load()
    idx = np.ascontiguousarray(idx, np.uint32)
    new = np.ascontiguousarray(new, dtype=abi.SPHERE_DTYPE)
    ms = np.zeros(3, np.float64)
    rc = lib.rt_debug_mf_update(sp.ctypes.data_as(ctypes.c_void_p), len(sp),
                                idx.ctypes.data_as(ctypes.c_void_p),
                                new.ctypes.data_as(ctypes.c_void_p), len(idx),
                                ms.ctypes.data_as(ctypes.c_void_p))
    return rc, ms


@pytest.fixture(scope="module")
def rtiow():
    return np.ascontiguousarray(scene.rtiow_final_scene().objects_gpu())


@pytest.fixture(scope="module")
def tenk():
    return np.ascontiguousarray(scene.ten_thousand_scene().objects_gpu())


def moved(sp, idx, delta):
    new = sp[idx].copy()
    new["center"] += np.asarray(delta, np.float32)
    return new


def test_one_small_move_is_in_place_and_byte_identical(rtiow):
    rc, ms = mf_update(rtiow, [100], moved(rtiow, [100], (0.05, 0.0, -0.03)))
    assert rc == 1, rc


def test_many_moves_in_many_blocks(rtiow):
    rng = np.random.default_rng(3)
    idx = rng.choice(np.arange(1, len(rtiow) - 3), 40, replace=False)
    d = rng.uniform(-0.05, 0.05, (40, 3)).astype(np.float32)
    d[:, 1] = 0
    new = rtiow[idx].copy()
    new["center"] += d
    rc, _ = mf_update(rtiow, idx, new)
    assert rc == 1, rc


def test_moving_a_large_sphere_in_place(rtiow):
    # the r = 1 spheres share the large spheres' block with the ground
    big = [i for i in range(len(rtiow)) if rtiow["radius"][i] >= 1.0 and rtiow["radius"][i] < 10]
    rc, _ = mf_update(rtiow, big[:1], moved(rtiow, big[:1], (0.1, 0.0, 0.1)))
    assert rc == 1, rc


def test_material_change_alone_is_in_place(rtiow):
    new = rtiow[[7]].copy()
    new["material"] = 3
    rc, _ = mf_update(rtiow, [7], new)
    assert rc == 1, rc


@pytest.mark.parametrize("case", ["far", "radius", "range", "scale"])
def test_fallbacks(rtiow, case):
    i = 50
    new = rtiow[[i]].copy()
    if case == "far":        # leaves its block's box: a new spatial order
        new["center"] += np.float32(30.0)
    elif case == "radius":   # the large / small split may change
        new["radius"] = np.float32(0.25)
    elif case == "range":    # outside the f16 split's range: the VALU filter
        new["center"][0, 0] = np.float32(5000.0)
    else:                    # changes sq (max |c_a c_b|): every row rescales
        new["center"][0, 0] = np.float32(3000.0)
    rc, _ = mf_update(rtiow, [i], new)
    assert rc == 0, rc


def test_ten_thousand_spheres_in_place_is_fast(tenk):
    rc, ms = mf_update(tenk, [4321], moved(tenk, [4321], (0.02, 0.0, 0.02)))
    assert rc == 1, rc
    full, inplace = ms[2], ms[1]
    print(f"10k spheres: full rebuild {full:.3f} ms, in place {inplace:.3f} ms")
    # the in-place update is one O(N) scale pass plus O(1) rows: well under
    # the 1 ms the verdict set, and far under the full rebuild
    assert inplace < 1.0 and inplace < full / 5
