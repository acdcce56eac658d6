"""Host-side logic on CPU: byte layouts, scene / camera builders, the C-ABI
library (loads, exports every symbol of include/rt_hip.h, host-only entry
points and error paths without a GPU)."""
import ctypes
import os

import numpy as np
import pytest

from bevy_raytrace_amd import abi, scene
from bevy_raytrace_amd.camera import RayTraceCamera, Transform, camera_block
from bevy_raytrace_amd.configs import WORKLOADS, pick_row_block


def test_std430_std140_layouts():
    # SphereGPU: vec3 center @0, f32 radius @12, u32 material @16, stride 32 (sphere.rs:12-17)
    d = abi.SPHERE_DTYPE
    assert d.itemsize == 32 and d.fields["radius"][1] == 12 and d.fields["material"][1] == 16
    # MaterialGPU: vec4 color @0, i32 @16, f32 fuzz @20, f32 ior @24 (ray_trace_materials.rs:33-43)
    m = abi.MATERIAL_DTYPE
    assert m.itemsize == 32 and m.fields["reflectance"][1] == 16
    assert m.fields["fuzziness"][1] == 20 and m.fields["index_of_refraction"][1] == 24
    # CameraGPU std140: transform 0, forward 64, fov 76, up 80, ipd 92,
    # right 96, lfl 108, position 112, fstop 124
    c = abi.CAMERA_DTYPE
    offs = {k: c.fields[k][1] for k in c.names}
    assert offs == {"transform": 0, "forward": 64, "fov": 76, "up": 80, "image_plane_distance": 92,
                    "right": 96, "lens_focal_length": 108, "position": 112, "fstop": 124}
    assert c.itemsize == 128


def test_camera_block_values():
    cam = RayTraceCamera().to_gpu()
    assert cam["fov"] == np.float32(1.5708)
    assert cam["image_plane_distance"] == 10 and cam["lens_focal_length"] == np.float32(0.1)
    assert cam["fstop"] == np.float32(1 / 32)
    np.testing.assert_array_equal(cam["position"], [13, 2, 3])
    # forward = -back, orthonormal basis
    T = cam["transform"].reshape(4, 4)[:3, :3].astype(np.float64)
    np.testing.assert_allclose(T @ T.T, np.eye(3), atol=1e-6)
    np.testing.assert_allclose(cam["forward"], -T[2], atol=0)
    t2 = Transform.from_xyz(0, 5, 10).looking_at((0, 0, 0))
    c2 = camera_block(t2)
    np.testing.assert_allclose(c2["forward"], -np.array([0, 5, 10]) / np.sqrt(125), atol=1e-6)


def test_scene_generators_deterministic():
    a = scene.rtiow_final_scene().objects_gpu()
    b = scene.rtiow_final_scene().objects_gpu()
    assert a.tobytes() == b.tobytes()
    c = scene.rtiow_final_scene(seed=7).objects_gpu()
    assert a.tobytes() != c.tobytes()


def test_scene_generator_shapes():
    ref = scene.reference_scene()
    sp, mt = ref.objects_gpu(), ref.materials_gpu()
    # ground + <=196 grid + 3 big (sphere.rs:37-148, dim 7), reference split: no glass
    assert 150 < len(sp) <= 199 and len(mt) == len(sp)
    assert set(np.unique(mt["reflectance"])) <= {0, 1}
    # spawn order: ground first, the 3 big spheres last (ECS query order)
    assert sp[0]["radius"] == 1000 and (sp[-3:]["radius"] == 1).all()
    # names -> index map in insertion order (IndexMap)
    assert ref.materials.get_index_of("ground") == 0 and ref.materials.get_index_of("right") == 3
    rt = scene.rtiow_final_scene()
    sp = rt.objects_gpu()
    assert 470 <= len(sp) <= 488
    assert set(np.unique(rt.materials_gpu()["reflectance"])) == {0, 1, 2}
    ten = scene.ten_thousand_scene()
    assert len(ten.objects_gpu()) == 10000
    c1 = scene.config1_scene()
    assert list(c1.materials_gpu()["reflectance"]) == [0, 0, 2, 1]


def test_scene_file_roundtrip(tmp_path):
    sc = scene.config1_scene()
    p = tmp_path / "s.npz"
    sc.save(p)
    sp, mt = scene.Scene.load_arrays(p)
    assert sp.tobytes() == sc.objects_gpu().tobytes()
    assert mt.tobytes() == sc.materials_gpu().tobytes()


def test_row_block_choice():
    assert pick_row_block(1080, 1) == 8
    for n in (2, 4, 8):
        b = pick_row_block(1080, n)
        assert 1080 % b == 0 and (1080 // b) % n == 0
    assert pick_row_block(4320, 8) == 1  # single rows, 540 per rank
    assert pick_row_block(225, 2) == 8  # no even split: the round-2 fallback
    assert WORKLOADS["rtiow1080"].spp == 64 and WORKLOADS["rtiow1080"].max_depth == 16


# ------------------------------------------------------------------ C-ABI
def test_library_exports_every_header_symbol():
    lib = abi.load()
    names = abi.header_symbols()
    assert {"rt_create", "rt_destroy", "rt_set_scene", "rt_render", "rt_render_device",
            "rt_render_async", "rt_wait", "rt_assemble_shards", "rt_assemble_shard_frames",
            "rt_last_error", "rt_version", "rt_shard_rows"} <= set(names)
    for n in names:
        assert hasattr(lib, n), n
    assert lib.rt_version() == 1


@pytest.mark.parametrize("H,B,K", [(1080, 8, 1), (1080, 5, 8), (23, 3, 2), (7, 8, 3), (4320, 8, 8)])
def test_shard_rows_host(H, B, K):
    lib = abi.load()
    tot = 0
    for k in range(K):
        n = lib.rt_shard_rows(H, B, K, k)
        assert n == len(abi.shard_rows(H, B, K, k))
        tot += n
    assert tot == H
    assert lib.rt_shard_rows(H, B, K, K) == 0


def test_serpentine_block_deal():
    """Blocks go to shards in groups of K, alternating direction, so every
    shard's rows sit at the same mean height (up to the last group)."""
    from bevy_raytrace_amd.distributed import ShardLayout
    assert [abi.block_owner(b, 4) for b in range(12)] == [0, 1, 2, 3, 3, 2, 1, 0, 0, 1, 2, 3]
    assert abi.shard_rows(20, 2, 3, 0) == [0, 1, 10, 11, 12, 13]
    H, B, K = 1080, 5, 8
    means = [np.mean(abi.shard_rows(H, B, K, k)) for k in range(K)]
    assert max(means) - min(means) < B * K / 4  # plain b % K would spread them by B*(K-1)
    lay = ShardLayout(H, B, K)
    for y in (0, 39, 40, 41, 79, 80, 1079):
        k, r = lay.source_index(y)
        assert abi.shard_rows(H, B, K, k)[r] == y


def test_null_context_errors_do_not_crash():
    lib = abi.load()
    p = abi.make_params(8, 8, 1, 1)
    assert lib.rt_render(None, None, ctypes.byref(p), None, None) == abi.RT_ERR_INVALID_ARG
    assert b"ctx is NULL" in lib.rt_last_error(None) or lib.rt_last_error(None)
    assert lib.rt_set_scene(None, None, 0, None, 0) == abi.RT_ERR_INVALID_ARG
    assert lib.rt_wait(None, None) == abi.RT_ERR_INVALID_ARG
    assert lib.rt_create(0, None) == abi.RT_ERR_INVALID_ARG


def test_create_without_gpu_reports_device_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    lib = abi.load()
    ctx = ctypes.c_void_p()
    rc = lib.rt_create(0, ctypes.byref(ctx))
    assert rc == abi.RT_ERR_DEVICE
    assert not ctx.value
    assert b"no HIP device" in lib.rt_last_error(None)


def test_bench_spawn_relays_rank0_line(monkeypatch, capsys):
    """bench.py --gpus N without WORLD_SIZE: a child torch.distributed.run on
    127.0.0.1 with N ranks and the same arguments; only rank 0's JSON line
    reaches stdout, and the launcher's exit status is returned."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    seen = {}

    def fake_run(cmd, stdout=None, env=None):
        seen["cmd"], seen["env"] = cmd, env
        out = b'RCCL banner\n{"metric": "m", "value": 1.0}\n'
        return subprocess.CompletedProcess(cmd, 0, stdout=out)

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    rc = bench.spawn_ranks(bench.parse())
    assert rc == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    out = capsys.readouterr()
    assert out.out.strip() == '{"metric": "m", "value": 1.0}'
    assert "RCCL banner" in out.err


def test_flag_constants_agree_across_bindings():
    """Every RT_FLAG_* of include/rt_hip.h has the same value in the Python
    binding (bevy_raytrace_amd/abi.py) and the Rust drop-in (bevy_shim/src/rt_hip.rs)."""
    import re
    from bevy_raytrace_amd import abi
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "include", "rt_hip.h")).read()
    flags = {m.group(1): int(m.group(2), 16) for m in
             re.finditer(r"#define (RT_FLAG_\w+)\s+0x([0-9a-fA-F]+)u", hdr)}
    rs = open(os.path.join(root, "bevy_shim", "src", "rt_hip.rs")).read()
    rflags = {m.group(1): int(m.group(2), 16) for m in
              re.finditer(r"pub const (RT_FLAG_\w+): u32 = 0x([0-9a-fA-F]+);", rs)}
    assert len(flags) >= 5
    for name, v in flags.items():
        assert getattr(abi, name) == v, name
        assert rflags.get(name) == v, name
    # the in-flight depth the shim sizes its host buffers by
    pend = int(re.search(r"#define RT_MAX_PENDING\s+(\d+)", hdr).group(1))
    rpend = int(re.search(r"pub const RT_MAX_PENDING: u32 = (\d+);", rs).group(1))
    assert pend == rpend == abi.RT_MAX_PENDING


def test_bench_roofline_recomputes_from_committed_counters():
    """bench.py's roofline (SIMD issue) follows from the committed PMC record:
    at the profiled launch time and clock its frac is the record's issue busy
    (<= 1), the busy is the documented formula over the raw counters, and a
    run on a faster clock at the same cycle count reads the same frac."""
    import json
    import bench
    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = bench.load_pmc("rtiow1080")
    assert e is not None and "simd_issue" in e
    si = e["simd_issue"]
    r = bench.simd_issue_roofline(e, e["frames_per_launch"], si["kernel_ms_under_pmc"],
                                  si["clock_ghz"])
    assert r["bound"] == "SIMD issue"
    assert 0.5 < r["frac"] <= 1.0
    assert abs(r["frac"] - si["busy"]) < 1e-3
    # the same cycles at another clock: the launch takes proportionally less time
    f = 2.4 / si["clock_ghz"]
    r2 = bench.simd_issue_roofline(e, e["frames_per_launch"], si["kernel_ms_under_pmc"] / f, 2.4)
    assert abs(r2["frac"] - r["frac"]) < 1e-3
    raw = json.load(open(os.path.join(ROOT, si["raw_record"])))
    c = raw["per_dispatch_mean"]["rt_render_kernel"]
    cyc = 4 * (c["SQ_ACTIVE_INST_VALU"] - c["SQ_ACTIVE_INST_VALU2"]) + 4 * c["SQ_INSTS_MFMA"]
    assert abs(cyc / (1024 * c["GRBM_GUI_ACTIVE"] / 8) - si["busy"]) < 1e-9
