"""The C++ host side above the C-ABI (bevy_raytrace_amd/host/rt_host.hpp:
MaterialCache, init_spheres, RayTraceCamera, RayTraceNode, RayTracePlugin)
against the Python mirror and the oracle: byte-identical scene, material and
camera records (CPU), and frames rendered through the C++ plugin surface,
with a scene edit between frames, bit-exact against the oracle (GPU)."""
import os
import struct
import subprocess

import numpy as np
import pytest

from bevy_raytrace_amd import abi, scene
from bevy_raytrace_amd.camera import RayTraceCamera, default_camera_block
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "bevy_raytrace_amd", "host")


def _bin(name):
    p = os.path.join(HOST, "bin", name)
    if not os.path.exists(p):
        pytest.fail(f"{p} missing: build with __graft_entry__.build()")
    return p


def test_cpp_records_match_python(tmp_path):
    """Scenes (config 1, the reference's dim-7 split, RTIOW dim 11, the 10 k
    scene) and the default camera block, C++ vs Python, byte for byte."""
    subprocess.run(["make", "-s", "-C", HOST], check=True, timeout=300)  # CPU-side build
    out = tmp_path / "dump.bin"
    subprocess.run([_bin("host_dump"), str(out)], check=True, timeout=120)
    data = out.read_bytes()
    off = 0
    for sc in (scene.config1_scene(), scene.reference_scene(), scene.rtiow_final_scene(),
               scene.ten_thousand_scene()):
        for arr in (sc.objects_gpu(), sc.materials_gpu()):
            n = struct.unpack_from("<I", data, off)[0]
            off += 4
            b = arr.tobytes()
            assert n == len(arr), sc.name
            assert data[off:off + len(b)] == b, sc.name
            off += len(b)
    cam = default_camera_block().tobytes()
    assert data[off:off + len(cam)] == cam
    assert off + len(cam) == len(data)
    assert RayTraceCamera().render_width == 1920


def _edit(sp, mt):
    """The edit host_frames.cpp makes between frames 1 and 2."""
    sp = sp.copy()
    mt = mt.copy()
    sp["radius"][1] = np.float32(0.75)
    mt[2]["color"] = (0.9, 0.2, 0.1, 1.0)
    mt[2]["reflectance"] = 1
    mt[2]["fuzziness"] = np.float32(0.3)
    return sp, mt


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, abi.RT_FLAG_NO_PRIMARY_CACHE], ids=["reuse", "noreuse"])
def test_cpp_plugin_frames_bit_exact(tmp_path, flags):
    out = tmp_path / "frames.bin"
    subprocess.run([_bin("host_frames"), str(out), str(flags)], check=True, timeout=300)
    data = out.read_bytes()
    W, H, S, D = 64, 36, 2, 8
    frames = struct.unpack_from("<I", data, 0)[0]
    off = 4
    sc = scene.config1_scene()
    sp, mt = sc.objects_gpu(), sc.materials_gpu()
    cam = default_camera_block()
    for i in range(frames):
        f0, segs = struct.unpack_from("<II", data, off)
        off += 8
        img = np.frombuffer(data, np.float32, W * H * 4, off).reshape(H, W, 4)
        off += W * H * 16
        if i == 1:
            sp, mt = _edit(sp, mt)
        assert f0 == i * S
        ref, rsegs = O.render(cam, sp, mt, W, H, S, D, frame0=f0)
        assert np.array_equal(img, ref, equal_nan=True), f"frame {i}"
        assert segs == rsegs
    full, spheres, materials = struct.unpack_from("<III", data, off)
    assert (full, spheres, materials) == (1, 1, 1)
