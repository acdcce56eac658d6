"""Self-tests of the WGSL interpreter behind tests/golden/wgsl_*.npz (CPU).

The interpreter (tests/golden/wgsl_exec.py) executes the reference's shaders
to make the fixtures that pin the oracle; these cases check the semantics it
must get right on small WGSL snippets written here: u32 wraparound, f32
rounding per operation (no contraction), abstract-literal conversion, value
semantics of structs, control flow, atomics, the host-shareable layout rules
used to decode the host records, and the fixed builtin forms."""
import os
import struct
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import wgsl_exec as W  # noqa: E402

from bevy_raytrace_amd.abi import MATERIAL_DTYPE, SPHERE_DTYPE  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from oracle import oracle as O  # noqa: E402

F = np.float32


def run_fn(src, name, *args):
    sh = W.Shader(src)
    return sh.call(("call", name, (), [("lit", a) for a in args]), [{}])


HASH = """
fn hash3( ni: u32 ) -> vec3<f32>
{
    var n = ni;
    n = (n << 13u) ^ n;
    n = n * (n * n * 15731u + 789221u) + 1376312589u;
    let k = n * vec3<u32>(n, n*16807u, n*48271u);
    let l = vec3<u32>(0x7fffffffu);
    let m = vec3<f32>(f32(k.x&l.x), f32(k.y&l.y), f32(k.z&l.z));
    return m / f32(0x7fffffff);
}
"""


@pytest.mark.parametrize("n", [0, 1, 2, 12345, 2073600, 0xFFFFFFFF])
def test_u32_wraparound_hash_matches_oracle(n):
    v = run_fn(HASH, "hash3", np.uint32(n))
    assert [float(x) for x in v] == [float(x) for x in O.hash3(n)]


def test_f32_rounding_per_op_and_literals():
    src = """
    let EPS: f32 = 0.001;
    fn f(a: f32, b: f32, c: f32) -> f32 { return a * b + c; }
    fn g(x: f32) -> f32 { return 0.5 * x + 1.0 + EPS; }
    """
    a, b, c = F(1.0000001), F(3.0000002), F(-3.0000005)
    got = run_fn(src, "f", a, b, c)
    assert type(got) is F and got == F(a * b) + c  # two roundings, not an FMA
    x = F(0.7)
    assert run_fn(src, "g", x) == (F(0.5) * x + F(1.0)) + F(0.001)


def test_struct_value_semantics_and_control_flow():
    src = """
    struct s { v: vec3<f32>, k: u32, };
    fn f(n: i32) -> u32 {
        var a = s(vec3<f32>(1.0), 0u);
        var b = a;
        b.k = 7u;
        var acc = 0u;
        for (var i: i32 = 0; i < n; i = i + 1) {
            if (i == 3) { continue; } else if (i > 5) { break; }
            acc += u32(i);
        }
        return a.k * 1000u + b.k * 100u + acc;
    }
    """
    # a untouched by b's write; loop adds 0+1+2+4+5 = 12
    assert int(run_fn(src, "f", np.int32(10))) == 0 * 1000 + 7 * 100 + 12


def test_builtin_forms():
    src = """
    fn n(v: vec3<f32>) -> vec3<f32> { return normalize(v); }
    fn p(x: f32) -> f32 { return pow(x, 5.0); }
    fn m(x: f32) -> f32 { return min(x, 1.0); }
    """
    v = W.Vec((F(0.3), F(-1.7), F(2.9)))
    l = np.sqrt((F(0.3) * F(0.3) + F(-1.7) * F(-1.7)) + F(2.9) * F(2.9))
    assert list(run_fn(src, "n", v)) == [F(0.3) / l, F(-1.7) / l, F(2.9) / l]
    x = F(0.61)
    assert run_fn(src, "p", x) == ((x * x) * (x * x)) * x
    assert run_fn(src, "m", F(np.nan)) == F(1.0)  # C fminf


def test_atomics_and_layout_decode():
    src = """
    struct sphere { center: vec3<f32>, radius: f32, material: u32, };
    struct object_list { sphere_count: u32, spheres: array<sphere>, };
    struct g { frame: u32, idx: atomic<u32>, };
    @group(0) @binding(0) var<storage, read> objects: object_list;
    @group(0) @binding(1) var<storage, read_write> globals: g;
    fn take() -> u32 { return atomicAdd(&globals.idx, 1u); }
    """
    sh = W.Shader(src)
    sp = np.zeros(3, SPHERE_DTYPE)
    sp["center"] = [[1, 2, 3], [4, 5, 6], [7, 8, 9]]
    sp["radius"] = [0.5, 1.5, 2.5]
    sp["material"] = [9, 8, 7]
    objs = sh.decode(sh.var_type("objects"), struct.pack("<I12x", 3) + sp.tobytes())
    assert int(objs.f["sphere_count"]) == 3 and len(objs.f["spheres"]) == 3
    s1 = objs.f["spheres"][1].f
    assert list(map(float, s1["center"])) == [4, 5, 6] and float(s1["radius"]) == 1.5
    assert int(s1["material"]) == 8  # 32-B stride: vec3 align 16
    glob = sh.decode(sh.var_type("globals"), struct.pack("<2I", 5, 41))
    sh.bind(objects=objs, globals=glob)
    assert [int(sh.call(("call", "take", (), []), [{}])) for _ in range(3)] == [41, 42, 43]
    assert int(glob.f["idx"]) == 44


def test_camera_block_decodes_as_the_shader_struct():
    src = """
    struct camera_config {
        transform: mat4x4<f32>, forward: vec3<f32>, fov: f32, up: vec3<f32>,
        image_plane_distance: f32, right: vec3<f32>, lens_focal_length: f32,
        position: vec3<f32>, fstop: f32,
    };
    @group(0) @binding(0) var<uniform> camera: camera_config;
    """
    sh = W.Shader(src)
    cam = default_camera_block()
    c = sh.decode(sh.var_type("camera"), cam.tobytes())
    assert float(c.f["fov"]) == float(cam["fov"])
    assert float(c.f["fstop"]) == float(cam["fstop"])
    assert [float(x) for x in c.f["transform"].cols[3]] == [float(x) for x in cam["transform"][12:16]]
    assert MATERIAL_DTYPE.itemsize == 32
