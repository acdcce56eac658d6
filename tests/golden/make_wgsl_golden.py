"""Golden fixtures from the reference's OWN shaders (TEST INFRASTRUCTURE; run
in the build container, where /root/reference exists -- never at test time).

The six WGSL kernels of the reference (assets/shaders/{clear,generate,prepass,
intersect,shade,collect}.wgsl) are parsed and executed by tests/golden/
wgsl_exec.py, scheduled exactly as RayTraceNode::run records them
(src/ray_trace_node.rs:195-224: clear, generate, 3 x {prepass, intersect,
shade}, collect; grid floor(W*H*SAMPLES_PER_RAY / 128) workgroups of 128,
ray_trace_node.rs:16,37-38; prepass one invocation, :74), with the host buffers
the reference's prepare systems fill: globals {frame, W, H, spp, 5 counters
reset} (src/ray_trace_globals.rs:56-68), rays / intersections zeroed
(src/ray_trace_rays.rs:50-66), the sphere list with its 16-B count header
(src/sphere.rs:166-197), materials (src/ray_trace_materials.rs:129-164) and the
128-B camera block (src/ray_trace_camera.rs:43-68) -- here our ABI records
(bevy_raytrace_amd.abi), decoded by the shaders' own struct declarations.

SAMPLES_PER_RAY = 1 (the reference's spp > 1 is not
reproduced by the oracle); where W*H is not a multiple of 128 the floor-divided
grid leaves the last pixels untraced (D1) and `processed` says how many
(row-major) pixels the comparison covers. Each fixture holds the inputs and the per-frame output image; the
oracle is checked against it in tests/test_oracle.py (depth 3 = the
reference's loop count).

usage: python tests/golden/make_wgsl_golden.py [--ref /root/reference]
"""
import argparse
import os
import struct
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))  # tests/: raygen
import wgsl_exec as W  # noqa: E402

from bevy_raytrace_amd import scene  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402

KERNELS = ("clear", "generate", "prepass", "intersect", "shade", "collect")
WORKGROUP = 128  # ray_trace_node.rs:16
BOUNCE_LOOPS = 3  # ray_trace_node.rs:213

CASES = [
    # name, scene, W, H, frames
    ("wgsl_config1_64x32", scene.config1_scene, 64, 32, (0, 1, 7, 1000)),
    ("wgsl_reference_32x16", scene.reference_scene, 32, 16, (0, 3)),
    ("wgsl_rtiow_16x8", scene.rtiow_final_scene, 16, 8, (0, 5)),
    # W*H = 800: the reference's floor(800/128) = 6 workgroups trace the first
    # 768 pixels only (D1); the test compares those
    ("wgsl_config1_40x20_ragged", scene.config1_scene, 40, 20, (0, 2)),
    # the headline scene (BASELINE configs[1]) at 64x36 (18 workgroups, no
    # floor remainder), 5 frames incl. >= 1000: 11,520 pixels of the
    # reference's own kernels on the dielectric / metal / Lambertian mix
    ("wgsl_rtiow_64x36", scene.rtiow_final_scene, 64, 36, (0, 1, 17, 1000, 4096)),
    # consecutive frames 0..7: the reference renders one sample per frame
    # (SAMPLES_PER_RAY = 1); an 8-spp render of this build is the blocked f32
    # sum of exactly these frames / 8 (rt_hip.h RT_SAMPLE_BLOCK), which the
    # accumulation tests check against these reference-executed frames
    ("wgsl_rtiow_32x16_accum8", scene.rtiow_final_scene, 32, 16, tuple(range(8))),
]

# Deeper schedules: the reference hard-codes 3 (intersect, shade) rounds
# (ray_trace_node.rs:213) and the kill of a hit at bounce 2 (shade.wgsl:236,
# `r.bounces == 2u`); this build's max_depth D generalises both. These
# fixtures run the reference's own shaders with exactly that one constant
# substituted (`2u` -> `D-1`, asserted to occur once) and D rounds -- the
# reference code, generalised the way rt_params.max_depth is defined.
DEEP_CASES = [
    # name, scene, W, H, frames, D
    ("wgsl_config1_32x16_d16", scene.config1_scene, 32, 16, (0, 5, 1000), 16),
    ("wgsl_rtiow_32x16_d16", scene.rtiow_final_scene, 32, 16, (0, 2, 999), 16),
]
KILL_TEXT = "r.bounces == 2u"


def deep_shade_source(src, depth):
    assert src.count(KILL_TEXT) == 1, "shade.wgsl's bounce kill changed"
    return src.replace(KILL_TEXT, f"r.bounces == {depth - 1}u")


def run_reference(shaders, cam_bytes, sph_bytes, mat_bytes, width, height, frame,
                  loops=BOUNCE_LOOPS):
    """One frame of RayTraceNode::run through the interpreted WGSL."""
    R = width * height
    groups = R // WORKGROUP  # ray_trace_node.rs:37-38 (floor)
    first = shaders["clear"]
    globals_ = first.decode(first.var_type("globals"),
                            struct.pack("<9I", frame, width, height, 1, 0, 0, 0, 0, 0))
    rays = first.decode(first.var_type("ray_buffer"),
                        struct.pack("<I12x", R) + bytes(48 * R))
    isect = first.decode(first.var_type("intersection_buffer"), bytes(64 * R))
    out = np.zeros((height, width, 4), np.float32)
    for sh in shaders.values():
        res = {}
        for name in sh.m["vars"]:
            ty = sh.var_type(name)
            if name == "camera":
                res[name] = sh.decode(ty, cam_bytes)
            elif name == "globals":
                res[name] = globals_
            elif name == "ray_buffer":
                res[name] = rays
            elif name == "intersection_buffer":
                res[name] = isect
            elif name == "objects":
                res[name] = sh.decode(ty, struct.pack("<I12x", len(sph_bytes) // 32) + sph_bytes)
            elif name == "materials":
                res[name] = sh.decode(ty, mat_bytes)
            elif name == "output":
                res[name] = out
            else:
                raise KeyError(name)
        sh.bind(**res)
    shaders["clear"].dispatch("main", groups, WORKGROUP)
    shaders["generate"].dispatch("main", groups, WORKGROUP)
    for _ in range(loops):
        shaders["prepass"].dispatch("main", 1, 1)
        shaders["intersect"].dispatch("main", groups, WORKGROUP)
        shaders["shade"].dispatch("main", groups, WORKGROUP)
    shaders["collect"].dispatch("main", groups, WORKGROUP)
    return out


ISECT_CASES = [
    # name, scene, number of adversarial rays (tests/raygen.py)
    ("wgsl_isect_config1", scene.config1_scene, 2048),
    ("wgsl_isect_reference", scene.reference_scene, 512),
    ("wgsl_isect_rtiow", scene.rtiow_final_scene, 256),
    # BASELINE configs[4]'s 10,000-sphere list (streamed, not staged)
    ("wgsl_isect_spheres10k", scene.ten_thousand_scene, 384),
]


def run_intersect_world(sh, sph_bytes, rays):
    """intersect.wgsl's intersect_world (:133-143) for each ray (min EPSILON,
    max VERY_FAR, as generate.wgsl:82 / shade.wgsl:127 build them)."""
    sh.bind(objects=sh.decode(sh.var_type("objects"),
                              struct.pack("<I12x", len(sph_bytes) // 32) + sph_bytes))
    eps, far = sh.consts["EPSILON"], sh.consts["VERY_FAR"]
    out = {"t": [], "material": [], "front_face": [], "position": [], "normal": []}
    with np.errstate(all="ignore"):
        for r in rays:
            ray = W.Struct("ray", {"origin": W.Vec(W.F32(v) for v in r[:3]), "min": eps,
                                   "dir": W.Vec(W.F32(v) for v in r[3:]), "max": far,
                                   "pixel": W.U32(0), "bounces": W.U32(0)})
            hit = sh.call(("call", "intersect_world", (), [("lit", ray)]), [{}]).f
            out["t"].append(hit["t"])
            out["material"].append(int(hit["material"]))
            out["front_face"].append(int(hit["front_face"]))
            out["position"].append([float(v) for v in hit["position"]])
            out["normal"].append([float(v) for v in hit["normal"]])
    return {k: np.array(v, np.float32 if k in ("t", "position", "normal") else np.uint32)
            for k, v in out.items()}


_REF = "/root/reference"


def ALL_CASES():
    """(name, scene, W, H, frames, depth) of every frame fixture."""
    return [c + (BOUNCE_LOOPS,) for c in CASES] + list(DEEP_CASES)


def _shaders(ref, depth=BOUNCE_LOOPS):
    srcs = {k: open(os.path.join(ref, "assets", "shaders", k + ".wgsl")).read() for k in KERNELS}
    if depth != BOUNCE_LOOPS:
        srcs["shade"] = deep_shade_source(srcs["shade"], depth)
    return {k: W.Shader(srcs[k]) for k in KERNELS}


def _frame_job(args):
    """One frame of one case (a worker process: frames are independent)."""
    ref, name, f = args
    _, mk, w, h, _, depth = next(c for c in ALL_CASES() if c[0] == name)
    sc = mk()
    sp, mt = sc.objects_gpu(), sc.materials_gpu()
    t0 = time.time()
    img = run_reference(_shaders(ref, depth), default_camera_block().tobytes(), sp.tobytes(),
                        mt.tobytes(), w, h, f, loops=depth)
    print(f"{name} frame {f}: {time.time() - t0:.1f} s", flush=True)
    return img


def _isect_job(args):
    """A slice of one intersect_world ray set (a worker process)."""
    ref, name, lo, hi = args
    _, mk, n = next(c for c in ISECT_CASES if c[0] == name)
    from raygen import adversarial_rays
    sp = mk().objects_gpu()
    rays = adversarial_rays(sp, n, seed=7)[lo:hi]
    return run_intersect_world(_shaders(ref)["intersect"], sp.tobytes(), rays)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=_REF)
    ap.add_argument("--only", default="")
    ap.add_argument("--jobs", type=int, default=1, help="worker processes")
    a = ap.parse_args()
    from multiprocessing import Pool
    pool = Pool(a.jobs) if a.jobs > 1 else None
    run = pool.map if pool else lambda fn, xs: [fn(x) for x in xs]
    cam = default_camera_block()
    for name, mk, w, h, frames, depth in ALL_CASES():
        if a.only and a.only != name:
            continue
        sc = mk()
        sp, mt = sc.objects_gpu(), sc.materials_gpu()
        imgs = run(_frame_job, [(a.ref, name, f) for f in frames])
        np.savez_compressed(os.path.join(HERE, name + ".npz"),
                            spheres=np.frombuffer(sp.tobytes(), np.uint8),
                            materials=np.frombuffer(mt.tobytes(), np.uint8),
                            camera=np.frombuffer(cam.tobytes(), np.uint8),
                            params=np.array([w, h, 1, depth], np.uint32),
                            frames=np.array(frames, np.uint32),
                            processed=np.array([(w * h) // WORKGROUP * WORKGROUP], np.uint32),
                            images=np.stack(imgs))
    from raygen import adversarial_rays
    for name, mk, n in ISECT_CASES:
        if a.only and a.only != name:
            continue
        sc = mk()
        sp, mt = sc.objects_gpu(), sc.materials_gpu()
        rays = adversarial_rays(sp, n, seed=7)
        t0 = time.time()
        step = -(-n // max(1, a.jobs))
        parts = run(_isect_job, [(a.ref, name, lo, min(n, lo + step)) for lo in range(0, n, step)])
        res = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
        print(f"{name}: {n} rays {time.time() - t0:.1f} s", flush=True)
        np.savez_compressed(os.path.join(HERE, name + ".npz"),
                            spheres=np.frombuffer(sp.tobytes(), np.uint8),
                            materials=np.frombuffer(mt.tobytes(), np.uint8), rays=rays, **res)


if __name__ == "__main__":
    main()
