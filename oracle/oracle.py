"""ctypes wrapper of the C oracle (oracle/build/librt_oracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py. The product package never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "librt_oracle.so")

_lib = None


def default_threads():
    """Threads the oracle runs on by default: the CPUs this process may use,
    capped by the cgroup CPU quota (the GPU box shows 256 cores under a 16-CPU
    quota; more threads than the quota only time-slice)."""
    n = len(os.sched_getaffinity(0)) or os.cpu_count() or 1
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return n


class _Params(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                ("spp", ctypes.c_uint32), ("max_depth", ctypes.c_uint32),
                ("frame0", ctypes.c_uint32), ("row_block", ctypes.c_uint32),
                ("shard_count", ctypes.c_uint32), ("shard_index", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("_reserved", ctypes.c_uint32 * 3)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        vp, u32, fp = ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_float)
        lib.rto_hash3.argtypes = [u32, fp]
        lib.rto_tan_half.argtypes = [ctypes.c_float]
        lib.rto_tan_half.restype = ctypes.c_float
        lib.rto_primary_ray.argtypes = [vp, u32, u32, u32, u32, fp, fp]
        lib.rto_sky.argtypes = [fp, fp]
        lib.rto_sincos.argtypes = [ctypes.c_float, fp, fp]
        lib.rto_intersect.argtypes = [vp, u32, fp, fp, fp, fp, fp, ctypes.POINTER(u32)]
        lib.rto_intersect.restype = ctypes.c_int
        lib.rto_intersect_batch.argtypes = [vp, u32, vp, u32, vp, vp, ctypes.c_int]
        lib.rto_trace_path.argtypes = [vp, vp, u32, vp, u32, u32, u32, u32, u32, u32, u32, fp,
                                       ctypes.POINTER(u32)]
        lib.rto_render.argtypes = [vp, vp, u32, vp, u32, ctypes.POINTER(_Params), vp,
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
        lib.rto_render.restype = ctypes.c_int
        lib.rto_render_rows.argtypes = [vp, vp, u32, vp, u32, ctypes.POINTER(_Params), vp, u32, vp,
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
        lib.rto_render_rows.restype = ctypes.c_int
        _lib = lib
    return _lib


def _f3(a=None):
    return (ctypes.c_float * 3)(*(a if a is not None else (0.0, 0.0, 0.0)))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None and a.size else None


def hash3(n):
    out = _f3()
    load().rto_hash3(n, out)
    return np.array(out[:], dtype=np.float32)


def tan_half(fov):
    return np.float32(load().rto_tan_half(fov))


def primary_ray(cam, width, height, x, y):
    cam = np.ascontiguousarray(cam)
    o, d = _f3(), _f3()
    load().rto_primary_ray(cam.ctypes.data_as(ctypes.c_void_p), width, height, x, y, o, d)
    return np.array(o[:], np.float32), np.array(d[:], np.float32)


def sincos(theta):
    """rt_sincos of the opt-in thin-lens sampling (include/rt_hip.h)."""
    s, c = ctypes.c_float(0), ctypes.c_float(0)
    load().rto_sincos(float(theta), ctypes.byref(s), ctypes.byref(c))
    return np.float32(s.value), np.float32(c.value)


def sky(d):
    out = _f3()
    load().rto_sky(_f3(d), out)
    return np.array(out[:], np.float32)


def intersect_batch(spheres, rays, nthreads=None):
    """rays (n, 6) float32 -> (index int32, t float32), intersect.wgsl:133-143."""
    r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
    idx = np.empty(r.shape[0], np.int32)
    t = np.empty(r.shape[0], np.float32)
    load().rto_intersect_batch(_ptr(spheres), len(spheres), r.ctypes.data_as(ctypes.c_void_p),
                               r.shape[0], idx.ctypes.data_as(ctypes.c_void_p),
                               t.ctypes.data_as(ctypes.c_void_p), nthreads or default_threads())
    return idx, t


def trace_path(cam, spheres, materials, width, height, x, y, frame, max_depth):
    cam = np.ascontiguousarray(cam)
    out, segs = _f3(), ctypes.c_uint32(0)
    load().rto_trace_path(cam.ctypes.data_as(ctypes.c_void_p), _ptr(spheres), len(spheres),
                          _ptr(materials), len(materials), width, height, x, y, frame,
                          max_depth, out, ctypes.byref(segs))
    return np.array(out[:], np.float32), segs.value


RAW_SUMS = 0x80000000


def _block_owner(b, K):
    """Row block -> shard, serpentine (mirror of rto_block_owner)."""
    g, i = divmod(b, K)
    return K - 1 - i if g & 1 else i


def _params(width, height, spp, max_depth, frame0, row_block, shard_count, shard_index, flags=0):
    p = _Params()
    p.width, p.height, p.spp, p.max_depth = width, height, spp, max_depth
    p.frame0, p.row_block, p.shard_count, p.shard_index = frame0, row_block, shard_count, shard_index
    p.flags = flags
    return p


def render(cam, spheres, materials, width, height, spp, max_depth, frame0=0, row_block=8,
           shard_count=1, shard_index=0, nthreads=None, raw_sums=False, flags=0):
    """Render the shard's rows -> (rows, W, 4) float32, segments.
    raw_sums: the block-folded sample sums instead of sum / spp (alpha 0)."""
    cam = np.ascontiguousarray(cam)
    nthreads = nthreads or default_threads()
    B = max(1, row_block)
    nrows = sum(1 for y in range(height)
                if _block_owner(y // B, shard_count) == shard_index)
    out = np.zeros((nrows, width, 4), dtype=np.float32)
    segs = ctypes.c_uint64(0)
    p = _params(width, height, spp, max_depth, frame0, row_block, shard_count, shard_index,
                (RAW_SUMS if raw_sums else 0) | flags)
    rc = load().rto_render(cam.ctypes.data_as(ctypes.c_void_p), _ptr(spheres), len(spheres),
                           _ptr(materials), len(materials), ctypes.byref(p),
                           out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(segs), nthreads)
    if rc != 0:
        raise ValueError("oracle rejected the arguments")
    return out, segs.value


def render_rows(cam, spheres, materials, width, height, spp, max_depth, rows, frame0=0,
                nthreads=None, flags=0):
    cam = np.ascontiguousarray(cam)
    nthreads = nthreads or default_threads()
    rows = np.ascontiguousarray(rows, dtype=np.uint32)
    out = np.zeros((rows.size, width, 4), dtype=np.float32)
    segs = ctypes.c_uint64(0)
    p = _params(width, height, spp, max_depth, frame0, 1, 1, 0, flags)
    rc = load().rto_render_rows(cam.ctypes.data_as(ctypes.c_void_p), _ptr(spheres), len(spheres),
                                _ptr(materials), len(materials), ctypes.byref(p),
                                rows.ctypes.data_as(ctypes.c_void_p), rows.size,
                                out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(segs), nthreads)
    if rc != 0:
        raise ValueError("oracle rejected the arguments")
    return out, segs.value
