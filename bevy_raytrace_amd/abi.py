"""ctypes binding of the C-ABI in include/rt_hip.h (librt_hip.so).

The numpy dtypes below are byte-for-byte the reference's GPU layouts:
  SPHERE_DTYPE   = SphereGPU   (src/sphere.rs:12-17), 32 B
  MATERIAL_DTYPE = MaterialGPU (src/ray_trace_materials.rs:33-43), 32 B
  CAMERA_DTYPE   = CameraGPU   (src/ray_trace_camera.rs:14-25), 128 B std140

The library is loaded from the package directory only (built in-tree by
`__graft_entry__.build()`); if it is missing, `load()` raises — there is no CPU
fallback in the product path.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "librt_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "rt_hip.h")

RT_OK = 0
RT_ERR_INVALID_ARG = -1
RT_ERR_NO_SCENE = -2
RT_ERR_DEVICE = -3
RT_ERR_OUT_OF_MEMORY = -4
RT_ERR_BAD_SCENE = -5

RT_LAMBERTIAN = 0
RT_METALLIC = 1
RT_DIELECTRIC = 2

RT_SAMPLE_BLOCK = 8
RT_FLAG_NO_PRIMARY_CACHE = 0x1
RT_FLAG_JITTER = 0x2             # opt-in sub-pixel jitter (include/rt_hip.h)
RT_FLAG_THIN_LENS = 0x4          # opt-in thin-lens sample (generate.wgsl:85-107)
RT_FLAG_CULL = 0x8               # culled list: group bounds, identical hits (include/rt_hip.h)
RT_FLAG_VALU_FILTER = 0x10       # packed-fp32 VALU filter instead of the matrix-core one (identical hits)
RT_FLAG_IMAGE_OUT = 0x20         # device output in the image layout (owned rows at their image rows)
RT_MAX_PENDING = 2          # frames in flight per ctx (rt_render_device / rt_render_async)

SPHERE_DTYPE = np.dtype(
    [("center", "<f4", (3,)), ("radius", "<f4"), ("material", "<u4"), ("_pad", "<u4", (3,))]
)
MATERIAL_DTYPE = np.dtype(
    [("color", "<f4", (4,)), ("reflectance", "<i4"), ("fuzziness", "<f4"),
     ("index_of_refraction", "<f4"), ("_pad", "<i4")]
)
CAMERA_DTYPE = np.dtype(
    [("transform", "<f4", (16,)),
     ("forward", "<f4", (3,)), ("fov", "<f4"),
     ("up", "<f4", (3,)), ("image_plane_distance", "<f4"),
     ("right", "<f4", (3,)), ("lens_focal_length", "<f4"),
     ("position", "<f4", (3,)), ("fstop", "<f4")]
)
assert SPHERE_DTYPE.itemsize == 32 and MATERIAL_DTYPE.itemsize == 32
assert CAMERA_DTYPE.itemsize == 128


class RtParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                ("spp", ctypes.c_uint32), ("max_depth", ctypes.c_uint32),
                ("frame0", ctypes.c_uint32), ("row_block", ctypes.c_uint32),
                ("shard_count", ctypes.c_uint32), ("shard_index", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("_reserved", ctypes.c_uint32 * 3)]


class RtStats(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_uint64), ("traced_segments", ctypes.c_uint64),
                ("sphere_tests", ctypes.c_uint64), ("paths", ctypes.c_uint64),
                ("kernel_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("kernel_launches", ctypes.c_uint32), ("short_math", ctypes.c_uint32),
                ("clock_ghz", ctypes.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if not k.startswith("_")}


assert ctypes.sizeof(RtParams) == 48
assert ctypes.sizeof(RtStats) == 64


class RayTraceError(RuntimeError):
    """Raised for a negative status from the C-ABI (message from rt_last_error)."""

    def __init__(self, status, message):
        super().__init__(f"rt status {status}: {message}")
        self.status = status


def make_params(width, height, spp, max_depth, frame0=0, row_block=8, shard_count=1,
                shard_index=0, flags=0):
    p = RtParams()
    p.width, p.height, p.spp, p.max_depth = int(width), int(height), int(spp), int(max_depth)
    p.frame0, p.row_block = int(frame0), int(row_block)
    p.shard_count, p.shard_index, p.flags = int(shard_count), int(shard_index), int(flags)
    return p


def shard_rows(height, row_block, shard_count, shard_index):
    """Rows owned by a shard, increasing y (mirror of rt_shard_rows)."""
    B = max(1, int(row_block))
    K = max(1, int(shard_count))
    return [y for y in range(int(height)) if block_owner(y // B, K) == int(shard_index)]


def block_owner(b, K):
    """Row block b -> owning shard: groups of K blocks dealt serpentine
    (rt_hip.h rt_params; rt_internal.h rt_block_owner)."""
    g, i = divmod(int(b), int(K))
    return K - 1 - i if g & 1 else i


_VP = ctypes.c_void_p
_U32 = ctypes.c_uint32
_PROTOS = {
    "rt_version": (ctypes.c_int, []),
    "rt_shard_rows": (_U32, [_U32, _U32, _U32, _U32]),
    "rt_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_VP)]),
    "rt_destroy": (None, [_VP]),
    "rt_set_scene": (ctypes.c_int, [_VP, _VP, _U32, _VP, _U32]),
    "rt_render": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(RtParams), _VP, ctypes.POINTER(RtStats)]),
    "rt_render_device": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(RtParams), _VP, _VP]),
    "rt_render_frames_device": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(RtParams), ctypes.c_uint32,
                                               _VP, _VP]),
    "rt_reserve": (ctypes.c_int, [_VP, ctypes.POINTER(RtParams), ctypes.c_uint32]),
    "rt_render_async": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(RtParams), _VP]),
    "rt_host_register": (ctypes.c_int, [_VP, _VP, ctypes.c_size_t]),
    "rt_host_unregister": (ctypes.c_int, [_VP, _VP]),
    "rt_wait": (ctypes.c_int, [_VP, ctypes.POINTER(RtStats)]),
    "rt_assemble_shards": (ctypes.c_int, [_VP, _VP, _U32, _VP, _U32, _U32, _U32, _U32, _VP]),
    "rt_assemble_shard_frames": (ctypes.c_int,
                                 [_VP, _VP, _U32, _U32, _VP, _U32, _U32, _U32, _U32, _VP]),
    "rt_intersect": (ctypes.c_int, [_VP, _VP, _U32, _VP, _VP]),
    "rt_intersect_ex": (ctypes.c_int, [_VP, _VP, _U32, _U32, _VP, _VP]),
    "rt_update_spheres": (ctypes.c_int, [_VP, _U32, _VP, _U32]),
    "rt_render_progressive": (ctypes.c_int, [_VP, _VP, ctypes.POINTER(RtParams), ctypes.c_int, _VP,
                                             ctypes.POINTER(ctypes.c_uint64)]),
    "rt_encode_srgb8": (ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint64, _VP]),
    "rt_update_materials": (ctypes.c_int, [_VP, _U32, _VP, _U32]),
    "rt_acquire": (ctypes.c_int, [_VP, _VP]),
    "rt_last_error": (ctypes.c_char_p, [_VP]),
}

_libs = {}


def header_symbols(path=HEADER_PATH):
    """Function names declared in include/rt_hip.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z_]+)\s*\(", text)))


def _share_torch_hip_runtime():
    """One HIP runtime per process. PyTorch-ROCm bundles its own libamdhip64
    (SONAME libamdhip64.so.7, loaded by path from torch/lib); librt_hip.so
    needs libamdhip64.so.7. Pre-loading torch's copy RTLD_GLOBAL makes our
    library bind to it, so device pointers, streams and the device list are
    shared with torch whichever of the two is imported first."""
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    cand = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so")
    if os.path.exists(cand):
        ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)


def load(path=None):
    """Load librt_hip.so (raises if it was not built — no fallback).
    `path` selects another build of the same ABI (e.g. a diagnostic build)."""
    path = os.path.abspath(path or LIB_PATH)
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(
            f"{path} is missing: build the HIP library first (python -c "
            "'import __graft_entry__ as g; g.build()'). There is no CPU fallback.")
    _share_torch_hip_runtime()
    lib = ctypes.CDLL(path)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name, None)
        if fn is None:  # an older diagnostic build (tools/); the product exports all
            continue
        fn.restype = res
        fn.argtypes = args
    if hasattr(lib, "rt_debug_math"):  # internal diagnostic symbol (tests/test_gpu_math.py)
        lib.rt_debug_math.restype = ctypes.c_int
        lib.rt_debug_math.argtypes = [ctypes.c_int, _VP, ctypes.c_uint32, _VP]
    if hasattr(lib, "rt_debug_mfma_acc"):  # internal (tests/test_gpu_mfma_acc.py)
        lib.rt_debug_mfma_acc.restype = ctypes.c_int
        lib.rt_debug_mfma_acc.argtypes = [_VP, _VP, _VP, ctypes.c_uint32]
    if hasattr(lib, "rt_debug_counters"):  # internal diagnostic symbol
        lib.rt_debug_counters.restype = ctypes.c_int
        lib.rt_debug_counters.argtypes = [_VP, ctypes.POINTER(ctypes.c_uint64)]
    if hasattr(lib, "rt_debug_counters32"):  # internal diagnostic symbol (RT_PROFILE builds)
        lib.rt_debug_counters32.restype = ctypes.c_int
        lib.rt_debug_counters32.argtypes = [_VP, ctypes.POINTER(ctypes.c_uint64)]
    if hasattr(lib, "rt_debug_intersect_tiles"):  # internal (tests/test_gpu_intersect.py)
        lib.rt_debug_intersect_tiles.restype = ctypes.c_int
        lib.rt_debug_intersect_tiles.argtypes = [_VP, ctypes.POINTER(ctypes.c_uint64)]
    if hasattr(lib, "rt_debug_tune"):  # internal A/B knobs (tests, tools/)
        lib.rt_debug_tune.restype = ctypes.c_int
        lib.rt_debug_tune.argtypes = [_VP, ctypes.c_char_p, ctypes.c_char_p]
    if hasattr(lib, "rt_debug_alloc_count"):  # internal (tests)
        lib.rt_debug_alloc_count.restype = ctypes.c_uint64
        lib.rt_debug_alloc_count.argtypes = [_VP]
    if hasattr(lib, "rt_debug_mf_rebuilds"):  # internal (tests/test_gpu_parity.py)
        lib.rt_debug_mf_rebuilds.restype = ctypes.c_int
        lib.rt_debug_mf_rebuilds.argtypes = [_VP, ctypes.POINTER(ctypes.c_uint64)]
    if hasattr(lib, "rt_debug_mf_update"):  # internal, host only (tests/test_scene_update.py)
        lib.rt_debug_mf_update.restype = ctypes.c_int
        lib.rt_debug_mf_update.argtypes = [_VP, _U32, _VP, _VP, _U32, _VP]
    if hasattr(lib, "rt_debug_cull_layout"):  # internal, host only (tests/test_cull.py)
        lib.rt_debug_cull_layout.restype = ctypes.c_int
        lib.rt_debug_cull_layout.argtypes = [_VP, _U32, _VP, _VP, _U32, _VP, _U32]
    _libs[path] = lib
    return lib


def cull_layout(spheres, lib=None):
    """The culled list the library builds for RT_FLAG_CULL (host only, no
    device): (perm, group_bounds, cluster_bounds, ngroups, nclusters).
    perm[p] = original index of permuted position p (-1 = pad); bounds are
    (n, 4) rows (Cx, Cy, Cz, S_B): one per group slot (nclusters * 8) and one
    per cluster slot (supers * 8)."""
    import numpy as np
    lib = lib or load()
    sp = np.ascontiguousarray(spheres)
    n = len(sp)
    counts = (ctypes.c_uint32 * 4)()
    ptr = sp.ctypes.data_as(_VP) if n else None
    if lib.rt_debug_cull_layout(ptr, n, counts, None, 0, None, 0) != 0:
        raise RuntimeError("rt_debug_cull_layout failed")
    ng, nc, nrec, ns = counts[0], counts[1], counts[2], counts[3]
    perm = np.empty(nrec, dtype=np.uint32)
    bnd = np.empty((ns + nc) * 32, dtype=np.float32)
    if lib.rt_debug_cull_layout(ptr, n, counts, perm.ctypes.data_as(_VP), nrec,
                                bnd.ctypes.data_as(_VP), (ns + nc) * 32) != 0:
        raise RuntimeError("rt_debug_cull_layout failed")
    b = bnd.reshape(ns + nc, 4, 8).transpose(0, 2, 1).reshape((ns + nc) * 8, 4)
    perm = perm.astype(np.int64) - (perm == 0xFFFFFFFF) * (1 << 32)
    return perm, b[ns * 8:], b[:ns * 8], ng, nc


def check(lib, ctx, status):
    if status != RT_OK:
        msg = lib.rt_last_error(ctx)
        raise RayTraceError(status, msg.decode() if msg else "")
    return status
