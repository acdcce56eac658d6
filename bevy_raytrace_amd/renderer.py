"""Host-side handle on one GPU: a thin owner of an `rt_ctx*` (include/rt_hip.h).

This is the Python mirror of what the reference's render-world resources and
RayTraceNode do per frame (src/plugin.rs:25-122, src/ray_trace_node.rs:195-224):
upload the scene once, then render frames from a camera block + parameters.
All compute happens in librt_hip.so on the GPU; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import abi
from .abi import RtStats, check, make_params


class Renderer:
    def __init__(self, device: int = 0, lib_path=None):
        self.lib = abi.load(lib_path)
        ctx = ctypes.c_void_p()
        rc = self.lib.rt_create(int(device), ctypes.byref(ctx))
        check(self.lib, None, rc)
        self.ctx = ctx
        self.device = int(device)
        self._keep = None
        self.n_spheres = 0

    def close(self):
        if self.ctx:
            self.lib.rt_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- scene
    def set_scene(self, spheres: np.ndarray, materials: np.ndarray):
        sp = np.ascontiguousarray(spheres, dtype=abi.SPHERE_DTYPE)
        mt = np.ascontiguousarray(materials, dtype=abi.MATERIAL_DTYPE)
        rc = self.lib.rt_set_scene(self.ctx, sp.ctypes.data_as(ctypes.c_void_p) if sp.size else None,
                                   sp.size, mt.ctypes.data_as(ctypes.c_void_p) if mt.size else None,
                                   mt.size)
        check(self.lib, self.ctx, rc)
        self.n_spheres = int(sp.size)

    def update_spheres(self, first: int, spheres: np.ndarray):
        sp = np.ascontiguousarray(spheres, dtype=abi.SPHERE_DTYPE)
        rc = self.lib.rt_update_spheres(self.ctx, int(first), sp.ctypes.data_as(ctypes.c_void_p),
                                        sp.size)
        check(self.lib, self.ctx, rc)

    def update_materials(self, first: int, materials: np.ndarray):
        mt = np.ascontiguousarray(materials, dtype=abi.MATERIAL_DTYPE)
        rc = self.lib.rt_update_materials(self.ctx, int(first), mt.ctypes.data_as(ctypes.c_void_p),
                                          mt.size)
        check(self.lib, self.ctx, rc)

    # --------------------------------------------------------------- render
    def render(self, camera: np.ndarray, width, height, spp, max_depth, frame0=0, row_block=8,
               shard_count=1, shard_index=0, flags=0):
        """Synchronous render to a host array (rows, W, 4) float32 + stats dict."""
        cam = np.ascontiguousarray(camera, dtype=abi.CAMERA_DTYPE)
        p = make_params(width, height, spp, max_depth, frame0, row_block, shard_count, shard_index,
                        flags)
        rows = self.lib.rt_shard_rows(p.height, p.row_block, max(1, p.shard_count), p.shard_index)
        out = np.empty((rows, int(width), 4), dtype=np.float32)
        st = RtStats()
        rc = self.lib.rt_render(self.ctx, cam.ctypes.data_as(ctypes.c_void_p), ctypes.byref(p),
                                out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(st))
        check(self.lib, self.ctx, rc)
        return out, st.as_dict()

    def render_progressive(self, camera: np.ndarray, width, height, spp, max_depth, frame0=0,
                           reset=False, row_block=8, shard_count=1, shard_index=0, flags=0):
        """Render spp more samples into the device running sum; returns the
        running mean image (rows, W, 4) and the total samples so far."""
        cam = np.ascontiguousarray(camera, dtype=abi.CAMERA_DTYPE)
        p = make_params(width, height, spp, max_depth, frame0, row_block, shard_count, shard_index,
                        flags)
        rows = self.lib.rt_shard_rows(p.height, p.row_block, max(1, p.shard_count), p.shard_index)
        out = np.empty((rows, int(width), 4), dtype=np.float32)
        total = ctypes.c_uint64(0)
        rc = self.lib.rt_render_progressive(self.ctx, cam.ctypes.data_as(ctypes.c_void_p),
                                            ctypes.byref(p), 1 if reset else 0,
                                            out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(total))
        check(self.lib, self.ctx, rc)
        return out, int(total.value)

    def encode_srgb8(self, rgba_ptr: int, out_ptr: int, npix: int, stream=None):
        """Device Rgba32Float -> device sRGB RGBA8."""
        rc = self.lib.rt_encode_srgb8(self.ctx, ctypes.c_void_p(int(rgba_ptr)),
                                      ctypes.c_void_p(int(out_ptr)), int(npix),
                                      ctypes.c_void_p(int(stream)) if stream else None)
        check(self.lib, self.ctx, rc)

    def acquire(self, stream=None):
        """System-scope acquire on this device (rt_acquire): after other ranks
        wrote their rows into this device's image (RT_FLAG_IMAGE_OUT) and the
        host saw them complete, work enqueued after this on `stream` reads them."""
        rc = self.lib.rt_acquire(self.ctx, ctypes.c_void_p(int(stream)) if stream else None)
        check(self.lib, self.ctx, rc)

    def render_device(self, camera: np.ndarray, out_ptr: int, width, height, spp, max_depth,
                      frame0=0, row_block=8, shard_count=1, shard_index=0, flags=0, stream=None):
        """Enqueue a render into a device buffer (e.g. a torch tensor's data_ptr()).

        `stream` is a raw hipStream_t handle (int) or None for the ctx stream.
        Call wait() for the stats.
        """
        cam = np.ascontiguousarray(camera, dtype=abi.CAMERA_DTYPE)
        p = make_params(width, height, spp, max_depth, frame0, row_block, shard_count, shard_index,
                        flags)
        self._keep = (cam, p)
        rc = self.lib.rt_render_device(self.ctx, cam.ctypes.data_as(ctypes.c_void_p),
                                       ctypes.byref(p), ctypes.c_void_p(int(out_ptr)),
                                       ctypes.c_void_p(int(stream)) if stream else None)
        check(self.lib, self.ctx, rc)

    def render_frames_device(self, camera: np.ndarray, nframes: int, out_ptr: int, width, height,
                             spp, max_depth, frame0=0, row_block=8, shard_count=1, shard_index=0,
                             flags=0, stream=None):
        """Enqueue `nframes` frames (frame i = samples frame0 + i*spp ...) in one
        launch into consecutive device images at out_ptr. Call wait() for stats."""
        cam = np.ascontiguousarray(camera, dtype=abi.CAMERA_DTYPE)
        p = make_params(width, height, spp, max_depth, frame0, row_block, shard_count, shard_index,
                        flags)
        self._keep = (cam, p)
        rc = self.lib.rt_render_frames_device(self.ctx, cam.ctypes.data_as(ctypes.c_void_p),
                                              ctypes.byref(p), int(nframes),
                                              ctypes.c_void_p(int(out_ptr)),
                                              ctypes.c_void_p(int(stream)) if stream else None)
        check(self.lib, self.ctx, rc)

    def render_async(self, camera: np.ndarray, out: np.ndarray, width, height, spp, max_depth,
                     frame0=0, row_block=8, shard_count=1, shard_index=0, flags=0):
        """rt_render_async: enqueue one frame whose image lands in the HOST
        array `out` (rows, W, 4) float32 -- the Bevy shim's per-frame call
        (bevy_shim/src/ray_trace_node.rs). Call wait() before reading it."""
        cam = np.ascontiguousarray(camera, dtype=abi.CAMERA_DTYPE)
        p = make_params(width, height, spp, max_depth, frame0, row_block, shard_count, shard_index,
                        flags)
        rows = self.lib.rt_shard_rows(p.height, p.row_block, max(1, p.shard_count), p.shard_index)
        if out.dtype != np.float32 or not out.flags.c_contiguous or out.size < rows * int(width) * 4:
            raise ValueError("render_async: out must be a C-contiguous float32 array of "
                             f"{rows} x {width} x 4")
        self._keep_async = getattr(self, "_keep_async", [])[-1:] + [(cam, p, out)]
        rc = self.lib.rt_render_async(self.ctx, cam.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.byref(p), out.ctypes.data_as(ctypes.c_void_p))
        check(self.lib, self.ctx, rc)

    def host_register(self, arr: np.ndarray):
        """rt_host_register: page-lock a host array render_async writes (it
        must outlive the registration: host_unregister or close)."""
        check(self.lib, self.ctx, self.lib.rt_host_register(
            self.ctx, ctypes.c_void_p(arr.ctypes.data), arr.nbytes))

    def host_unregister(self, arr: np.ndarray):
        check(self.lib, self.ctx, self.lib.rt_host_unregister(self.ctx, ctypes.c_void_p(arr.ctypes.data)))

    def reserve(self, nframes, width, height, spp, max_depth, frame0=0, row_block=8,
                shard_count=1, shard_index=0, flags=0):
        """Allocate the work buffers of a render_frames_device(nframes, ...) in
        every in-flight slot now (rt_reserve), so later renders allocate nothing."""
        p = make_params(width, height, spp, max_depth, frame0, row_block, shard_count, shard_index,
                        flags)
        check(self.lib, self.ctx, self.lib.rt_reserve(self.ctx, ctypes.byref(p), int(nframes)))

    def wait(self):
        st = RtStats()
        rc = self.lib.rt_wait(self.ctx, ctypes.byref(st))
        check(self.lib, self.ctx, rc)
        return st.as_dict()

    def intersect(self, rays: np.ndarray, flags=0):
        """Closest hit for rays (n, 6) float32 [origin, direction] -> (index int32, t float32).
        flags: RT_FLAG_CULL traces the culled list (rt_intersect_ex; same hits)."""
        r = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 6)
        n = r.shape[0]
        idx = np.empty(n, dtype=np.int32)
        t = np.empty(n, dtype=np.float32)
        rc = self.lib.rt_intersect_ex(self.ctx, r.ctypes.data_as(ctypes.c_void_p), n, flags,
                                      idx.ctypes.data_as(ctypes.c_void_p),
                                      t.ctypes.data_as(ctypes.c_void_p))
        check(self.lib, self.ctx, rc)
        return idx, t

    def tune(self, name=None, value=None, **knobs):
        """Set A/B knobs of this context (internal rt_debug_tune; the product
        defaults need none): tune("scratch_bytes", 4096), tune(wide_max=0),
        tune(tail="0,0,6"). tune(None) restores every default."""
        if name is None and not knobs:
            check(self.lib, self.ctx, self.lib.rt_debug_tune(self.ctx, None, None))
            return
        if name is not None:
            knobs[name] = value
        for k, v in knobs.items():
            check(self.lib, self.ctx, self.lib.rt_debug_tune(self.ctx, str(k).encode(),
                                                            str(v).encode()))

    def alloc_count(self):
        """Device allocations this context has made (internal)."""
        return int(self.lib.rt_debug_alloc_count(self.ctx))

    def debug_counters(self):
        """Diagnostic counters of the last call (non-zero only for -DRT_PROFILE
        builds): 32 when the library has rt_debug_counters32, else 16."""
        if hasattr(self.lib, "rt_debug_counters32"):
            out = (ctypes.c_uint64 * 32)()
            self.lib.rt_debug_counters32(self.ctx, out)
        else:
            out = (ctypes.c_uint64 * 16)()
            self.lib.rt_debug_counters(self.ctx, out)
        return list(out)

    def intersect_tiles(self):
        """The last intersect()'s matrix-core walk: (block-half tiles walked,
        tiles without block bounds), summed over its waves; (0, 0) when it
        took the VALU walk or the culled list (internal diagnostic)."""
        out = (ctypes.c_uint64 * 2)()
        check(self.lib, self.ctx, self.lib.rt_debug_intersect_tiles(self.ctx, out))
        return int(out[0]), int(out[1])

    def assemble_shard_frames(self, gathered_ptr: int, max_rows, frames, image_ptr: int, width,
                              height, row_block, shard_count, stream=None):
        """rt_assemble_shard_frames: `frames` frames of (shard, frame)-ordered
        slabs in one launch."""
        rc = self.lib.rt_assemble_shard_frames(self.ctx, ctypes.c_void_p(int(gathered_ptr)),
                                               max_rows, frames, ctypes.c_void_p(int(image_ptr)),
                                               width, height, row_block, shard_count,
                                               ctypes.c_void_p(int(stream)) if stream else None)
        check(self.lib, self.ctx, rc)

    def assemble_shards(self, gathered_ptr: int, max_rows, image_ptr: int, width, height,
                        row_block, shard_count, stream=None):
        rc = self.lib.rt_assemble_shards(self.ctx, ctypes.c_void_p(int(gathered_ptr)), max_rows,
                                         ctypes.c_void_p(int(image_ptr)), width, height,
                                         row_block, shard_count,
                                         ctypes.c_void_p(int(stream)) if stream else None)
        check(self.lib, self.ctx, rc)
