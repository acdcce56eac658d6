"""Row-tiled multi-GPU rendering.

One process per GPU. Every pixel is independent (intersect/shade/collect are
index-local, intersect.wgsl:153-162, shade.wgsl:207-257, collect.wgsl:116-117;
the seed depends only on the GLOBAL pixel and frame, shade.wgsl:216-218), so
the image is split into blocks of `row_block` rows dealt to the ranks in
groups of `world`, serpentine (abi.block_owner: group g deals to ranks
0..world-1 when g is even, world-1..0 when odd). Each rank renders its rows into a slab padded to
`max_rows`; one gather (RCCL over xGMI for backend "nccl", gloo in CPU tests)
lands the slabs on rank 0, which re-assembles the image (rt_assemble_shards on
the device; `assemble_host` is the numpy statement of the same mapping) -- or,
with rank 0's image mapped into every rank (ipc_export / ipc_import), each
rank writes its rows straight into it (RT_FLAG_IMAGE_OUT) and nothing is
gathered.
The scene is replicated: every rank builds it from the same seed.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from .abi import block_owner, shard_rows


@dataclass(frozen=True)
class ShardLayout:
    height: int
    row_block: int
    world: int

    def rows(self, rank):
        return shard_rows(self.height, self.row_block, self.world, rank)

    @property
    def max_rows(self):
        return max(len(self.rows(k)) for k in range(self.world))

    def source_index(self, y):
        """(rank, local row) holding global row y."""
        blk = y // self.row_block
        return (block_owner(blk, self.world),
                (blk // self.world) * self.row_block + y % self.row_block)


def assemble_host(gathered: np.ndarray, layout: ShardLayout) -> np.ndarray:
    """gathered: (world, max_rows, W, 4) -> (H, W, 4); mirrors rt_assemble_kernel."""
    W = gathered.shape[2]
    out = np.empty((layout.height, W, gathered.shape[3]), dtype=gathered.dtype)
    for y in range(layout.height):
        k, r = layout.source_index(y)
        out[y] = gathered[k, r]
    return out


def gather_to_root(dist, slab, world, rank, like=None):
    """Gather equal-size slabs to rank 0. Returns the (world, ...) stack on
    rank 0, None elsewhere. `slab` is a torch tensor (CPU for gloo, device for
    nccl)."""
    import torch
    if rank == 0:
        parts = [torch.empty_like(slab) for _ in range(world)]
        dist.gather(slab, parts, dst=0)
        return torch.stack(parts, 0)
    dist.gather(slab, None, dst=0)
    return None


# ---- rank 0's image mapped into every rank (HIP IPC) ------------------------
# With RT_FLAG_IMAGE_OUT each rank writes its rows straight into rank 0's
# image at their image rows (over xGMI), so the row tiling needs no gather and
# no re-assembly. The handle names the allocation that holds
# the pointer; the offset of the pointer inside it travels with it.

class _IpcHandle(ctypes.Structure):
    # hipIpcMemHandle_t (HIP_IPC_HANDLE_SIZE); bytes, not c_char (a c_char
    # array reads back only up to its first NUL)
    _fields_ = [("reserved", ctypes.c_ubyte * 64)]


_HIP = None


def _hip():
    """The process's HIP runtime: torch's bundled libamdhip64 (the one
    librt_hip.so binds to, abi._share_torch_hip_runtime)."""
    global _HIP
    if _HIP is None:
        import importlib.util
        import os
        spec = importlib.util.find_spec("torch")
        cand = os.path.join(os.path.dirname(spec.origin), "lib", "libamdhip64.so") if spec else ""
        h = ctypes.CDLL(cand if cand and os.path.exists(cand) else "libamdhip64.so.7")
        h.hipIpcGetMemHandle.restype = ctypes.c_int
        h.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(_IpcHandle), ctypes.c_void_p]
        h.hipIpcOpenMemHandle.restype = ctypes.c_int
        h.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), _IpcHandle, ctypes.c_uint]
        h.hipIpcCloseMemHandle.restype = ctypes.c_int
        h.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
        h.hipMemGetAddressRange.restype = ctypes.c_int
        h.hipMemGetAddressRange.argtypes = [ctypes.POINTER(ctypes.c_void_p),
                                            ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
        h.hipDeviceCanAccessPeer.restype = ctypes.c_int
        h.hipDeviceCanAccessPeer.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                             ctypes.c_int]
        _HIP = h
    return _HIP


def ipc_export(ptr: int) -> bytes:
    """A device pointer as 72 bytes another process can map (ipc_import)."""
    h = _hip()
    base, size = ctypes.c_void_p(), ctypes.c_size_t()
    rc = h.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(ptr))
    if rc != 0:
        raise RuntimeError(f"hipMemGetAddressRange failed ({rc})")
    handle = _IpcHandle()
    rc = h.hipIpcGetMemHandle(ctypes.byref(handle), ctypes.c_void_p(base.value))
    if rc != 0:
        raise RuntimeError(f"hipIpcGetMemHandle failed ({rc})")
    return bytes(handle.reserved) + (ptr - base.value).to_bytes(8, "little")  # 64 + 8 bytes


def ipc_import(blob: bytes):
    """Map another process's pointer (ipc_export) into this one, on the
    current device: (mapping to close with ipc_close, the pointer)."""
    h = _hip()
    if len(blob) != 72:
        raise ValueError(f"ipc_import: {len(blob)}-byte blob (72 expected)")
    handle = _IpcHandle()
    ctypes.memmove(ctypes.addressof(handle), blob[:64], 64)
    base = ctypes.c_void_p()
    rc = h.hipIpcOpenMemHandle(ctypes.byref(base), handle, 1)  # hipIpcMemLazyEnablePeerAccess
    if rc != 0:
        raise RuntimeError(f"hipIpcOpenMemHandle failed ({rc})")
    return base.value, base.value + int.from_bytes(blob[64:72], "little")


def ipc_close(mapping: int):
    _hip().hipIpcCloseMemHandle(ctypes.c_void_p(mapping))


def can_access_peer(device: int, peer: int):
    """hipDeviceCanAccessPeer(device, peer): True / False, or None for the same
    device (a rehearsal with every rank on one GPU) or a failed query."""
    if device == peer:
        return None
    v = ctypes.c_int(0)
    rc = _hip().hipDeviceCanAccessPeer(ctypes.byref(v), int(device), int(peer))
    return None if rc != 0 else bool(v.value)


def check_rows(rows):
    """The rows the N>1 cross-rank check re-renders on rank 0: for every rank,
    its first, middle and last owned row (`rows[k]` = rank k's image rows in
    its order), each once -- the rows at both ends of every rank's shard."""
    out = []
    for k, rk in enumerate(rows):
        if not rk:
            continue
        for y in (rk[0], rk[len(rk) // 2], rk[-1]):
            if all(y != y2 for _, y2 in out):
                out.append((k, int(y)))
    return out
