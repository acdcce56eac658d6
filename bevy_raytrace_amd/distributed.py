"""Row-tiled multi-GPU rendering.

One process per GPU. Every pixel is independent (intersect/shade/collect are
index-local, intersect.wgsl:153-162, shade.wgsl:207-257, collect.wgsl:116-117;
the seed depends only on the GLOBAL pixel and frame, shade.wgsl:216-218), so
the image is split into blocks of `row_block` rows dealt to the ranks in
groups of `world`, serpentine (abi.block_owner: group g deals to ranks
0..world-1 when g is even, world-1..0 when odd). Each rank renders its rows into a slab padded to
`max_rows`; one gather (RCCL over xGMI for backend "nccl", gloo in CPU tests)
lands the slabs on rank 0, which re-assembles the image (rt_assemble_shards on
the device; `assemble_host` is the numpy statement of the same mapping).
The scene is replicated: every rank builds it from the same seed.
"""
from __future__ import annotations

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
