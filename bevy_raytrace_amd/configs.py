"""The BASELINE.json workloads."""
from __future__ import annotations

from dataclasses import dataclass

from . import scene as _scene

SCENE_SEED = 20221015


@dataclass(frozen=True)
class Workload:
    key: str
    width: int
    height: int
    spp: int
    max_depth: int
    scene: str        # scene factory name in bevy_raytrace_amd.scene
    gpus: int = 1
    note: str = ""

    def make_scene(self):
        return getattr(_scene, self.scene)(SCENE_SEED) if self.scene != "config1_scene" \
            else _scene.config1_scene()


WORKLOADS = {
    "config1": Workload("config1", 400, 225, 16, 8, "config1_scene", 1,
                        "ground + Lambertian + glass + metal; the reference's CPU-runnable case"),
    "rtiow1080": Workload("rtiow1080", 1920, 1080, 64, 16, "rtiow_final_scene", 1,
                          "RTIOW final scene, headline metric config (BASELINE.json configs[1])"),
    "rtiow4k": Workload("rtiow4k", 3840, 2160, 256, 32, "rtiow_final_scene", 1,
                        "same scene, 4K, 256 spp, depth 32"),
    "rtiow8k": Workload("rtiow8k", 7680, 4320, 1024, 16, "rtiow_final_scene", 8,
                        "same scene, 8K, 1024 spp, row-tiled over 8 GPUs"),
    "spheres10k1080": Workload("spheres10k1080", 1920, 1080, 128, 16, "ten_thousand_scene", 1,
                               "10,000 spheres, 128 spp (sphere list streamed)"),
    # the reference's own per-frame workload through the drop-in path:
    # RENDER_TARGET_SIZE 1920x1080, SAMPLES_PER_RAY 1 (src/lib.rs:25-26), 3
    # (intersect, shade) rounds (src/ray_trace_node.rs:213), its dim-7 scene
    # with its own material split (src/sphere.rs:48-91)
    "reference1080": Workload("reference1080", 1920, 1080, 1, 3, "reference_scene", 1,
                              "the reference's own frame: 1 spp, depth 3, dim-7 scene"),
}

HEADLINE = "rtiow1080"


def pick_row_block(height: int, shards: int, max_block: int = 8) -> int:
    """Row block of the N-way row tiling (interleaved blocks):
    single rows -- the finest serpentine deal, whose shards cost the most
    nearly the same (N=8 at 1080p/64: slowest shard 1.633 ms/frame with
    1-row blocks, 1.654 with 5-row blocks; spread 1.3 % vs 3.5 %; with the
    pixel-major work order a shard's tile shape no longer sets its waves'
    coherence) -- when they split the image evenly; otherwise
    the largest block <= max_block that does; otherwise max_block."""
    if shards > 1 and height % shards == 0:
        return 1
    for b in range(max_block, 0, -1):
        if height % b == 0 and (height // b) % shards == 0:
            return b
    return max_block
