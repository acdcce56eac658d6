"""Mirror of the reference's plugin surface for the hot path.

Reference (crate-private there, src/lib.rs:1-12):
  RayTracePlugin       src/plugin.rs:19-47   installs camera/globals/rays/... plugins + graph node
  RayTraceNode         src/ray_trace_node.rs:23-224  update() (pipeline readiness), run() (dispatch)
  RayTraceOutputImage  src/ray_trace_output.rs:19-20  Rgba32Float W x H storage texture
  GlobalsGPU.frame     src/ray_trace_globals.rs:56-68  frame counter = RNG seed input, +1 per frame
  SphereRenderPlugin   src/sphere.rs:150-164  spawns init_spheres, extracts ObjectListGPU

A `World` here is a plain resource map. RayTraceNode.update() creates the GPU
context and re-uploads the scene when it changed (the reference re-uploads
every frame, sphere.rs:180-197); run() renders one frame into the output image
and advances the frame counter. All rendering is librt_hip.so.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .camera import RayTraceCamera
from .renderer import Renderer
from .scene import MaterialCache, Scene, init_spheres

RENDER_TARGET_SIZE = (1920, 1080)   # src/lib.rs:25
SAMPLES_PER_RAY = 1                 # src/lib.rs:26
MAX_DEPTH = 3                       # src/ray_trace_node.rs:213 (3 x intersect/shade)


@dataclass
class RayTraceOutputImage:
    """The W x H Rgba32Float image (src/ray_trace_output.rs:41-61), host copy."""
    width: int
    height: int
    data: np.ndarray = None

    def __post_init__(self):
        if self.data is None:
            self.data = np.ones((self.height, self.width, 4), dtype=np.float32)


@dataclass
class RayTraceSettings:
    """The reference's compile-time constants made runtime parameters."""
    samples_per_ray: int = SAMPLES_PER_RAY
    max_depth: int = MAX_DEPTH
    device: int = 0
    flags: int = 0


@dataclass
class World:
    resources: dict = field(default_factory=dict)

    def insert_resource(self, r):
        self.resources[type(r)] = r
        return self

    def resource(self, t):
        return self.resources[t]

    def get_resource(self, t):
        return self.resources.get(t)


@dataclass
class FrameCounter:
    frame: int = 0


class RayTraceNode:
    """render_graph::Node replacement (src/ray_trace_node.rs:173-224)."""

    def __init__(self):
        self.renderer = None
        self._sp = None
        self._mt = None
        self.last_stats = None
        self.uploads = {"full": 0, "spheres": 0, "materials": 0}

    def update(self, world: World):
        """Extract + prepare (sphere.rs:166-197): upload only what changed."""
        settings = world.resource(RayTraceSettings)
        if self.renderer is None:
            self.renderer = Renderer(settings.device)
        sc = world.resource(Scene)
        sp, mt = sc.objects_gpu(), sc.materials_gpu()
        if self._sp is None or len(sp) != len(self._sp) or len(mt) != len(self._mt):
            self.renderer.set_scene(sp, mt)
            self.uploads["full"] += 1
        else:
            for new, old, up, key in ((mt, self._mt, self.renderer.update_materials, "materials"),
                                      (sp, self._sp, self.renderer.update_spheres, "spheres")):
                dirty = np.nonzero(new.view(np.uint8).reshape(len(new), -1)
                                   != old.view(np.uint8).reshape(len(old), -1))[0]
                if dirty.size:
                    i0, i1 = int(dirty.min()), int(dirty.max()) + 1
                    up(i0, new[i0:i1])
                    self.uploads[key] += 1
        self._sp, self._mt = sp, mt

    def run(self, world: World):
        settings = world.resource(RayTraceSettings)
        cam = world.resource(RayTraceCamera)
        out = world.resource(RayTraceOutputImage)
        fc = world.resource(FrameCounter)
        img, st = self.renderer.render(cam.to_gpu(), cam.render_width, cam.render_height,
                                       settings.samples_per_ray, settings.max_depth,
                                       frame0=fc.frame, flags=settings.flags)
        out.data[...] = img
        fc.frame += settings.samples_per_ray  # ray_trace_globals.rs:67 (+1 per frame per sample)
        self.last_stats = st
        return st


class RayTracePlugin:
    """src/plugin.rs:25-47 + SphereRenderPlugin (sphere.rs:150-164)."""

    def __init__(self, settings: RayTraceSettings = None, scene: Scene = None):
        self.settings = settings or RayTraceSettings()
        self.scene = scene

    def build(self, world: World) -> RayTraceNode:
        w, h = RENDER_TARGET_SIZE
        if world.get_resource(RayTraceCamera) is None:
            world.insert_resource(RayTraceCamera(w, h))        # camera.rs:31-37
        cam = world.resource(RayTraceCamera)
        world.insert_resource(self.settings)
        world.insert_resource(FrameCounter())
        world.insert_resource(RayTraceOutputImage(cam.render_width, cam.render_height))
        if world.get_resource(Scene) is None:
            world.insert_resource(self.scene or init_spheres())  # sphere.rs:37-148
        return RayTraceNode()

    @staticmethod
    def frame(world: World, node: RayTraceNode):
        """One Render-stage pass: update then run (Bevy's graph runner order)."""
        node.update(world)
        return node.run(world)


__all__ = ["RayTracePlugin", "RayTraceNode", "RayTraceOutputImage", "RayTraceSettings",
           "World", "FrameCounter", "MaterialCache", "RENDER_TARGET_SIZE", "SAMPLES_PER_RAY",
           "MAX_DEPTH"]
