"""Scene: Sphere / RayTraceMaterial / MaterialCache and the seeded generators.

Mirrors the reference's main-world scene API:
  Reflectance            src/ray_trace_materials.rs:12-17
  RayTraceMaterial       src/ray_trace_materials.rs:25-31
  MaterialCache          src/ray_trace_materials.rs:50-67 (IndexMap: insertion order = GPU index)
  init_materials_cache   src/ray_trace_materials.rs:83-127
  Sphere                 src/sphere.rs:31-35
  init_spheres           src/sphere.rs:37-148
  extract / prepare      src/sphere.rs:166-197 -> ObjectListGPU (here: SPHERE_DTYPE array)

Divergence D4: the reference draws from an unseeded
thread_rng (sphere.rs:46); here the generator is a seeded PCG32 so a scene is
reproducible from (dim, split, seed), and the scene file is the input.
"""
from __future__ import annotations

import enum
import json
import os
from collections import OrderedDict
from dataclasses import dataclass, field

import numpy as np

from .abi import MATERIAL_DTYPE, SPHERE_DTYPE

F = np.float32


class Reflectance(enum.IntEnum):
    Lambertian = 0
    Metallic = 1
    Dielectric = 2


@dataclass
class RayTraceMaterial:
    color: tuple = (0.0, 0.0, 0.0, 1.0)
    reflectance: Reflectance = Reflectance.Lambertian
    fuzziness: float = 0.0
    index_of_refraction: float = 0.0


@dataclass
class MaterialCache:
    """Ordered name -> material map; get_index_of is the GPU material index."""
    materials: "OrderedDict[str, RayTraceMaterial]" = field(default_factory=OrderedDict)

    def insert(self, name, mat):
        self.materials[name] = mat

    def get(self, key):
        return self.materials[key]

    def get_index_of(self, key):
        return list(self.materials.keys()).index(key)

    def __len__(self):
        return len(self.materials)

    def to_gpu(self) -> np.ndarray:
        """MaterialGPU array (ray_trace_materials.rs:144-153: colour passed raw)."""
        arr = np.zeros(len(self.materials), dtype=MATERIAL_DTYPE)
        for i, m in enumerate(self.materials.values()):
            arr[i]["color"] = np.asarray(m.color, dtype=np.float32)
            arr[i]["reflectance"] = int(m.reflectance)
            arr[i]["fuzziness"] = F(m.fuzziness)
            arr[i]["index_of_refraction"] = F(m.index_of_refraction)
        return arr


@dataclass
class Sphere:
    """Sphere component + its Transform translation (sphere.rs:31-35, 171-176)."""
    center: tuple
    radius: float
    material: int


@dataclass
class Scene:
    spheres: list
    materials: MaterialCache
    name: str = "scene"

    def objects_gpu(self) -> np.ndarray:
        """ObjectListGPU.spheres (sphere.rs:166-197), query order = spawn order."""
        arr = np.zeros(len(self.spheres), dtype=SPHERE_DTYPE)
        for i, s in enumerate(self.spheres):
            arr[i]["center"] = np.asarray(s.center, dtype=np.float32)
            arr[i]["radius"] = F(s.radius)
            arr[i]["material"] = int(s.material)
        return arr

    def materials_gpu(self) -> np.ndarray:
        return self.materials.to_gpu()

    def save(self, path):
        """Binary scene file: the exact 32-B GPU records + a small JSON header."""
        sp, mt = self.objects_gpu(), self.materials_gpu()
        np.savez(path, spheres=sp.view(np.uint8), materials=mt.view(np.uint8),
                 meta=np.frombuffer(json.dumps({"name": self.name}).encode(), np.uint8))

    @staticmethod
    def load_arrays(path):
        z = np.load(path, allow_pickle=False)
        sp = z["spheres"].view(SPHERE_DTYPE)
        mt = z["materials"].view(MATERIAL_DTYPE)
        return sp, mt


class Pcg32:
    """PCG-XSH-RR 32 (O'Neill); next_f32 in [0, 1) with 24 bits."""

    MUL = 6364136223846793005
    MASK = (1 << 64) - 1

    def __init__(self, seed, stream=54):
        self.inc = ((stream << 1) | 1) & self.MASK
        self.state = 0
        self.next_u32()
        self.state = (self.state + seed) & self.MASK
        self.next_u32()

    def next_u32(self):
        old = self.state
        self.state = (old * self.MUL + self.inc) & self.MASK
        xorshifted = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xorshifted >> rot) | (xorshifted << ((-rot) & 31))) & 0xFFFFFFFF

    def f32(self):
        return F((self.next_u32() >> 8) * (1.0 / 16777216.0))


def init_materials_cache(split="reference") -> MaterialCache:
    """ray_trace_materials.rs:83-127 (reference) or the RTIOW final-scene big
    spheres (glass centre, Lambertian left, metal right)."""
    c = MaterialCache()
    c.insert("ground", RayTraceMaterial((0.5, 0.5, 0.5, 1.0), Reflectance.Lambertian, 1.0, 0.0))
    if split == "reference":
        c.insert("center", RayTraceMaterial((0.7, 0.3, 0.3, 1.0), Reflectance.Lambertian, 1.0, 0.0))
        c.insert("left", RayTraceMaterial((0.8, 0.8, 0.8, 1.0), Reflectance.Metallic, 0.1, 1.5))
        c.insert("right", RayTraceMaterial((0.7, 0.6, 0.5, 1.0), Reflectance.Metallic, 0.0, 1.5))
    elif split == "rtiow":
        c.insert("center", RayTraceMaterial((1.0, 1.0, 1.0, 1.0), Reflectance.Dielectric, 0.0, 1.5))
        c.insert("left", RayTraceMaterial((0.4, 0.2, 0.1, 1.0), Reflectance.Lambertian, 1.0, 0.0))
        c.insert("right", RayTraceMaterial((0.7, 0.6, 0.5, 1.0), Reflectance.Metallic, 0.0, 1.5))
    elif split == "config1":
        c.insert("center", RayTraceMaterial((0.7, 0.3, 0.3, 1.0), Reflectance.Lambertian, 1.0, 0.0))
        c.insert("left", RayTraceMaterial((1.0, 1.0, 1.0, 1.0), Reflectance.Dielectric, 0.0, 1.5))
        c.insert("right", RayTraceMaterial((0.7, 0.6, 0.5, 1.0), Reflectance.Metallic, 0.0, 1.5))
    else:
        raise ValueError(f"unknown split {split!r}")
    return c


def init_spheres(sphere_dim=7, split="reference", seed=20221015, max_grid=None) -> Scene:
    """sphere.rs:37-148 with a seeded RNG.

    split="reference": the reference's own material split (sphere.rs:61-91):
      U < 0.8 -> Lambertian rgb = (U, U, U); else Metallic rgb = (U, U, U), fuzz = 0.5*U.
    split="rtiow": the RTIOW final-scene split (the commented block sphere.rs:101-120):
      U < 0.8 -> Lambertian albedo = (U*U, U*U, U*U); < 0.95 -> Metallic albedo
      U[0.5,1), fuzz U[0,0.5); else Dielectric 1.5.
    Draw order per candidate: center.x, center.z, then (if accepted) the material.
    max_grid caps the number of accepted grid spheres (config 5: 9,996).
    """
    rng = Pcg32(seed)
    mats = init_materials_cache(split)
    spheres = [Sphere((0.0, -1000.0, -1.0), 1000.0, mats.get_index_of("ground"))]
    ref = np.array([4.0, 0.2, 0.0], dtype=np.float32)
    accepted = 0
    for a in range(-sphere_dim, sphere_dim):
        for b in range(-sphere_dim, sphere_dim):
            cx = F(F(a) + F(0.9) * rng.f32())
            cz = F(F(b) + F(0.9) * rng.f32())
            center = np.array([cx, F(0.2), cz], dtype=np.float32)
            dv = center - ref
            if not (np.sqrt((dv[0] * dv[0] + dv[1] * dv[1]) + dv[2] * dv[2]) > F(0.9)):
                continue
            if max_grid is not None and accepted >= max_grid:
                continue
            name = f"material_{a}_{b}"
            choose = rng.f32()
            if split == "reference" or split == "config1":
                if choose < F(0.8):
                    m = RayTraceMaterial((rng.f32(), rng.f32(), rng.f32(), 1.0),
                                         Reflectance.Lambertian, 1.0, 0.0)
                else:
                    col = (rng.f32(), rng.f32(), rng.f32(), 1.0)
                    m = RayTraceMaterial(col, Reflectance.Metallic, F(rng.f32() * F(0.5)), 0.0)
            else:
                if choose < F(0.8):
                    c1 = [rng.f32() for _ in range(3)]
                    c2 = [rng.f32() for _ in range(3)]
                    m = RayTraceMaterial((F(c1[0] * c2[0]), F(c1[1] * c2[1]), F(c1[2] * c2[2]), 1.0),
                                         Reflectance.Lambertian, 1.0, 0.0)
                elif choose < F(0.95):
                    col = tuple(F(F(0.5) + F(0.5) * rng.f32()) for _ in range(3)) + (1.0,)
                    m = RayTraceMaterial(col, Reflectance.Metallic, F(F(0.5) * rng.f32()), 0.0)
                else:
                    m = RayTraceMaterial((1.0, 1.0, 1.0, 1.0), Reflectance.Dielectric, 0.0, 1.5)
            mats.insert(name, m)
            spheres.append(Sphere((float(cx), 0.2, float(cz)), 0.2, mats.get_index_of(name)))
            accepted += 1
    spheres.append(Sphere((0.0, 1.0, 0.0), 1.0, mats.get_index_of("center")))
    spheres.append(Sphere((-4.0, 1.0, 0.0), 1.0, mats.get_index_of("left")))
    spheres.append(Sphere((4.0, 1.0, 0.0), 1.0, mats.get_index_of("right")))
    return Scene(spheres, mats, name=f"grid{sphere_dim}_{split}_{seed}")


def config1_scene() -> Scene:
    """Config 1 (BASELINE.json configs[0]): ground + Lambertian + glass + metal."""
    mats = init_materials_cache("config1")
    spheres = [Sphere((0.0, -1000.0, -1.0), 1000.0, 0),
               Sphere((0.0, 1.0, 0.0), 1.0, 1),
               Sphere((-4.0, 1.0, 0.0), 1.0, 2),
               Sphere((4.0, 1.0, 0.0), 1.0, 3)]
    return Scene(spheres, mats, name="config1")


def rtiow_final_scene(seed=20221015) -> Scene:
    """Config 2-4 scene: the RTIOW final scene, dim=11 (a, b in [-11, 11))."""
    return init_spheres(11, "rtiow", seed)


def ten_thousand_scene(seed=20221015) -> Scene:
    """Config 5: dim=50 grid, first 9,996 accepted + ground + 3 big = 10,000."""
    return init_spheres(50, "rtiow", seed, max_grid=9996)


def reference_scene(seed=20221015) -> Scene:
    """The reference's own scene: dim=7, its own material split."""
    return init_spheres(7, "reference", seed)
