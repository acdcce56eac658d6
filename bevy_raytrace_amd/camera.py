"""Ray-trace camera: RayTraceCamera resource and the 128-B CameraGPU block.

Mirrors src/camera.rs:13-37 (RayTraceCamera {render_width, render_height,
transform}; default pose Transform::from_xyz(13,2,3).looking_at(ZERO, Y)) and
src/ray_trace_camera.rs:12-68 (CameraGPU packing: fov = 1.5708,
image_plane_distance = 10, lens_focal_length = 0.1, fstop = 1/32).

The camera matrix is built directly from the orthonormal look-at basis in f32
(glam's quaternion round trip is not reproduced; the 128-B block is
the input fixture, so parity does not depend on it).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from .abi import CAMERA_DTYPE

CAMERA_FOV = np.float32(1.5708)          # src/ray_trace_camera.rs:12
IMAGE_PLANE_DISTANCE = np.float32(10.0)  # :59
LENS_FOCAL_LENGTH = np.float32(0.1)      # :60
FSTOP = np.float32(1.0) / np.float32(32.0)  # :61

F = np.float32


def _cross(a, b):
    return np.array([a[1] * b[2] - a[2] * b[1],
                     a[2] * b[0] - a[0] * b[2],
                     a[0] * b[1] - a[1] * b[0]], dtype=np.float32)


def _normalize(v):
    v = np.asarray(v, dtype=np.float32)
    l = np.sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2])
    return (v / l).astype(np.float32)


@dataclass
class Transform:
    """Translation + rotation basis (columns right, up, back), Bevy-style."""
    translation: np.ndarray = field(default_factory=lambda: np.zeros(3, np.float32))
    basis: np.ndarray = field(default_factory=lambda: np.eye(3, dtype=np.float32))

    @staticmethod
    def from_xyz(x, y, z):
        return Transform(np.array([x, y, z], dtype=np.float32))

    def looking_at(self, target, up=(0.0, 1.0, 0.0)):
        """Bevy Transform::look_at: back = normalize(eye - target), right =
        normalize(up x back), up' = back x right."""
        back = _normalize(self.translation - np.asarray(target, dtype=np.float32))
        right = _normalize(_cross(np.asarray(up, dtype=np.float32), back))
        upv = _cross(back, right)
        return Transform(self.translation.copy(), np.stack([right, upv, back], 1).astype(np.float32))

    def right(self):
        return self.basis[:, 0].copy()

    def up(self):
        return self.basis[:, 1].copy()

    def forward(self):
        return (-self.basis[:, 2]).astype(np.float32)

    def compute_matrix(self):
        """Column-major 4x4 (glam Mat4 layout): m[col*4 + row]."""
        m = np.zeros(16, dtype=np.float32)
        for c in range(3):
            m[c * 4:c * 4 + 3] = self.basis[:, c]
        m[12:15] = self.translation
        m[15] = 1.0
        return m


@dataclass
class RayTraceCamera:
    """src/camera.rs:13-19."""
    render_width: int = 1920
    render_height: int = 1080
    transform: Transform = field(
        default_factory=lambda: Transform.from_xyz(13.0, 2.0, 3.0).looking_at((0.0, 0.0, 0.0)))

    def to_gpu(self) -> np.ndarray:
        """Pack CameraGPU exactly as ray_trace_camera.rs:43-68 does."""
        return camera_block(self.transform)


def camera_block(transform: Transform, fov=CAMERA_FOV, image_plane_distance=None,
                 lens_focal_length=None, fstop=None) -> np.ndarray:
    """CameraGPU block (ray_trace_camera.rs:43-68); the lens constants default
    to the reference's (ray_trace_camera.rs:59-62) and only matter to the
    opt-in thin-lens sampling (RT_FLAG_THIN_LENS) and the focus plane."""
    c = np.zeros((), dtype=CAMERA_DTYPE)
    c["transform"] = transform.compute_matrix()
    c["forward"] = transform.forward()
    c["fov"] = F(fov)
    c["up"] = transform.up()
    c["image_plane_distance"] = (IMAGE_PLANE_DISTANCE if image_plane_distance is None
                                 else F(image_plane_distance))
    c["right"] = transform.right()
    c["lens_focal_length"] = LENS_FOCAL_LENGTH if lens_focal_length is None else F(lens_focal_length)
    c["position"] = transform.translation
    c["fstop"] = FSTOP if fstop is None else F(fstop)
    return c


def default_camera_block() -> np.ndarray:
    return RayTraceCamera().to_gpu()
