"""Generate tests/golden/*.npz from the C oracle (cross-checked against the
numpy restatement before writing). Inputs + expected outputs only (data
fixtures); the reference ships none of its own."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bevy_raytrace_amd import scene  # noqa: E402
from bevy_raytrace_amd.camera import default_camera_block  # noqa: E402
from oracle import oracle as O, rt_oracle_np as N  # noqa: E402

CASES = [
    ("config1_64x36_s8_d8", scene.config1_scene, 64, 36, 8, 8, 0),
    ("reference_96x54_s1_d3", scene.reference_scene, 96, 54, 1, 3, 7),
    ("rtiow_64x36_s4_d16", scene.rtiow_final_scene, 64, 36, 4, 16, 0),
    ("rtiow_40x24_s11_d5_f1000", scene.rtiow_final_scene, 40, 24, 11, 5, 1000),
]


def main():
    out_dir = os.path.join(ROOT, "tests", "golden")
    os.makedirs(out_dir, exist_ok=True)
    cam = default_camera_block()
    for name, mk, W, H, S, D, f0 in CASES:
        sc = mk()
        sp, mt = sc.objects_gpu(), sc.materials_gpu()
        img, segs = O.render(cam, sp, mt, W, H, S, D, frame0=f0)
        img2, segs2 = N.render(np.frombuffer(cam.tobytes(), np.float32), sp, mt, W, H, S, D, frame0=f0)
        assert np.array_equal(img, img2, equal_nan=True) and segs == segs2, name
        np.savez_compressed(os.path.join(out_dir, name + ".npz"),
                            spheres=np.frombuffer(sp.tobytes(), np.uint8),
                            materials=np.frombuffer(mt.tobytes(), np.uint8),
                            camera=np.frombuffer(cam.tobytes(), np.uint8),
                            params=np.array([W, H, S, D, f0], np.uint32),
                            image=img, segments=np.array([segs], np.uint64))
        print(name, img.shape, segs)


if __name__ == "__main__":
    main()
