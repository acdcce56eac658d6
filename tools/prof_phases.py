"""Phase breakdown of rt_render_kernel from the -DRT_PROFILE diagnostic build.
Shares (not absolute times) are meaningful: the stamps perturb the kernel."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bevy_raytrace_amd import abi, scene
from bevy_raytrace_amd.camera import default_camera_block
from bevy_raytrace_amd.renderer import Renderer

lib = sys.argv[1] if len(sys.argv) > 1 else "tools/librt_hip_prof.so"
cam = default_camera_block()
NAMES = {0: "refill", 1: "filter", 2: "drain", 12: "bookkeep", 3: "shade", 7: "tail"}
for key, sc, W, H, S, D in [("rtiow1080", scene.rtiow_final_scene(), 1920, 1080, 64, 16),
                            ("spheres10k", scene.ten_thousand_scene(), 1920, 1080, 8, 16)]:
    r = Renderer(0, lib_path=lib)
    sp, mt = sc.objects_gpu(), sc.materials_gpu()
    r.set_scene(sp, mt)
    for flags in (abi.RT_FLAG_NO_PRIMARY_CACHE, 0):
        img, st = r.render(cam, W, H, S, D, flags=flags)
        c = r.debug_counters()
        tot = sum(c[i] for i in NAMES)
        print(f"{key} flags={flags} kernel_ms={st['kernel_ms']:.2f} traced={st['traced_segments']}")
        print("  phase shares: " + ", ".join(f"{NAMES[i]}={c[i]/tot:.3f}" for i in NAMES))
        it = max(c[4], 1)
        print(f"  wave iterations={c[4]} lanes/iter={c[9]/it:.1f} cand-groups/iter={c[5]/it:.1f} "
              f"of {(len(sp)+7)//8} drain-max/iter={c[6]/it:.2f} flushes/iter={c[11]/it:.3f} "
              f"wave-cycles total={c[8]} per-iter={c[8]/it:.0f}")
        print(f"  exact tests per iter: wave-max {c[13]/it:.2f}  wave-max full-path {c[14]/it:.2f}  "
              f"lane-sum {c[15]/it:.1f} (per lane {c[15]/max(c[9],1):.2f})")
    r.close()
