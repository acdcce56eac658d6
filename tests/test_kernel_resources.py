"""The render kernels' resources in the shipped code (CPU: hipcc cross-compiles
the device assembly with the library's flags, `make asm`): no VGPR spills and
no scratch, at most 128 VGPRs (4 waves per SIMD) and at most 40 KiB of LDS per
256-thread workgroup (4 workgroups per CU) -- the occupancy DESIGN.md §2 and
§4.1 state, which a source change could silently lose (round 5's bound-chunk
loads spilled 28 B per lane before they were fixed; the 16 x 16 walk spilled
20+ VGPRs at first)."""
import os
import re
import shutil
import subprocess

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bevy_raytrace_amd", "csrc")

pytestmark = pytest.mark.skipif(
    shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
    reason="needs hipcc")


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    out = tmp_path_factory.mktemp("asm") / "rt.s"
    subprocess.run(["make", "-s", "asm", f"ASM={out}"], cwd=CSRC, check=True, capture_output=True)
    text = out.read_text()
    m = re.search(r"\.amdgpu_metadata\n(.*?)\n\s*\.end_amdgpu_metadata", text, re.S)
    assert m, "no AMDGPU metadata in the assembly"
    meta = yaml.safe_load(m.group(1))
    return {k[".name"]: k for k in meta["amdhsa.kernels"]}


@pytest.mark.parametrize("name", ["_Z16rt_render_kernel", "_Z22rt_render_multi_kernel"])
def test_render_kernel_fits_four_workgroups_per_cu_without_spills(kernels, name):
    (k,) = [v for n, v in kernels.items() if n.startswith(name)]
    assert k[".vgpr_spill_count"] == 0, k[".vgpr_spill_count"]
    assert k[".private_segment_fixed_size"] == 0, "scratch in the render kernel"
    assert k[".vgpr_count"] + k.get(".agpr_count", 0) <= 128
    assert k[".group_segment_fixed_size"] <= 160 * 1024 // 4
