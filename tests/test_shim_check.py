"""tools/check_shim.py over the Rust drop-in (bevy_shim/manifest.json) and the
reference crate read as text. Build-container only: skipped where the
reference sources are absent (the GPU box)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
CHECK = os.path.join(ROOT, "tools", "check_shim.py")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")),
                                reason="reference sources not present")


def _run(manifest=None):
    args = [sys.executable, CHECK, REF] + ([manifest] if manifest else [])
    return subprocess.run(args, capture_output=True, text=True, timeout=60)


def test_shim_crate_is_closed():
    p = _run()
    assert p.returncode == 0, p.stdout
    assert p.stdout.startswith("OK")


def test_check_catches_a_kept_file_using_a_deleted_module(tmp_path):
    """Round 1's manifest kept the reference's ray_trace_output.rs, whose
    queue system needs RayTracePipeline: the check must fail on it."""
    man = json.load(open(os.path.join(ROOT, "bevy_shim", "manifest.json")))
    del man["replace"]["src/ray_trace_output.rs"]
    path = tmp_path / "manifest.json"
    path.write_text(json.dumps(man))
    p = _run(str(path))
    assert p.returncode == 1
    assert "RayTracePipeline" in p.stdout
