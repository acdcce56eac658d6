"""The cross-device hand-off of RT_FLAG_IMAGE_OUT rows is in the shipped code
(CPU: hipcc cross-compiles the device assembly of the library's sources with
the library's flags, `make asm`).

Protocol (visibility): a rank writing its rows into another
device's image stores every byte of them with system-scope write-through
stores (sc0 sc1) and every writing wave waits for them (s_waitcnt vmcnt(0))
before it ends -- MI355X_MICROARCH.md's write-through producer form, no
release needed (round 5; the round-4 per-wave release is a knob for A/B);
the image's owner reads them after a system-scope acquire (rt_acquire), once
the host has seen the writers complete."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bevy_raytrace_amd", "csrc")

pytestmark = pytest.mark.skipif(
    shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
    reason="needs hipcc")


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("asm") / "rt.s"
    subprocess.run(["make", "-s", "asm", f"ASM={out}"], cwd=CSRC, check=True,
                   capture_output=True)
    return out.read_text()


def kernel_body(asm, name):
    """Instructions of one kernel: from its label to its end marker."""
    m = re.search(r"^" + re.escape(name) + r"[A-Za-z0-9_]*:", asm, re.M)
    assert m, f"kernel {name} not in the assembly"
    end = asm.find(".Lfunc_end", m.end())
    lines = asm[m.end():end].split("\n")
    return [ln.split(";")[0].strip() for ln in lines
            if ln.strip() and not ln.strip().startswith((";", "."))]


def test_collect_writes_image_rows_through_and_drains_them(asm):
    body = kernel_body(asm, "_Z17rt_collect_kernel")
    stores = [i for i, ln in enumerate(body) if ln.startswith("global_store_dwordx4")]
    through = [i for i in stores if re.search(r"\bsc0 sc1\b", body[i])]
    assert through, "no system-scope write-through store of an image pixel"
    # after the last write-through store, a vmcnt(0) wait before the wave
    # ends (the store is inline asm: hipcc does not count it, the kernel
    # waits explicitly)
    end = max(i for i, ln in enumerate(body) if ln == "s_endpgm")
    assert any(ln.startswith("s_waitcnt") and "vmcnt(0)" in ln
               for ln in body[max(through) + 1:end])
    # the round-4 per-wave release survives only as the A/B knob's branch
    wbl2 = [i for i, ln in enumerate(body) if ln == "buffer_wbl2 sc0 sc1"]
    assert len(wbl2) <= 1


def test_acquire_kernel_invalidates_at_system_scope(asm):
    body = kernel_body(asm, "_Z17rt_acquire_kernel")
    assert "buffer_inv sc0 sc1" in body
    i = body.index("buffer_inv sc0 sc1")
    assert any(ln.startswith("s_waitcnt") and "vmcnt(0)" in ln for ln in body[i + 1:])


def test_render_kernel_has_no_system_scope_traffic(asm):
    """The render kernel writes only device-local memory (direct output is
    off for another device's image, rt_api.cpp): the single-device hot path
    pays for no system-scope store or release."""
    body = kernel_body(asm, "_Z16rt_render_kernel")
    assert not any("sc0 sc1" in ln for ln in body)
