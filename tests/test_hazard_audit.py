"""The wait-state audit (tools/hazard_audit.py) on the shipped kernels and on
synthetic sequences, one short and one padded per rule (CPU: hipcc
cross-compiles the device assembly here)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import hazard_audit as HA  # noqa: E402

KERNEL = "_Z4kernv:\n{body}\n\ts_endpgm\n"

CASES = {
    # rule: (short sequence, padded sequence)
    "R1": ("v_pk_fma_f32 v[2:3], v[4:5], s[0:1], v[2:3]\n v_add_f32_e32 v6, v2, v7",
           "v_pk_fma_f32 v[2:3], v[4:5], s[0:1], v[2:3]\n s_nop 0\n v_add_f32_e32 v6, v2, v7"),
    "R2": ("v_cmp_ge_f32_e64 s[4:5], v1, v2\n v_mov_b32_e32 v9, 0\n"
           " v_cndmask_b32_e64 v3, 0, 1, s[4:5]",
           "v_cmp_ge_f32_e64 s[4:5], v1, v2\n s_nop 1\n v_cndmask_b32_e64 v3, 0, 1, s[4:5]"),
    "R3": ("v_mfma_f32_32x32x16_f16 v[0:15], v[16:19], v[20:23], 0\n s_nop 7\n"
           " v_or_b32_e32 v30, v0, v1",
           "v_mfma_f32_32x32x16_f16 v[0:15], v[16:19], v[20:23], 0\n s_nop 11\n"
           " v_or_b32_e32 v30, v0, v1"),
    "R4": ("v_add_u32_e32 v1, v2, v3\n v_permlane32_swap_b32_e32 v1, v4",
           "v_add_u32_e32 v1, v2, v3\n s_nop 1\n v_permlane32_swap_b32_e32 v1, v4"),
    "R5": ("v_add_u32_e32 v1, v2, v3\n v_readfirstlane_b32 s6, v1",
           "v_add_u32_e32 v1, v2, v3\n s_nop 0\n v_readfirstlane_b32 s6, v1"),
}


def audit_text(tmp_path, body):
    p = tmp_path / "k.s"
    p.write_text(KERNEL.format(body="\n".join("\t" + ln.strip() for ln in body.split("\n"))))
    return [b[0] for (_, items) in HA.parse(str(p)) for b in HA.audit_kernel("k", items)]


@pytest.mark.parametrize("rule", sorted(CASES))
def test_rule_detects_short_and_accepts_padded(tmp_path, rule):
    short, padded = CASES[rule]
    assert rule in audit_text(tmp_path, short)
    assert audit_text(tmp_path, padded) == []


def test_r6_packed_half_select_beside_mfma(tmp_path):
    """op_sel / op_sel_hi on a VGPR source of v_pk_fma_f32 is refused in a
    kernel with MFMAs; on an SGPR source, or without MFMAs, it is not."""
    mf = "v_mfma_f32_32x32x16_f16 v[0:15], v[16:19], v[20:23], 0\n s_nop 11\n"
    bc = "v_pk_fma_f32 v[30:31], v[32:33], s[0:1], v[34:35] op_sel_hi:[0,1,1]"
    assert "R6" in audit_text(tmp_path, mf + bc)
    assert audit_text(tmp_path, bc) == []
    sg = "v_pk_fma_f32 v[30:31], s[2:3], v[32:33], v[34:35] op_sel_hi:[0,1,1]"
    assert audit_text(tmp_path, mf + sg) == []


def test_chained_mfma_accumulate_needs_no_wait(tmp_path):
    body = ("v_mfma_f32_32x32x16_f16 v[0:15], v[16:19], v[20:23], 0\n"
            " v_mfma_f32_32x32x16_f16 v[0:15], v[24:27], v[28:31], v[0:15]")
    assert audit_text(tmp_path, body) == []


def test_hazard_across_a_branch_is_followed(tmp_path):
    # the producer sits in a predecessor block reached by a branch
    body = ("v_mfma_f32_32x32x16_f16 v[0:15], v[16:19], v[20:23], 0\n s_nop 3\n"
            " s_cbranch_vccz .LBB0_2\n s_nop 7\n.LBB0_2:\n v_or_b32_e32 v30, v0, v1")
    assert "R3" in audit_text(tmp_path, body)


def test_r1_producer_with_src0_broadcast_needs_no_wait(tmp_path):
    # hipcc emits no s_nop after this form (tools/ubench/pk_opsel_probe.hip)
    body = ("v_pk_fma_f32 v[2:3], v[4:5], s[0:1], v[2:3] op_sel_hi:[0,1,1]\n"
            " v_add_f32_e32 v6, v2, v7")
    assert audit_text(tmp_path, body) == []


@pytest.mark.skipif(shutil.which("make") is None or not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="needs hipcc")
def test_shipped_kernels_have_every_wait_state(tmp_path):
    out = tmp_path / "rt.s"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "hazard_audit.py")],
                       capture_output=True, text=True, env=dict(os.environ, RT_AUDIT_ASM=str(out)))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "short pairs / refused forms: 0" in r.stdout
