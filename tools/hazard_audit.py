"""Wait-state audit of the shipped gfx950 code object's assembly.

hipcc pads the hazards of the instructions it generates itself (LLVM's
GCNHazardRecognizer), but it treats an inline-asm statement as one opaque
instruction: nothing inside the string is padded, and across the statement's
boundary it adds only a fixed one-state pad. This tool re-checks, for every
kernel of `make asm`'s output, the gfx950 wait-state rules the kernel's own
instruction mix can trigger, on compiler code and on inline asm alike,
following control flow backwards through every predecessor of a block:

  R1  v_pk_*_f32 whose src0 has op_sel_hi = 1 (the default form) writes a VGPR
      pair -> the next VALU reading or writing it: 1 wait state (hipcc emits
      `s_nop 0` there; a producer with op_sel_hi:[0,..] on src0 needs none:
      LLVM's dst-sel forwarding rule reads src0_modifiers bit 3).
  R2  VALU writes an SGPR / VCC (v_cmp_*_e64 sdst, v_cmp_*_e32 -> vcc, the
      carry-out of v_add/sub*_co) -> a VALU reading it as a lane mask
      (v_cndmask_b32, v_addc/v_subb carry-in, v_div_fmas): 2 wait states
      (hipcc: `s_nop 1`).
  R3  v_mfma_f32_32x32x16_* (8 passes) writes vdst -> any non-MFMA instruction
      reading or writing those VGPRs: 12 wait states (hipcc: `s_nop 11`);
      the next MFMA taking the same registers whole as C needs none.
  R4  VALU writes a VGPR -> v_permlane16/32_swap reading it: 2 wait states.
  R5  VALU writes a VGPR -> v_readlane / v_readfirstlane reading it: 1.
  R6  (not a wait-state rule) in a kernel that issues MFMAs, no v_pk_*_f32
      may select a VGPR source's halves with op_sel / op_sel_hi (anything but
      op_sel:0, op_sel_hi:1 on a VGPR operand). Measured on gfx950: such
      half-broadcasts return wrong values while other waves of the kernel run
      MFMAs (tools/ubench/opsel_mfma.hip, tools/isect_diag.py).
      hipcc itself emits these forms for f2{x, x} operands, so the rule is
      checked on compiler code as well as on inline asm.

The rules were read off hipcc's own output for probe kernels (the s_nop it
inserts between each producer/consumer pair; tools/ubench/pk_opsel_probe.hip)
and each is satisfied by every compiler-generated sequence of the kernels, so
the audit also checks its own rule set. A wait state is one instruction issued
in between (`s_nop N` counts N + 1).

usage: python tools/hazard_audit.py [file.s]   (default: builds /tmp/rt_audit.s)
exit status 1 if any pair is short of its wait states."""
from __future__ import annotations

import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bevy_raytrace_amd", "csrc")

REG = re.compile(r"\b([vs])(\d+)\b|\b([vs])\[(\d+):(\d+)\]|\b(vcc|exec)\b")
LABEL = re.compile(r"^(\.LBB\w+|[A-Za-z_]\w*):")
BRANCH = re.compile(r"^\s*(s_branch|s_cbranch_\w+)\s+(\.LBB\w+)")
NEED = {"R1": 1, "R2": 2, "R3": 12, "R4": 2, "R5": 1, "R6": 0}
WINDOW = 12  # the largest wait-state requirement above


def regs(text: str) -> set[str]:
    out = set()
    for m in REG.finditer(text):
        if m.group(1):
            out.add(f"{m.group(1)}{m.group(2)}")
        elif m.group(3):
            for k in range(int(m.group(4)), int(m.group(5)) + 1):
                out.add(f"{m.group(3)}{k}")
        else:
            out.add(m.group(6))
    if "vcc" in out:
        out |= {"vcc_lo", "vcc_hi"}
    return out


def split_ops(rest: str) -> list[str]:
    ops, depth, cur = [], 0, ""
    for ch in rest:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            ops.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        ops.append(cur.strip())
    return ops


class Inst:
    def __init__(self, idx: int, text: str, in_asm: bool):
        self.idx, self.text, self.in_asm = idx, text.strip(), in_asm
        parts = self.text.split(None, 1)
        self.op = parts[0]
        rest = parts[1] if len(parts) > 1 else ""
        # modifiers (op_sel, offsets, ...) follow the operands, space-separated
        self.mods = " ".join(t for t in rest.split() if ":" in t and "[" in t.split(":")[0] + "[" and
                             t.split(":")[0].isalpha() and not t.startswith(("v[", "s[")))
        self.ops = split_ops(re.sub(r"\s+(op_sel|op_sel_hi|offset|neg_lo|neg_hi|clamp|cbsz|abid|blgp)"
                                    r"\S*", "", rest))
        self.is_valu = self.op.startswith("v_")
        self.is_mfma = self.op.startswith("v_mfma")
        self.waits = (int(self.text.split()[1], 0) + 1) if self.op == "s_nop" else 1
        self.defs, self.uses, self.mask_uses = set(), set(), set()
        self.sdefs = set()
        if not self.is_valu:
            return
        ops = self.ops
        op = self.op
        if op.startswith("v_cmp"):
            if op.endswith("_e32"):
                self.sdefs = {"vcc", "vcc_lo", "vcc_hi"}
                self.uses = set().union(*(regs(o) for o in ops))
            else:
                self.sdefs = regs(ops[0]) if ops else set()
                self.uses = set().union(*(regs(o) for o in ops[1:])) if len(ops) > 1 else set()
            return
        if not ops:
            return
        self.defs = {r for r in regs(ops[0]) if r.startswith("v")}
        srcs = ops[1:]
        if re.match(r"v_(add|sub|subrev)(c)?_co_u32_e64", op) or re.match(r"v_(addc|subb|subbrev)_co_u32_e64", op):
            self.sdefs = regs(srcs[0]) if srcs else set()
            srcs = srcs[1:]
        if op.startswith(("v_addc", "v_subb")):
            if op.endswith("_e32"):
                self.mask_uses = {"vcc", "vcc_lo", "vcc_hi"}
            elif srcs:
                self.mask_uses = regs(srcs[-1])
                srcs = srcs[:-1]
        if op.startswith("v_cndmask_b32"):
            if op.endswith("_e32"):
                self.mask_uses = {"vcc", "vcc_lo", "vcc_hi"}
            elif srcs:
                self.mask_uses = regs(srcs[-1])
                srcs = srcs[:-1]
        if op.startswith("v_div_fmas"):
            self.mask_uses = {"vcc", "vcc_lo", "vcc_hi"}
        if op.startswith(("v_readlane", "v_readfirstlane")):
            self.sdefs = regs(ops[0])
            self.defs = set()
        self.uses = set().union(*(regs(o) for o in srcs)) if srcs else set()
        if self.is_mfma and len(ops) >= 4:
            self.mfma_c = regs(ops[3])
        # R1 producer: packed f32 with src0 op_sel_hi = 1 (absent = all ones)
        self.r1_producer = False
        if re.match(r"v_pk_\w+_f32", op):
            m = re.search(r"op_sel_hi:\[(\d)", self.text)
            self.r1_producer = m is None or m.group(1) == "1"


def parse(path: str):
    """Yields (kernel name, list of lines with Inst or label markers)."""
    kernels = []
    cur, name, in_asm = None, None, False
    for raw in open(path):
        line = raw.rstrip("\n")
        s = line.strip()
        if re.match(r"^_Z\w+:|^rt_\w+:", line) and not s.startswith("."):
            name = line.split(":")[0]
            cur = []
            kernels.append((name, cur))
            continue
        if cur is None:
            continue
        if s.startswith("s_endpgm"):
            cur.append(("inst", Inst(len(cur), s, in_asm)))
            cur = None
            continue
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = LABEL.match(s)
        if m:
            cur.append(("label", m.group(1)))
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        cur.append(("inst", Inst(len(cur), s, in_asm)))
    return kernels


def audit_kernel(name, items):
    # predecessors of each label: the fall-through line before it (unless an
    # unconditional branch / end) and every branch naming it
    label_at = {it[1]: i for i, it in enumerate(items) if it[0] == "label"}
    preds = {i: [] for i in label_at.values()}
    for i, it in enumerate(items):
        if it[0] == "inst":
            m = BRANCH.match(it[1].text)
            if m and m.group(2) in label_at:
                preds[label_at[m.group(2)]].append(i)
    for lab, i in label_at.items():
        j = i - 1
        if j >= 0 and not (items[j][0] == "inst" and items[j][1].op in ("s_branch", "s_endpgm",
                                                                          "s_setpc_b64")):
            preds[i].append(j)

    def back(i, budget, seen=()):
        """Instructions before line i within `budget` wait states, per path:
        yields (inst, waits between it and line i)."""
        stack = [(i - 1, 0, seen)]
        while stack:
            j, w, vis = stack.pop()
            while j >= 0 and w < budget:
                it = items[j]
                if it[0] == "label":
                    for p in preds.get(j, []):
                        if (p, j) not in vis:
                            stack.append((p, w, vis + ((p, j),)))
                    break
                inst = it[1]
                yield inst, w
                w += inst.waits
                j -= 1

    bad = []
    has_mfma = any(it[0] == "inst" and it[1].is_mfma for it in items)
    for it in items:
        if not has_mfma or it[0] != "inst" or not re.match(r"v_pk_\w+_f32", it[1].op):
            continue
        c = it[1]
        m1 = re.search(r"op_sel:\[([\d,]+)\]", c.text)
        m2 = re.search(r"op_sel_hi:\[([\d,]+)\]", c.text)
        sel = [int(x) for x in m1.group(1).split(",")] if m1 else [0, 0, 0]
        hi = [int(x) for x in m2.group(1).split(",")] if m2 else [1, 1, 1]
        for k, opnd in enumerate(c.ops[1:4]):
            if opnd.startswith("v") and k < len(sel) and (sel[k] != 0 or hi[k] != 1):
                bad.append(("R6", "asm" if c.in_asm else "compiler", c.text, c.text, 0))
                break
    for i, it in enumerate(items):
        if it[0] != "inst" or not it[1].is_valu:
            continue
        c = it[1]
        touched = c.uses | c.defs
        for p, w in back(i, WINDOW):
            if not p.is_valu:
                continue
            rule = None
            if p.r1_producer if hasattr(p, "r1_producer") else False:
                if (p.defs & touched) and w < NEED["R1"]:
                    rule = "R1"
            if p.sdefs and (p.sdefs & c.mask_uses) and w < NEED["R2"]:
                rule = "R2"
            if p.is_mfma and (p.defs & touched) and w < NEED["R3"]:
                chained = c.is_mfma and getattr(c, "mfma_c", set()) == p.defs and not (
                    p.defs & (c.uses - c.mfma_c))
                if not chained:
                    rule = "R3"
            if c.op.startswith(("v_permlane16_swap", "v_permlane32_swap")) and p.defs & (c.defs | c.uses) \
                    and not p.is_mfma and w < NEED["R4"]:
                rule = "R4"
            if c.op.startswith(("v_readlane", "v_readfirstlane")) and p.defs & c.uses and w < NEED["R5"]:
                rule = "R5"
            if rule:
                where = "asm" if (c.in_asm or p.in_asm) else "compiler"
                bad.append((rule, where, p.text, c.text, w))
    return bad


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else None
    if path is None:
        path = os.environ.get("RT_AUDIT_ASM", "/tmp/rt_audit.s")
        subprocess.run(["make", "-s", "asm", f"ASM={path}"], cwd=CSRC, check=True,
                       capture_output=True)
    total = 0
    for name, items in parse(path):
        bad = audit_kernel(name, items)
        n_asm = sum(1 for it in items if it[0] == "inst" and it[1].in_asm)
        print(f"{name[:60]:60s} {len(items):6d} lines, {n_asm:4d} asm instructions, "
              f"{len(bad)} short")
        for rule, where, p, c, w in bad[:20]:
            if rule == "R6":
                print(f"   R6 ({where}): {c!r}: VGPR half-select in a kernel with MFMAs")
            else:
                print(f"   {rule} ({where}): {p!r} -> {c!r}: {w} of {NEED[rule]} wait states")
        total += len(bad)
    print("short pairs / refused forms:", total)
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main())
