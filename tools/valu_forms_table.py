"""The per-form issue-price table of the render kernel's VALU forms
(DESIGN.md §5), from one tools/calls/gpu_r04_call2.sh run:

  - cycles per instruction per SIMD at 1, 2, 4, 6 waves per SIMD
    (tools/ubench/valu_forms: in-kernel s_memtime; the slowest wave's
    delta, which spans the SIMD's whole stream when its waves start together
    -- the per-wave median undercounts once the arbiter serialises waves);
  - the PMC record of the 4-wave run: quad-cycles per instruction counted by
    SQ_ACTIVE_INST_VALU, those shared with a second instruction
    (SQ_ACTIVE_INST_VALU2: dual issue), and the SQ_INSTS_VALU_<class>
    counter the form increments.

usage: python tools/valu_forms_table.py gpurun_out/r04/c2 > profiles/r04/valu_forms/table.txt
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r04/c2"


def ubench(w):
    out = {}
    path = os.path.join(d, f"valu_forms_w{w}.txt")
    if not os.path.exists(path):
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "r04",
                            "valu_forms", f"valu_forms_w{w}.txt")
    for ln in open(path):
        m = re.match(r"(\S+)\s+([\d.]+)\s+([\d.]+)\.\.([\d.]+)", ln)
        if m:
            out[m.group(1)] = (float(m.group(2)), float(m.group(3)), float(m.group(4)))
    return out


def pmc(sub):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
    last = {}
    for did in sorted(per, key=int):  # the last launch of each kernel
        last[names[did][2:]] = per[did]
    return last


W = [1, 2, 4, 6]
ub = {w: ubench(w) for w in W}
a, b = pmc("ub_pmc_1"), pmc("ub_pmc_2")
CLS = ["INT32", "FMA_F32", "ADD_F32", "MUL_F32", "TRANS_F32"]
print("# VALU form issue prices on gfx950 (MI355X), tools/ubench/valu_forms + rocprofv3 --pmc")
print("# cyc@W: cycles per wave64 instruction per SIMD at W waves/SIMD (slowest wave's span)")
print("# quads/inst: SQ_ACTIVE_INST_VALU per instruction; dual: SQ_ACTIVE_INST_VALU2 per instruction")
print(f"{'form':16s} " + " ".join(f"{'cyc@' + str(w):>7s}" for w in W)
      + f" {'quads':>6s} {'dual':>6s} {'busy':>6s}  class")
for name in ub[4]:
    c = a.get(name, {})
    n = c.get("SQ_INSTS_VALU") or 0
    cls = [x for x in CLS if n and c.get("SQ_INSTS_VALU_" + x, 0) > 0.4 * n]
    if n and b.get(name, {}).get("SQ_INSTS_VALU_CVT", 0) > 0.4 * n:
        cls.append("CVT")
    q = c.get("SQ_ACTIVE_INST_VALU", 0) / n if n else float("nan")
    q2 = c.get("SQ_ACTIVE_INST_VALU2", 0) / n if n else float("nan")
    print(f"{name:16s} " + " ".join(f"{ub[w].get(name, (0, 0, 0))[2]:7.2f}" for w in W)
          + f" {q:6.3f} {q2:6.3f} {q - q2:6.3f}  {','.join(cls) or '-'}")
print("# busy = quads - dual: the quad-cycles the form holds the SIMD's VALU issue port")
print("# mfma / mfma_or3: per MFMA (v_mfma_f32_32x32x16_f16); mfma_or3 adds 5 v_or3_b32 per MFMA,"
      " which run under the MFMA pipe's 32 cycles")
