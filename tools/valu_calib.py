"""VALU issue-cost calibration on gfx950 (tools/ubench/valu_busy under
rocprofv3 --pmc; tools/gpu_round.sh) and the render kernel's VALU busy from
the same counters.

For each microbench kernel (8 independent instructions of one form per loop
iteration, 6 waves per SIMD): cycles per wave64 instruction per SIMD =
(GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs / SQ_INSTS_VALU, and which
SQ_INSTS_VALU_<class> counter the form increments. SQ_ACTIVE_INST_VALU counts
one quad-cycle (4 cycles) per instruction (two for v_sqrt_f32) whatever the
form's issue cost, so AMD's VALUBusy = SQ_ACTIVE_INST_VALU x 4 / (SIMDs x
cycles) over-counts the 2-cycle forms and can exceed 1.

The render kernel's issue-weighted VALU busy prices each class at its
measured cost: FMA_F32 (v_fma_f32 and v_pk_fma_f32) 4, ADD_F32 / MUL_F32 2,
TRANS_F32 8; INT32 is a mix (v_add_u32 2, v_mul_lo_u32 4): priced 2 (lower
bound) and 4 (upper); the unclassified rest (v_max3 / v_cndmask / v_mov /
v_cmp / logic) at 4 (v_and_b32 is 2, v_cmp to SGPRs 5).
usage: python tools/valu_calib.py [profiles/r02_valu_pmc]"""
import csv
import os
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "r02_valu_pmc")
CLASSES = ("INT32", "FMA_F32", "ADD_F32", "MUL_F32", "TRANS_F32", "CVT")
FORMS = {"k_pk8": "v_pk_fma_f32", "k_fma8": "v_fma_f32", "k_add8": "v_add_u32",
         "k_mix": "v_pk_fma_f32 + v_max3_f32", "k_addf8": "v_add_f32", "k_mulf8": "v_mul_f32",
         "k_max8": "v_max_f32", "k_and8": "v_and_b32", "k_mullo8": "v_mul_lo_u32",
         "k_cnd8": "v_cndmask_b32", "k_cmp8": "v_cmp_ge_f32 (to SGPRs)", "k_sqrt8": "v_sqrt_f32"}


def load(prefix):
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for row in csv.DictReader(open(os.path.join(d, prefix + "_counter_collection.csv"))):
        per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
        names[row["Dispatch_Id"]] = row["Kernel_Name"].split("(")[0]
    dur = {}
    for row in csv.DictReader(open(os.path.join(d, prefix + "_kernel_trace.csv"))):
        dur[row["Dispatch_Id"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
    return per, names, dur


per, names, dur = load("ubench")
print("form                         cyc/inst/SIMD  ACTIVE/inst  class")
best = {}
for did in sorted(per, key=int):  # the second repetition of each kernel (the first warms up)
    best[names[did]] = did
for k, did in best.items():
    c = per[did]
    n = c["SQ_INSTS_VALU"]
    cyc = c["GRBM_GUI_ACTIVE"] / 8 * 1024 / n
    cls = [x for x in CLASSES if c.get("SQ_INSTS_VALU_" + x, 0) > 0.5 * n]
    print(f"{FORMS.get(k, k):28s} {cyc:10.2f}  {c['SQ_ACTIVE_INST_VALU'] / n:10.2f}   "
          f"{cls[0] if cls else '(none)'}")

per, names, dur = load("render")
for did, c in per.items():
    if names[did] != "rt_render_kernel":
        continue
    n = c["SQ_INSTS_VALU"]
    simd_cyc = 1024 * c["GRBM_GUI_ACTIVE"] / 8
    f = {x: c.get("SQ_INSTS_VALU_" + x, 0) for x in CLASSES}
    rest = n - sum(f.values())
    base = f["FMA_F32"] * 4 + (f["ADD_F32"] + f["MUL_F32"]) * 2 + f["TRANS_F32"] * 8 + \
        f["CVT"] * 4 + rest * 4
    lo, hi = (base + f["INT32"] * 2) / simd_cyc, (base + f["INT32"] * 4) / simd_cyc
    print(f"\nrt_render_kernel (one {dur[did]:.1f} ms launch, clock "
          f"{c['GRBM_GUI_ACTIVE'] / 8 / dur[did] / 1e6:.3f} GHz): {n:.4g} VALU instructions, "
          + ", ".join(f"{x} {v / n:.3f}" for x, v in f.items()) + f", other {rest / n:.3f}")
    print(f"  AMD VALUBusy (4 cycles per instruction): {c['SQ_ACTIVE_INST_VALU'] * 4 / simd_cyc:.3f}")
    print(f"  issue-weighted VALU busy: {lo:.3f} (INT32 at 2 cycles) .. {hi:.3f} (at 4)")
    break
