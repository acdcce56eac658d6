"""Summary of a rocprofv3 stochastic PC-sampling run of the render kernel
(tools/gpu_r04_pcs.sh): where the waves of rt_render_kernel are when sampled,
whether they issued, and the stall reason when they did not -- overall, per
instruction, and per instruction class.

usage: python tools/pcs_summary.py <out dir of gpu_r04_pcs.sh> [kernel substring]
"""
import csv
import glob
import os
import re
import sys
from collections import Counter, defaultdict

d = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "rt_render_kernel"


def find(pattern):
    fs = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return fs[0] if fs else None


kt = find("*kernel_trace.csv")
disp = set()
if kt:
    for r in csv.DictReader(open(kt)):
        if kname in r.get("Kernel_Name", ""):
            disp.add(r.get("Dispatch_Id"))
ps = find("*pc_sampling*stochastic*.csv") or find("*pc_sampling*.csv")
if not ps:
    sys.exit(f"no pc sampling csv under {d}")
rows = list(csv.DictReader(open(ps)))
cols = list(rows[0].keys()) if rows else []
print(f"# {ps}: {len(rows)} samples, columns: {cols}")


def col(*names):
    for n in names:
        for c in cols:
            if c.lower() == n.lower():
                return c
    for n in names:
        for c in cols:
            if n.lower() in c.lower():
                return c
    return None


c_disp = col("Dispatch_Id")
c_inst = col("Instruction")
c_comm = col("Instruction_Comment")
c_iss = col("Wave_Issued_Instruction", "Wave_Issued")
c_stall = col("Stall_Reason")
c_type = col("Instruction_Type")
c_pc = col("Code_Object_Offset", "Pc", "Code_Object_Offset_Pc")
if disp and c_disp:
    rows = [r for r in rows if r[c_disp] in disp]
print(f"# {len(rows)} samples of {kname} (dispatches {sorted(disp)})")

tot = len(rows)
iss = Counter()
stall = Counter()
per_inst = defaultdict(Counter)
per_mn = defaultdict(Counter)
for r in rows:
    issued = r.get(c_iss, "") in ("1", "true", "True") if c_iss else False
    why = "ISSUED" if issued else (r.get(c_stall) or "?")
    stall[why] += 1
    key = (r.get(c_pc, ""), r.get(c_inst, ""))
    per_inst[key][why] += 1
    mn = (r.get(c_inst, "") or "?").split()[0] if r.get(c_inst) else "?"
    per_mn[mn][why] += 1
    if c_type:
        iss[(r.get(c_type), issued)] += 1

print("\n## samples by state (issued, or the reason the wave did not issue)")
for k, v in stall.most_common():
    print(f"{k:40s} {v:9d} {v / tot:7.3f}")
if c_type:
    print("\n## samples by instruction type x issued")
    for (t, i), v in sorted(iss.items(), key=lambda x: -x[1])[:30]:
        print(f"{str(t):40s} {'issued' if i else 'stalled':8s} {v:9d} {v / tot:7.3f}")
print("\n## top mnemonics (share of samples; top states)")
for mn, c in sorted(per_mn.items(), key=lambda x: -sum(x[1].values()))[:40]:
    n = sum(c.values())
    top = ", ".join(f"{k} {v / n:.2f}" for k, v in c.most_common(3))
    print(f"{mn:34s} {n / tot:7.3f}  {top}")
print("\n## top instructions (pc, text: share; top states)")
for (pc, txt), c in sorted(per_inst.items(), key=lambda x: -sum(x[1].values()))[:80]:
    n = sum(c.values())
    top = ", ".join(f"{k} {v / n:.2f}" for k, v in c.most_common(3))
    t = re.sub(r"\s+", " ", txt)[:70]
    print(f"{pc:>10s} {n / tot:7.4f}  {t:70s} {top}")
