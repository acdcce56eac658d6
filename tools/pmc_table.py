"""Table of tools/pmc_ab.sh passes: per build, the render kernel's counters per
launch (summed over dimensions), its duration and derived rates.
usage: python tools/pmc_table.py [gpurun_out]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
KERNEL = os.environ.get("KERNEL", "rt_render_kernel")
builds = defaultdict(dict)
durs = defaultdict(list)
for path in sorted(glob.glob(os.path.join(d, "pab_*_*"))):
    m = re.match(r"pab_(\d+)_(\d+)$", os.path.basename(path))
    if not m or not os.path.isdir(path):
        continue
    b = int(m.group(1))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(f)):
            if row["Kernel_Name"].split("(")[0] != KERNEL:
                continue
            per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
        for c in per.values():  # one render launch per pass
            builds[b].update(c)
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Kernel_Name"].split("(")[0] == KERNEL:
                durs[b].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
names = sorted({k for c in builds.values() for k in c})
print(f"{'counter':28s}" + "".join(f"{'build ' + str(b):>18s}" for b in sorted(builds)))
for n in names:
    print(f"{n:28s}" + "".join(f"{builds[b].get(n, float('nan')):18.4g}" for b in sorted(builds)))
print(f"{'kernel ms (mean of passes)':28s}" +
      "".join(f"{sum(durs[b]) / max(1, len(durs[b])):18.3f}" for b in sorted(builds)))
for b in sorted(builds):
    c = builds[b]
    g = c.get("GRBM_GUI_ACTIVE", 0) / 8
    w = c.get("SQ_WAVE_CYCLES", 0)
    if g and w:
        print(f"build {b}: clock {g / (sum(durs[b]) / len(durs[b])) / 1e6:.3f} GHz, "
              f"cyc/VALU/SIMD {g * 1024 / c['SQ_INSTS_VALU']:.3f}, "
              f"wave: issuing {c['SQ_ACTIVE_INST_ANY'] / w:.3f} waiting {c['SQ_WAIT_ANY'] / w:.3f} "
              f"issue-stalled {c['SQ_WAIT_INST_ANY'] / w:.3f} (LDS {c.get('SQ_WAIT_INST_LDS', 0) / w:.3f})")
