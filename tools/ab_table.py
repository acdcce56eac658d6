"""Print an A/B table of bench.py JSON lines (tools/gpu_r04_ab.sh output):
Mrays/s, ms per step, render-kernel ms per launch, the run's clock and the
launch's cycles (clock-independent). usage: python tools/ab_table.py <dir>"""
import glob
import json
import os
import sys

d = sys.argv[1]
rows = {"base": [], "new": []}
for f in sorted(glob.glob(os.path.join(d, "ab_*_[0-9].json"))):
    kind = os.path.basename(f).split("_")[1]
    j = json.load(open(f))
    r = j["roofline"]
    cyc = r["kernel_ms_per_launch"] * r["clock_ghz_run"]
    rows[kind].append(cyc)
    print(f"{os.path.basename(f):16s} {j['value']:10.1f} Mrays/s {j['ms_per_step']:8.3f} ms/step "
          f"{r['kernel_ms_per_launch']:9.3f} ms {r['clock_ghz_run']:.4f} GHz {cyc:8.2f} Mcyc "
          f"frac {r['frac']}")
if rows["base"] and rows["new"]:
    b, n = sum(rows["base"]) / len(rows["base"]), sum(rows["new"]) / len(rows["new"])
    print(f"mean Mcyc per launch: base {b:.2f}, new {n:.2f} ({(n / b - 1) * 100:+.2f} %)")
