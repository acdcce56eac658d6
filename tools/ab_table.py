"""Print an A/B table of bench.py JSON lines (tools/calls/gpu_r04_ab.sh,
gpu_r04_sens.sh output: ab_<arm>_<i>.json): Mrays/s, ms per step,
render-kernel ms per launch, the run's clock and the launch's cycles
(clock-independent), then each arm's mean cycles against `base`.
usage: python tools/ab_table.py <dir>"""
import glob
import json
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
rows = defaultdict(list)
wall = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "ab_*_[0-9].json"))):
    kind = re.match(r"ab_(.+)_\d+\.json$", os.path.basename(f)).group(1)
    j = json.load(open(f))
    r = j["roofline"]
    cyc = r["kernel_ms_per_launch"] * r["clock_ghz_run"]
    rows[kind].append(cyc)
    wall[kind].append(r["kernel_ms_per_launch"])
    print(f"{os.path.basename(f):28s} {j['value']:10.1f} Mrays/s {j['ms_per_step']:8.3f} ms/step "
          f"{r['kernel_ms_per_launch']:9.3f} ms {r['clock_ghz_run']:.4f} GHz {cyc:8.2f} Mcyc "
          f"frac {r['frac']}")
if rows.get("base"):
    b = sum(rows["base"]) / len(rows["base"])
    for k, v in rows.items():
        if k == "base":
            continue
        n = sum(v) / len(v)
        bw, nw = sum(wall["base"]) / len(wall["base"]), sum(wall[k]) / len(wall[k])
        print(f"mean Mcyc per launch: base {b:.2f}, {k} {n:.2f} ({(n / b - 1) * 100:+.2f} %); "
              f"ms {bw:.2f} vs {nw:.2f} ({(nw / bw - 1) * 100:+.2f} %)")
