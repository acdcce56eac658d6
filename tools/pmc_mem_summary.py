"""Summary of tools/pmc_mem.sh passes for the render kernel: L1 hit rate, L2
requests and their average latency, L2 hit rate, LDS bank conflicts, and the
waves' waiting / issuing shares, per traced segment where it helps.

usage: python tools/pmc_mem_summary.py <out dir> [<out dir> ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    tot = defaultdict(float)
    for f in sorted(glob.glob(os.path.join(d, "mem_*", "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        ids = [i for i in per if "rt_render_kernel" in names[i]]
        if ids:
            last = max(ids, key=int)
            for k, v in per[last].items():
                tot[k] = v  # GRBM_GUI_ACTIVE repeats per pass: the last pass's
    return tot


for d in sys.argv[1:]:
    c = load(d)
    g = lambda k: c.get(k, float("nan"))  # noqa: E731
    simd = 1024 * g("GRBM_GUI_ACTIVE") / 8
    print(f"== {d}")
    print(f"  L1: accesses {g('TCP_TOTAL_CACHE_ACCESSES_sum'):.4g}, reads {g('TCP_TOTAL_READ_sum'):.4g}, "
          f"L2 read requests {g('TCP_TCC_READ_REQ_sum'):.4g} "
          f"(miss share {g('TCP_TCC_READ_REQ_sum') / g('TCP_TOTAL_CACHE_ACCESSES_sum'):.3f}), "
          f"avg L2 read latency {g('TCP_TCC_READ_REQ_LATENCY_sum') / g('TCP_TCC_READ_REQ_sum'):.0f} cycles")
    print(f"  L1 pending stall {g('TCP_PENDING_STALL_CYCLES_sum'):.4g}, TCR stall {g('TCP_TCR_TCP_STALL_CYCLES_sum'):.4g}")
    print(f"  L2: hit {g('TCC_HIT_sum'):.4g} miss {g('TCC_MISS_sum'):.4g} "
          f"(hit rate {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f})")
    print(f"  VMEM rd {g('SQ_INSTS_VMEM_RD'):.4g} wr {g('SQ_INSTS_VMEM_WR'):.4g}  LDS {g('SQ_INSTS_LDS'):.4g} "
          f"SMEM {g('SQ_INSTS_SMEM'):.4g} SALU {g('SQ_INSTS_SALU'):.4g} branch {g('SQ_INSTS_BRANCH'):.4g}")
    print(f"  LDS bank conflict cycles {g('SQ_LDS_BANK_CONFLICT'):.4g}, LDS active {g('SQ_LDS_IDX_ACTIVE'):.4g}")
    wc = g("SQ_WAVE_CYCLES")
    print(f"  wave cycles {wc:.4g}: wait_inst_any {g('SQ_WAIT_INST_ANY') / wc:.3f}, wait_any "
          f"{g('SQ_WAIT_ANY') / wc:.3f}, wait_inst_lds {g('SQ_WAIT_INST_LDS') / wc:.3f}, active_any "
          f"{g('SQ_ACTIVE_INST_ANY') / wc:.3f}, active_lds {g('SQ_ACTIVE_INST_LDS') / wc:.3f}, "
          f"active_sca {g('SQ_ACTIVE_INST_SCA') / wc:.3f}, active_misc {g('SQ_ACTIVE_INST_MISC') / wc:.3f}")
    print(f"  (wave-cycle counters are per 4 cycles? raw ratios shown; SIMD cycles {simd:.4g})")
