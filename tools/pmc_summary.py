"""Summarise the rocprofv3 PMC passes of tools/pmc_round.sh (gpurun_out/pmc_*)
into profiles/<round>_pmc_<workload>.json and profiles/pmc_traffic.json.

HBM bytes per render launch follow /opt/skills/guides/MI355X_MICROARCH.md
(HBM section): FETCH_SIZE and WRITE_SIZE in separate passes, in KB (x1024);
gfx950's FETCH_SIZE counts half the bytes of wide streaming reads (x2)."""
import csv, glob, json, os, sys
from collections import defaultdict

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out_dir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "gpurun_out")
tag = sys.argv[2] if len(sys.argv) > 2 else "r01"
wl = sys.argv[3] if len(sys.argv) > 3 else "rtiow1080"
fpl = int(sys.argv[4]) if len(sys.argv) > 4 else 24

vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> per-dispatch values
durs = defaultdict(list)
for f in sorted(glob.glob(os.path.join(out_dir, "pmc_*", "**", "*counter_collection.csv"),
                          recursive=True)):
    per = defaultdict(float)
    names = {}
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row["Kernel_Name"].split("(")[0]
            key = (row["Dispatch_Id"], row["Counter_Name"])
            per[key] += float(row["Counter_Value"])   # summed over dimensions
            names[row["Dispatch_Id"]] = k
    for (d, c), v in per.items():
        vals[names[d]][c].append(v)
for f in glob.glob(os.path.join(out_dir, "pmc_*", "**", "*kernel_trace.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row["Kernel_Name"].split("(")[0]
            durs[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)

mean = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
# the render kernel the workload ran: rt_render_kernel (lists of <= 16
# blocks) or rt_render_multi_kernel (longer lists), the one with the most time
RK = max((k for k in durs if k in ("rt_render_kernel", "rt_render_multi_kernel")),
         key=lambda k: sum(durs[k]), default="rt_render_kernel")
rk = mean.get(RK, {})
summary = {"command": "tools/pmc_round.sh: rocprofv3 --kernel-trace --pmc <group> -- python3 bench.py "
                      f"--steps {fpl} --warmup 0 --frames-per-launch {fpl} --no-cpu-baseline --reuse-steps 0",
           "render_kernel": RK,
           "per_dispatch_mean": mean,
           "render_kernel_ms_under_pmc": (sum(durs[RK]) / len(durs[RK]) if durs[RK] else None)}
if rk:
    w = rk.get("SQ_WAVE_CYCLES"), rk.get("SQ_BUSY_CYCLES"), rk.get("GRBM_GUI_ACTIVE")
    if rk.get("SQ_ACTIVE_INST_VALU") and rk.get("SQ_WAVES"):
        summary["valu_inst_per_wave"] = rk["SQ_INSTS_VALU"] / rk["SQ_WAVES"]
with open(os.path.join(root, "profiles", f"{tag}_pmc_{wl}.json"), "w") as fh:
    json.dump(summary, fh, indent=1)
if "FETCH_SIZE" in rk and "WRITE_SIZE" in rk:
    fetch = rk["FETCH_SIZE"] * 1024 * 2
    write = rk["WRITE_SIZE"] * 1024
    tp = os.path.join(root, "profiles", "pmc_traffic.json")
    d = json.load(open(tp)) if os.path.exists(tp) else {}
    d[wl] = {"render_kernel": RK, "hbm_bytes_per_launch": int(fetch + write), "fetch_bytes": int(fetch),
             "write_bytes": int(write), "frames_per_launch": fpl,
             "source": f"profiles/{tag}_pmc_{wl}.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, "
                       "separate passes; FETCH_SIZE x2 per gfx950 correction, x1024 KB->B)",
             "note": f"per {fpl}-frame render launch"}
    # VALU occupancy of the same launch (separate --pmc pass), two historical
    # forms kept for comparison with rounds 1-3: AMD's VALUBusy (one quad-cycle
    # per counted SQ_ACTIVE_INST_VALU, which ignores gfx950's dual issue and
    # can exceed 1) and round 3's price form (every non-INT32 op 4 cycles,
    # INT32 2). Neither is the roofline: the measured SIMD-issue busy below
    # subtracts the dual-issued quad-cycles (SQ_ACTIVE_INST_VALU2) instead of
    # pricing by class (profiles/r04/valu_forms/table.txt).
    if rk.get("SQ_ACTIVE_INST_VALU") and rk.get("GRBM_GUI_ACTIVE"):
        simd_cycles = 1024 * rk["GRBM_GUI_ACTIVE"] / 8
        ent = d[wl]
        ent["valu"] = {
            "sq_active_inst_valu": rk["SQ_ACTIVE_INST_VALU"], "sq_insts_valu": rk.get("SQ_INSTS_VALU"),
            "sq_insts_valu_int32": rk.get("SQ_INSTS_VALU_INT32"),
            "grbm_gui_active": rk["GRBM_GUI_ACTIVE"],
            "kernel_ms_under_pmc": summary["render_kernel_ms_under_pmc"],
            "valubusy_amd": rk["SQ_ACTIVE_INST_VALU"] * 4 / simd_cycles,
            "formula_amd": "SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)",
        }
        if rk.get("SQ_INSTS_VALU_INT32") is not None and rk.get("SQ_INSTS_VALU"):
            i32 = rk["SQ_INSTS_VALU_INT32"]
            mf = rk.get("SQ_INSTS_MFMA") or 0.0  # counted in SQ_INSTS_VALU (mfma_count ubench)
            ent["valu"]["valubusy_issue"] = ((rk["SQ_INSTS_VALU"] - mf - i32) * 4 + i32 * 2) / simd_cycles
            ent["valu"]["formula_issue"] = ("((SQ_INSTS_VALU - SQ_INSTS_MFMA - SQ_INSTS_VALU_INT32) x 4 + "
                                            "SQ_INSTS_VALU_INT32 x 2) / (1024 x GRBM_GUI_ACTIVE / 8)")
    # matrix-core filter (f16 MFMA tiles) of the same launch: executed MFMA
    # flops (MOPS x 512) and the matrix pipe's busy share of the SIMD cycles
    if rk.get("SQ_INSTS_VALU_MFMA_MOPS_F16") and rk.get("GRBM_GUI_ACTIVE"):
        simd_cycles = 1024 * rk["GRBM_GUI_ACTIVE"] / 8
        d[wl]["mfma"] = {
            "mfma_f16_flops": rk["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512,
            "sq_insts_mfma": rk.get("SQ_INSTS_MFMA"),
            "sq_valu_mfma_busy_cycles": rk.get("SQ_VALU_MFMA_BUSY_CYCLES"),
            "mfma_busy": (rk["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
                          if rk.get("SQ_VALU_MFMA_BUSY_CYCLES") else None),
            "formula_busy": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)",
            "formula_flops": "SQ_INSTS_VALU_MFMA_MOPS_F16 x 512",
        }
    # SIMD issue, the resource the kernel is bound by, MEASURED
    # rather than priced: SQ_ACTIVE_INST_VALU counts the quad-cycles each VALU
    # instruction occupies its SIMD's vector issue (1 for a wave64 VALU op or an
    # MFMA, 2 for a transcendental), and SQ_ACTIVE_INST_VALU2 the quad-cycles in
    # which the SIMD issued two VALU instructions (gfx950 dual-issues v_fma_f32 /
    # v_fmac / v_add / v_sub / v_mul _f32, v_add / v_sub _u32, v_and / v_or /
    # v_xor / v_bitop3 _b32 and v_mov_b32: 0.58 quad-cycles each at 4 waves per
    # SIMD; every other form a full one -- tools/ubench/valu_forms,
    # profiles/r04/valu_forms/), so (ACTIVE_INST_VALU - ACTIVE_INST_VALU2) is the
    # quad-cycles the VALU issue port was taken. An MFMA holds the issue for 8
    # cycles (MI355X_MICROARCH.md, issue-cost row): one counted quad-cycle + 4
    # cycles more each.
    if (rk.get("SQ_ACTIVE_INST_VALU") and rk.get("SQ_ACTIVE_INST_VALU2") is not None
            and rk.get("GRBM_GUI_ACTIVE") and rk.get("SQ_INSTS_MFMA") is not None):
        simd_cycles = 1024 * rk["GRBM_GUI_ACTIVE"] / 8
        mf = rk["SQ_INSTS_MFMA"]
        valu_cyc = 4 * (rk["SQ_ACTIVE_INST_VALU"] - rk["SQ_ACTIVE_INST_VALU2"])
        issue = valu_cyc + 4 * mf
        kms = summary["render_kernel_ms_under_pmc"]
        d[wl]["simd_issue"] = {
            "issue_cycles_per_launch": issue,
            "valu_cycles": valu_cyc, "mfma_extra_hold_cycles": 4 * mf,
            "simd_cycles": simd_cycles,
            "busy": issue / simd_cycles,
            "valu_share": valu_cyc / simd_cycles,
            "mfma_share": 4 * mf / simd_cycles,
            "dual_issued_share_of_valu_quads": rk["SQ_ACTIVE_INST_VALU2"] / rk["SQ_ACTIVE_INST_VALU"],
            "clock_ghz": rk["GRBM_GUI_ACTIVE"] / 8 / (kms * 1e-3) / 1e9 if kms else None,
            "kernel_ms_under_pmc": kms,
            "formula": "(4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) + 4 x SQ_INSTS_MFMA) / "
                       "(1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)",
            "prices": {"dual-issue forms (v_fma/v_fmac/v_add/v_sub/v_mul_f32, v_add/v_sub_u32, "
                       "v_and/v_or/v_xor/v_bitop3_b32, v_mov_b32)": "0.58 quad-cycles measured "
                       "(2.3 cycles) when paired, 4 cycles alone",
                       "other VALU forms": "4 cycles", "transcendental": "8 cycles",
                       "MFMA 32x32x16": "8 cycles of issue (32 of matrix pipe)"},
            "price_source": "tools/ubench/valu_forms at 4 waves/SIMD + its PMC passes "
                            "(profiles/r04/valu_forms/table.txt)",
            "raw_record": f"profiles/{tag}_pmc_{wl}.json",
            "clock_formula": "GRBM_GUI_ACTIVE / 8 XCDs / render kernel time under the profiler",
        }
    json.dump(d, open(tp, "w"), indent=1)
print(json.dumps({k: summary[k] for k in summary if k != "per_dispatch_mean"}, indent=1))
print(json.dumps(rk, indent=1))
