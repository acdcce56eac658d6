"""Static instruction mix of rt_render_kernel by phase, from its assembly built
with line tables (`make asm EXTRA=-gline-tables-only`: the same code as the
product, tools/isa_diff.py checks it): every instruction is attributed to the
source line of its `.loc` (the innermost inlined location); lines of shared
helpers (rt_math.h, rt_dev_math.h, the HIP headers) inherit the phase of the
instruction before them. Phases follow the RT_PROFILE marks (rt_kernels.hip
render_body, rt_dev_intersect.h intersect_world_mfma): refill, setup (ray
column + bound tiles), walk (tiles + queue appends), drain (exact tests),
shade (the shading loop + slot buffer), other. Prints, per phase and per
basic block, the instruction counts by class and the issue cycles one pass
costs at 4 waves per SIMD (profiles/r04/valu_forms/table.txt: dual-issued
forms 2.32 cycles, other VALU 4, transcendentals 8, an MFMA 8 of issue).
usage: python tools/isa_phases.py <asm.s> [--blocks]"""
import re
import sys
from collections import defaultdict

DUAL = re.compile(r"^v_(fma_f32|fmac_f32|add_f32|sub_f32|subrev_f32|mul_f32|add_u32|sub_u32|subrev_u32|"
                  r"and_b32|or_b32|xor_b32|bitop3_b32|mov_b32)")
TRANS = re.compile(r"^v_(rcp|rsq|sqrt|exp|log|sin|cos)_f32")


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if TRANS.match(op):
            return "trans"
        return "valu2" if DUAL.match(op) else "valu"
    return "other"


CYC = {"valu2": 2.32, "valu": 4.0, "trans": 8.0, "mfma": 8.0}


def phase_of(fname, line, fns):
    """(file, line) -> phase, or None for a shared helper line."""
    f = fname.split("/")[-1]
    if f == "rt_dev_intersect.h":
        for name, (a, b) in fns.items():
            if ":" not in name and a <= line <= b:
                return name
        return None
    if f == "rt_dev_path.h":
        for name, (a, b) in fns.items():
            if name.startswith("path:") and a <= line <= b:
                return name[5:]
        return None
    if f == "rt_kernels.hip":
        for name, (a, b) in fns.items():
            if name.startswith("k:") and a <= line <= b:
                return name[2:]
        return None
    return None


def source_ranges(root):
    """Line ranges of the phase-defining code, found by markers in the sources."""
    def find(path, pat, start=0):
        lines = open(path).read().splitlines()
        for i in range(start, len(lines)):
            if re.search(pat, lines[i]):
                return i + 1
        raise KeyError(pat)
    di = f"{root}/bevy_raytrace_amd/csrc/rt_dev_intersect.h"
    dp = f"{root}/bevy_raytrace_amd/csrc/rt_dev_path.h"
    kh = f"{root}/bevy_raytrace_amd/csrc/rt_kernels.hip"
    r = {}
    ex0 = find(di, r"__device__ __forceinline__ void exact_core")
    r["drain"] = (ex0 - 3, find(di, r"^__device__ __forceinline__ void exact_test"))
    r["drain2"] = (find(di, r"void mfma_drain"), find(di, r"^// The ORs of a tile"))
    r["walk_or"] = (find(di, r"^// The ORs of a tile"), find(di, r"^// Called by the whole wave"))
    w0 = find(di, r"int intersect_world_mfma\(")
    r["setup"] = (w0, find(di, r"float best_t = VERY_FAR;", w0))
    r["walk"] = (find(di, r"float best_t = VERY_FAR;", w0), find(di, r"^#endif  // RT_MFMA_FILTER"))
    r["path:refill"] = (find(dp, r"void start_sample"), find(dp, r"^// One path step after"))
    r["path:shade"] = (find(dp, r"^// One path step after"), find(dp, r"^// ---- collect"))
    b0 = find(kh, r"void render_body\(")
    r["k:refill"] = (find(kh, r"---- refill", b0), find(kh, r"---- intersect \(intersect", b0))
    r["k:setup"] = (find(kh, r"---- intersect \(intersect", b0), find(kh, r"---- shade; a finished", b0))
    r["k:shade"] = (find(kh, r"---- shade; a finished", b0), find(kh, r"^    sb_flush\(\);", b0))
    return r


def main():
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fns = source_ranges(root)
    text = open(sys.argv[1]).read().splitlines()
    files = {}
    start = next(i for i, l in enumerate(text) if re.match(r"^_Z16rt_render_kernel\S*:", l))
    cur_loc, cur_phase = None, "other"
    blocks = []  # (label, phase counts)
    blk = None
    per_phase = defaultdict(lambda: defaultdict(int))
    for l in text[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"\s*\.file\s+(\d+)\s+\"([^\"]*)\"\s+\"([^\"]*)\"", l)
        if m:
            files[int(m.group(1))] = m.group(3)
            continue
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            fi, ln = int(m.group(1)), int(m.group(2))
            if ln:
                ph = phase_of(files.get(fi, "?"), ln, fns)
                if ph:
                    cur_phase = {"drain2": "drain", "walk_or": "walk"}.get(ph, ph)
            continue
        if re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:)", l):
            blk = {"label": l.split()[0].rstrip(":") if l.startswith(".") else l.split()[1].rstrip(":"),
                   "n": defaultdict(int), "phase": None}
            blocks.append(blk)
            continue
        t = l.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        op = t.split()[0]
        k = klass(op)
        per_phase[cur_phase][k] += 1
        if blk is not None:
            blk["n"][k] += 1
            blk["phase"] = blk["phase"] or cur_phase
    print("static instructions per phase (one pass through every block):")
    for ph, n in sorted(per_phase.items()):
        cyc = sum(CYC.get(k, 0) * v for k, v in n.items())
        print(f"  {ph:8s} " + " ".join(f"{k}={v}" for k, v in sorted(n.items())) + f"  issue {cyc:.0f} cyc")
    if "--blocks" in sys.argv:
        for b in blocks:
            n = b["n"]
            cyc = sum(CYC.get(k, 0) * v for k, v in n.items())
            print(f"{b['label']:12s} {b['phase'] or '-':8s} " + " ".join(f"{k}={v}" for k, v in sorted(n.items()))
                  + f"  {cyc:.0f}")


if __name__ == "__main__":
    main()
