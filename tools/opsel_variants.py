"""Diagnostic builds for the op_sel finding: the
current tree with filter8's ray constants read through op_sel / op_sel_hi
half-broadcasts of 4 VGPR pairs (round 2's first form) instead of 7
duplicated pairs, in two register forms:
  tools/librt_opsel_fixed.so   outputs on hard-coded v[40:47], max chain inside
  tools/librt_opsel_owned.so   outputs on compiler-allocated registers
Both with RT_ISECT_PATHTAG (bit 24 of a hit index marks the matrix-core walk,
tools/isect_diag.py). The sources are patched in a temporary copy; nothing of
the product changes. usage: python tools/opsel_variants.py"""
import os
import re
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

OPSEL_OPS = [  # (dst, src0 pair, op_sel, op_sel_hi, sgpr operand, src2) per chain step
    ("r0", "cx", "op_sel:[0,0,1] op_sel_hi:[0,1,1]", "r1"),
    ("r0", "cy", "op_sel:[1,0,0] op_sel_hi:[1,1,1]", None),
    ("r1", "cz", "op_sel:[0,0,0] op_sel_hi:[0,1,1]", None),
    (None, "s", "", None),
    ("r3", "cz", "op_sel:[0,0,0] op_sel_hi:[0,1,1]", None),
    ("r2", "cy", "op_sel:[1,0,0] op_sel_hi:[1,1,1]", None),
    ("r2", "cx", "op_sel:[0,0,0] op_sel_hi:[0,1,1]", None),
]


def asm_lines():
    out = []
    for src0, sop, mods, first in OPSEL_OPS:
        for g in "abcd":
            h = f"%[h{g}]"
            if src0 is None:  # hb^2 + S
                out.append(f"v_pk_fma_f32 {h}, {h}, {h}, %[s{g}]")
            elif first:
                out.append(f"v_pk_fma_f32 {h}, %[{src0}], %[{sop}{g}], %[{first}] {mods}")
            else:
                out.append(f"v_pk_fma_f32 {h}, %[{src0}], %[{sop}{g}], {h} {mods}")
    return out


def filter8_src(fixed):
    lines = asm_lines()
    if fixed:
        lines += ["v_max3_f32 %[hm], v40, v41, v42", "v_max3_f32 %[hm], %[hm], v43, v44",
                  "v_max3_f32 %[hm], %[hm], v45, v46", "v_max_f32 %[hm], %[hm], v47"]
        outs = ('[ha] "={v[40:41]}"(ha), [hb] "={v[42:43]}"(hb), [hc] "={v[44:45]}"(hc), '
                '[hd] "={v[46:47]}"(hd), [hm] "=&v"(hmax)')
    else:
        outs = '[ha] "=&v"(ha), [hb] "=&v"(hb), [hc] "=&v"(hc), [hd] "=&v"(hd)'
    body = "\\n\\t".join(lines)
    ins = ('[r0] "v"(R.r0), [r1] "v"(R.r1), [r2] "v"(R.r2), [r3] "v"(R.r3), '
           + ", ".join(f'[{k}{g}] "s"({k}{g})' for k in ("cx", "cy", "cz", "s") for g in "abcd"))
    src = f'''struct RayP {{
    f2 r0, r1, r2, r3;  // (-dnx, -dny), (-dnz, k1), (o2x, o2y), (o2z, T)
    float T;
}};

__device__ __forceinline__ RayP ray_pack(const RayF& r) {{
    RayP p;
    p.r0 = f2{{r.dx.x, r.dy.x}};
    p.r1 = f2{{r.dz.x, r.k1.x}};
    p.r2 = f2{{r.o2x.x, r.o2y.x}};
    p.r3 = f2{{r.o2z.x, r.T}};
    p.T = r.T;
    return p;
}}

__device__ __forceinline__ void filter8(const RayP& R, f2 cxa, f2 cxb, f2 cxc, f2 cxd, f2 cya,
                                        f2 cyb, f2 cyc, f2 cyd, f2 cza, f2 czb, f2 czc, f2 czd,
                                        f2 sa, f2 sb, f2 sc, f2 sd, f2& ha, f2& hb, f2& hc,
                                        f2& hd, float& hmax) {{
    asm volatile("{body}" : {outs} : {ins});
'''
    if not fixed:
        src += '''    asm volatile("v_max3_f32 %0, %1, %2, %3\\n\\tv_max3_f32 %0, %0, %4, %5\\n\\t"
                 "v_max3_f32 %0, %0, %6, %7\\n\\tv_max_f32 %0, %0, %8"
                 : "=&v"(hmax) : "v"(ha.x), "v"(ha.y), "v"(hb.x), "v"(hb.y), "v"(hc.x),
                   "v"(hc.y), "v"(hd.x), "v"(hd.y));
'''
    return src + "}\n\n"


def build(name, fixed):
    tmp = tempfile.mkdtemp()
    try:
        shutil.copytree(os.path.join(ROOT, "bevy_raytrace_amd"), os.path.join(tmp, "bevy_raytrace_amd"),
                        ignore=shutil.ignore_patterns("*.so", "__pycache__"))
        shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
        p = os.path.join(tmp, "bevy_raytrace_amd", "csrc", "rt_dev_intersect.h")
        s = open(p).read()
        a = s.index("struct RayP {")
        b = s.index("__device__ __forceinline__ uint32_t ge(")
        s = s[:a] + filter8_src(fixed) + s[b:]
        open(p, "w").write(s)
        out = os.path.join(ROOT, "tools", name)
        subprocess.run(["make", "-s", "-C", os.path.dirname(p), f"OUT={out}",
                        "EXTRA=-DRT_ISECT_PATHTAG"], check=True)
        print("built", out)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    build("librt_opsel_fixed.so", True)
    build("librt_opsel_owned.so", False)
