"""Compare one kernel's instruction stream between two `make asm` outputs
(labels and comments dropped, register numbers kept): a change meant to leave
the render kernel untouched must print "identical".
usage: python tools/isa_diff.py a.s b.s [kernel substring, default rt_render_kernel]"""
import difflib
import re
import sys


def body(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines)
                 if re.match(r"^_Z\d+" + name + r"\S*:", l))
    out = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        t = l.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        out.append(re.sub(r"\.LBB\d+_\d+", "L", t))
    return out


def main():
    a, b = sys.argv[1], sys.argv[2]
    name = sys.argv[3] if len(sys.argv) > 3 else "rt_render_kernel"
    x, y = body(a, name), body(b, name)
    if x == y:
        print(f"{name}: identical ({len(x)} instructions)")
        return 0
    d = list(difflib.unified_diff(x, y, lineterm="", n=1))
    print(f"{name}: {len(x)} -> {len(y)} instructions, {sum(1 for l in d if l[:1] in '+-') - 2} lines differ")
    print("\n".join(d[:80]))
    return 1


if __name__ == "__main__":
    sys.exit(main())
