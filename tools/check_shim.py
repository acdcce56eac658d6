#!/usr/bin/env python3
"""Static check of the Rust drop-in (bevy_shim/) against the reference crate,
run in the build container (no rustc here; /root/reference is read as text).

It applies bevy_shim/manifest.json to the reference's src/ virtually and
checks that the resulting crate is closed:
  1. every `mod x;` of lib.rs (after the manifest's edits) has a file, and
     every module file is declared;
  2. every `use crate::...` / inline `crate::a::B` path resolves to a module
     of the crate and a `pub` item of that module (or of lib.rs);
  3. no remaining file names an item that only a deleted file defined
     (e.g. `RayTracePipeline` of ray_trace_pipeline.rs, the resource the
     reference's ray_trace_output.rs `queue` system takes);
  4. every field the shim reads off another module's struct
     (`resource::<T>().field`, `.buffer.get().field`) is `pub` there.
Prints one line per finding and `OK` / `FAIL`; exit status 1 on a finding.
"""
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
MANIFEST = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "bevy_shim", "manifest.json")

ITEM = re.compile(r"^\s*(pub(?:\([a-z]+\))?\s+)?(?:unsafe\s+)?(struct|enum|fn|const|static|type|trait|mod)\s+"
                  r"([A-Za-z_][A-Za-z0-9_]*)", re.M)


def strip_comments(src):
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def items(src):
    """{name: is_pub} of the module's top-level-ish items."""
    out = {}
    for m in ITEM.finditer(strip_comments(src)):
        out[m.group(3)] = bool(m.group(1)) or out.get(m.group(3), False)
    return out


def struct_fields(src):
    """{struct: {field: is_pub}} (named and tuple structs)."""
    out = {}
    s = strip_comments(src)
    for m in re.finditer(r"struct\s+([A-Za-z_]\w*)\s*(?:<[^>]*>)?\s*\{(.*?)\n\}", s, re.S):
        out[m.group(1)] = {f.group(2): bool(f.group(1)) for f in
                           re.finditer(r"^\s*(pub\s+)?([a-z_]\w*)\s*:", m.group(2), re.M)}
    for m in re.finditer(r"struct\s+([A-Za-z_]\w*)\s*\(([^;]*)\)\s*;", s):
        out[m.group(1)] = {str(i): f.strip().startswith("pub") for i, f in
                           enumerate(m.group(2).split(","))}
    return out


def use_paths(src):
    """Every crate:: path: (module or None, item) pairs."""
    s = strip_comments(src)
    paths = []
    for m in re.finditer(r"\buse\s+crate::(.*?);", s, re.S):
        body = re.sub(r"\s+", "", m.group(1))
        def expand(prefix, rest):
            if rest.startswith("{") and rest.endswith("}"):
                depth, cur, parts = 0, "", []
                for ch in rest[1:-1]:
                    if ch == "," and depth == 0:
                        parts.append(cur)
                        cur = ""
                        continue
                    depth += ch == "{"
                    depth -= ch == "}"
                    cur += ch
                if cur:
                    parts.append(cur)
                for p in parts:
                    expand(prefix, p)
                return
            if "::" in rest and not rest.startswith("{"):
                head, tail = rest.split("::", 1)
                expand(prefix + [head], tail)
                return
            paths.append(prefix + [rest])
        expand([], body)
    for m in re.finditer(r"(?<!use )\bcrate::([A-Za-z_]\w*(?:::[A-Za-z_]\w*)*)", s):
        paths.append(m.group(1).split("::"))
    out = []
    for p in paths:
        p = [x.split("as")[0] if "as" in x and x != "as" else x for x in p]
        if len(p) == 1:
            out.append((None, p[0]))
        else:
            out.append((p[0], p[1]))
    return out


def main():
    man = json.load(open(MANIFEST))
    findings = []
    files = {}
    for f in glob.glob(os.path.join(REF, "src", "*.rs")):
        files["src/" + os.path.basename(f)] = open(f).read()
    deleted = {}
    for d in man["delete"]:
        path = os.path.join(REF, d)
        if not os.path.exists(path):
            findings.append(f"delete list names {d}, which the reference does not have")
            continue
        if d.endswith(".rs"):
            deleted[d] = files.pop(d)
    for dst, src in list(man["replace"].items()) + list(man["add"].items()):
        if dst in man["replace"] and dst not in files:
            findings.append(f"replace target {dst} is not in the reference")
        files[dst] = open(os.path.join(ROOT, src)).read()
    # lib.rs edits
    lib = files["src/lib.rs"]
    for mname in man["lib_rs"]["remove_mods"]:
        new = re.sub(rf"^\s*(pub\s+)?mod\s+{mname}\s*;\s*\n", "", lib, flags=re.M)
        if new == lib:
            findings.append(f"lib.rs has no `mod {mname};` to remove")
        lib = new
    for mname in man["lib_rs"]["add_mods"]:
        lib = f"mod {mname};\n" + lib
    files["src/lib.rs"] = lib
    mods = set(re.findall(r"^\s*(?:pub\s+)?mod\s+([a-z_]\w*)\s*;", strip_comments(lib), re.M))
    for m in sorted(mods):
        if f"src/{m}.rs" not in files:
            findings.append(f"lib.rs declares `mod {m};` but src/{m}.rs is gone")
    for f in sorted(files):
        if f.startswith("src/") and f not in ("src/lib.rs", "src/main.rs"):
            if os.path.basename(f)[:-3] not in mods:
                findings.append(f"{f} is not declared in lib.rs")
    # 2. paths
    mod_items = {f"src/{m}.rs"[4:-3]: items(files[f"src/{m}.rs"]) for m in mods
                 if f"src/{m}.rs" in files}
    root_items = items(lib)
    for f, src in sorted(files.items()):
        if not f.endswith(".rs") or f == "build.rs":
            continue
        for mod, it in use_paths(src):
            if mod is None:
                if it not in root_items and it not in mods:
                    findings.append(f"{f}: crate::{it} is not defined at the crate root")
                continue
            if mod not in mod_items:
                findings.append(f"{f}: crate::{mod}::{it} -- module {mod} is not in the crate")
                continue
            if it in ("*", "self"):
                continue
            if it not in mod_items[mod]:
                findings.append(f"{f}: crate::{mod}::{it} -- {mod} defines no {it}")
            elif not mod_items[mod][it]:
                findings.append(f"{f}: crate::{mod}::{it} is not pub")
    # 3. items only deleted files defined
    kept_defs = set()
    for f, src in files.items():
        if f.endswith(".rs"):
            kept_defs |= set(items(src))
    gone = set()
    for src in deleted.values():
        gone |= {n for n in items(src) if n not in kept_defs and n[0].isupper()}
    for f, src in sorted(files.items()):
        if not f.endswith(".rs"):
            continue
        s = strip_comments(src)
        for n in sorted(gone):
            if re.search(rf"\b{n}\b", s):
                findings.append(f"{f}: uses {n}, defined only in a deleted file")
    # 4. fields the replaced/added files read off other modules' structs
    fields = {}
    for f, src in files.items():
        if f.endswith(".rs"):
            for k, v in struct_fields(src).items():
                fields.setdefault(k, {}).update(v)
    for dst in list(man["replace"]) + list(man["add"]):
        if not dst.endswith(".rs"):
            continue
        s = strip_comments(files[dst])
        for m in re.finditer(r"resource::<([A-Z]\w*)>\(\)\s*\.\s*(\w+)", s):
            t, fld = m.group(1), m.group(2)
            if t in fields and fld in fields[t] and not fields[t][fld]:
                findings.append(f"{dst}: reads private field {t}.{fld}")
            elif t in fields and fld not in fields[t] and not fld[0].isupper() and fld not in (
                    "get", "clone", "iter", "get_mut"):
                findings.append(f"{dst}: {t} has no field {fld}")
        for m in re.finditer(r"resource::<([A-Z]\w*)>\(\)\s*\.\s*buffer\s*\.\s*get\(\)\s*\.\s*(\w+)", s):
            t, fld = m.group(1), m.group(2)
            inner = {"GlobalsGPUStorage": "GlobalsGPU", "ObjectListStorage": "ObjectListGPU",
                     "CameraGPUStorage": "CameraGPU"}.get(t)
            if inner and fld in fields.get(inner, {}) and not fields[inner][fld]:
                findings.append(f"{dst}: reads private field {inner}.{fld}")
    for x in findings:
        print(x)
    print("OK" if not findings else f"FAIL ({len(findings)})")
    print(f"crate after the shim: {len(mods)} modules ({', '.join(sorted(mods))}); "
          f"deleted {len(deleted)} .rs files; items only they defined: {len(gone)}")
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main())
