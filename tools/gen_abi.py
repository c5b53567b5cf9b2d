"""Generate the ABI artefacts that mirror include/shd_accel.h, and parse them back (tests).

    python tools/gen_abi.py            rewrite rust/shadow-accel-sys/src/lib.rs and
                                       tests/abi/shd_layout.c from the header

* rust/shadow-accel-sys/src/lib.rs: the `-sys` crate's declarations (`#[repr(C)]` structs, the
  constants, every `extern "C"` function), the role cbindgen plays for the reference's own C
  headers (src/main/build.rs:42-130), run the other way: C header -> Rust.
* tests/abi/shd_layout.c: `_Static_assert`s of sizeof / offsetof for every field of every struct
  the header defines, with the numbers gcc gives on this (LP64) target.  Compiled by the CPU tests
  (tests/test_abi_layout.py), which also hold the ctypes mirror (shadow_amd/_native.py) and the
  Rust structs (laid out by C's rules) against the same numbers.
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "shd_accel.h")
RUST = os.path.join(ROOT, "rust", "shadow-accel-sys", "src", "lib.rs")
LAYOUT_C = os.path.join(ROOT, "tests", "abi", "shd_layout.c")

C2R = {"uint8_t": "u8", "uint32_t": "u32", "int32_t": "i32", "uint64_t": "u64", "int64_t": "i64",
       "int": "c_int", "float": "f32", "double": "f64", "size_t": "usize", "char": "c_char", "void": "c_void"}
# C layout of the Rust-side types (LP64)
RSIZE = {"u8": 1, "u32": 4, "i32": 4, "u64": 8, "i64": 8, "c_int": 4, "f32": 4, "f64": 8, "usize": 8,
         "c_char": 1, "shd_status": 4}


def _strip(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def header_src() -> str:
    return _strip(open(HEADER).read())


def parse_structs(src: str | None = None) -> dict[str, list[tuple[str, str]]]:
    """{struct: [(field, C type), ...]} of every `typedef struct X { ... } X;` in the header."""
    src = src if src is not None else header_src()
    out = {}
    for name, body in re.findall(r"typedef struct (\w+)\s*\{(.*?)\}\s*\w+\s*;", src, flags=re.S):
        fields = []
        for decl in [d.strip() for d in body.split(";") if d.strip()]:
            decl = re.sub(r"\s+", " ", decl)
            fp = re.match(r"(.+?)\(\s*\*\s*(\w+)\s*\)\s*\((.*)\)$", decl)
            if fp:   # function pointer field
                fields.append((fp.group(2), "fnptr:" + fp.group(1).strip() + "|" + fp.group(3)))
                continue
            m = re.match(r"((?:const )?\w+(?: ?\*)*) ?(.*)$", decl)
            base, names = m.group(1), m.group(2)
            for nm in names.split(","):
                nm = nm.strip()
                stars = len(nm) - len(nm.lstrip("*"))
                fields.append((nm.lstrip("*").strip(), (base + "*" * stars).replace(" *", "*")))
        out[name] = fields
    return out


def parse_functions(src: str | None = None) -> dict[str, tuple[str, list[tuple[str, str]]]]:
    """{name: (return C type, [(arg, C type), ...])} of every shd_* prototype in the header."""
    src = src if src is not None else header_src()
    out = {}
    for ret, name, args in re.findall(r"^([a-z_][\w ]*?\**)\s*\b(shd_\w+)\s*\(([^;{]*?)\)\s*;", src, flags=re.M):
        al = []
        args = re.sub(r"\s+", " ", args).strip()
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                m = re.match(r"(.*?)(\w+)$", a)
                al.append((m.group(2), m.group(1).replace(" ", "").replace("const", "const ")))
        out[name] = (ret.replace(" ", ""), al)
    return out


def parse_consts(src: str | None = None) -> dict[str, int]:
    src = src if src is not None else header_src()
    out = {}
    for k, v in re.findall(r"#define (SHD_\w+) (0x[0-9A-Fa-f]+|\d+)u?\b", src):
        out[k] = int(v, 0)
    for k, v in re.findall(r"\b(SHD_(?:OK|ERR_\w+)) = (\d+)", src):
        out[k] = int(v)
    return out


def rust_type(ct: str) -> str:
    ct = ct.strip()
    stars = ct.count("*")
    base = ct.replace("*", "").strip()
    const = base.startswith("const ")
    base = base.replace("const ", "").strip()
    r = C2R.get(base, base)
    if stars == 0:
        return r
    if stars == 1:
        return ("*const " if const else "*mut ") + r
    # T** (const applies to the pointee): *mut *mut T / *mut *const T
    return "*mut " + ("*const " if const else "*mut ") + r


def gen_rust() -> str:
    src = header_src()
    L = ["// Generated from include/shd_accel.h by tools/gen_abi.py -- do not edit by hand.",
         "// tests/test_abi_layout.py holds every struct's C layout and the function list against the header.",
         "#![allow(non_camel_case_types, non_upper_case_globals, dead_code)]",
         "use std::os::raw::{c_char, c_int, c_void};", "",
         "pub type shd_status = i32;"]
    for k, v in parse_consts(src).items():
        ty = "shd_status" if k == "SHD_OK" or k.startswith("SHD_ERR_") else ("u32" if v < 2**32 else "u64")
        L.append(f"pub const {k}: {ty} = {v:#x};" if v >= 0x10000 else f"pub const {k}: {ty} = {v};")
    L += ["", "#[repr(C)] pub struct shd_ctx { _p: [u8; 0] }", "#[repr(C)] pub struct shd_gml { _p: [u8; 0] }", ""]
    for name, fields in parse_structs(src).items():
        body = []
        for f, ct in fields:
            if ct.startswith("fnptr:"):
                ret, args = ct[6:].split("|")
                at = ", ".join(rust_type(re.match(r"(.*?)(\w+)$", a.strip()).group(1).replace(" ", "").replace("const", "const "))
                               for a in args.split(","))
                rt = "" if ret == "void" else " -> " + rust_type(ret)
                body.append(f"    pub {f}: Option<unsafe extern \"C\" fn({at}){rt}>,")
            else:
                body.append(f"    pub {f}: {rust_type(ct)},")
        L.append(f"#[repr(C)] #[derive(Clone, Copy)] pub struct {name} {{")
        L += body
        L.append("}")
    L += ["", "extern \"C\" {"]
    for name, (ret, args) in parse_functions(src).items():
        a = ", ".join(f"{n}: {rust_type(t)}" for n, t in args)
        rt = "" if ret == "void" else " -> " + rust_type(ret)
        L.append(f"    pub fn {name}({a}){rt};")
    L += ["}", ""]
    return "\n".join(L)


def probe_layout() -> dict:
    """gcc's sizeof / offsetof of every struct field (compiled against the header)."""
    structs = parse_structs()
    lines = ["#include <stddef.h>", "#include <stdio.h>", '#include "shd_accel.h"', "int main(void) {",
             '  printf("{");']
    first = True
    for name, fields in structs.items():
        sep = "" if first else ","
        first = False
        lines.append(f'  printf("{sep}\\"{name}\\": {{\\"size\\": %zu, \\"align\\": %zu, \\"fields\\": {{", '
                     f"sizeof({name}), _Alignof({name}));")
        for i, (f, _) in enumerate(fields):
            s2 = "" if i == 0 else ","
            lines.append(f'  printf("{s2}\\"{f}\\": [%zu, %zu]", offsetof({name}, {f}), sizeof((({name}*)0)->{f}));')
        lines.append('  printf("}}");')
    lines += ['  printf("}\\n");', "  return 0;", "}"]
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        exe = os.path.join(d, "p")
        open(c, "w").write("\n".join(lines))
        subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), c, "-o", exe])
        return json.loads(subprocess.check_output([exe]).decode())


def gen_layout_c(layout: dict) -> str:
    L = ["/* Generated by tools/gen_abi.py from include/shd_accel.h (gcc, LP64): the ABI of every struct,",
         " * pinned.  Compiled by tests/test_abi_layout.py; a layout change fails here until the generator",
         " * is rerun and the change is reviewed (SHD_ABI_VERSION, INTEGRATION.md, the Rust crate). */",
         "#include <stddef.h>", '#include "shd_accel.h"', ""]
    for name, v in layout.items():
        L.append(f'_Static_assert(sizeof({name}) == {v["size"]}, "{name} size");')
        for f, (off, sz) in v["fields"].items():
            L.append(f'_Static_assert(offsetof({name}, {f}) == {off}, "{name}.{f} offset");')
    L.append("")
    L.append("int shd_layout_checked(void) { return 1; }")
    L.append("")
    return "\n".join(L)


def rust_layout(path: str = RUST) -> dict:
    """C layout of the Rust crate's #[repr(C)] structs (field types from the crate's own text)."""
    txt = open(path).read()
    out = {}
    for name, body in re.findall(r"#\[repr\(C\)\](?: #\[derive\([^)]*\)\])? pub struct (\w+) \{\n(.*?)\n\}", txt, flags=re.S):
        off, align, fields = 0, 1, {}
        for f, ty in re.findall(r"pub (\w+): ([^,\n]+),", body):
            ty = ty.strip()
            if ty.startswith("*") or ty.startswith("Option<"):
                sz = 8
            else:
                sz = RSIZE[ty]
            off = (off + sz - 1) // sz * sz
            fields[f] = [off, sz]
            off += sz
            align = max(align, sz)
        out[name] = {"size": (off + align - 1) // align * align, "fields": fields}
    return out


def rust_functions(path: str = RUST) -> list[str]:
    return re.findall(r"pub fn (shd_\w+)\(", open(path).read())


def main():
    os.makedirs(os.path.dirname(RUST), exist_ok=True)
    os.makedirs(os.path.dirname(LAYOUT_C), exist_ok=True)
    open(RUST, "w").write(gen_rust())
    open(LAYOUT_C, "w").write(gen_layout_c(probe_layout()))
    print("wrote", RUST, LAYOUT_C)


if __name__ == "__main__":
    sys.exit(main())
