"""The Rust binding a maintainer adds to the reference crate (integration/rust/)
against include/marshrutka_pf.h.  There is no Rust toolchain in this image, so the
Rust files are not compiled; instead:

* every `#[repr(C)]` struct of integration/rust/src/ffi.rs has the header's fields in
  the header's order, and the repr(C) layout computed from its Rust field types has
  the size and field offsets a C compiler gives the header's struct (gcc compiles a
  probe over the header itself);
* the `extern "C"` block declares exactly the header's functions with the header's
  parameter counts, and every constant it defines has the header's value;
* engine.rs (the new body of FindPath::eval, src/pathfinder.rs:199-248) only calls
  functions and constants that ffi.rs declares.
"""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "marshrutka_pf.h")
FFI = os.path.join(ROOT, "integration", "rust", "src", "ffi.rs")
ENGINE = os.path.join(ROOT, "integration", "rust", "src", "engine.rs")

PRIM = {"u8": (1, 1), "i8": (1, 1), "u16": (2, 2), "i16": (2, 2), "u32": (4, 4), "i32": (4, 4),
        "u64": (8, 8), "i64": (8, 8), "f64": (8, 8)}


def _strip_rust_comments(src):
    return re.sub(r"//[^\n]*", "", src)


def rust_structs():
    src = _strip_rust_comments(open(FFI).read())
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive\([^)]*\)\]\s*)*pub struct (\w+)\s*\{(.*?)\}", src, re.S):
        fields = re.findall(r"pub (\w+):\s*([^,]+?)\s*,", m.group(2) + ",")
        out[m.group(1)] = fields
    return out


def rust_layout(structs, name):
    """(size, align, {field: offset}) of a repr(C) struct."""
    off, align, offs = 0, 1, {}
    for f, ty in structs[name]:
        s, a = rust_type(structs, ty)
        off = (off + a - 1) // a * a
        offs[f] = (off, s)
        off += s
        align = max(align, a)
    return (off + align - 1) // align * align, align, offs


def rust_type(structs, ty):
    ty = ty.strip()
    arr = re.fullmatch(r"\[(\w+);\s*(\d+)\]", ty)
    if arr:
        s, a = rust_type(structs, arr.group(1))
        return s * int(arr.group(2)), a
    if ty in PRIM:
        return PRIM[ty]
    s, a, _ = rust_layout(structs, ty)
    return s, a


def header_src():
    return re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)


def header_structs():
    out = {}
    for m in re.finditer(r"typedef struct (\w+)\s*\{(.*?)\}\s*\w+\s*;", header_src(), re.S):
        names = []
        for decl in m.group(2).split(";"):
            decl = decl.strip()
            if not decl:
                continue
            toks = re.sub(r"\[[^\]]*\]", "", decl).split(None, 1)[1]
            names += [t.strip().lstrip("*") for t in toks.split(",")]
        out[m.group(1)] = names
    return out


def header_functions():
    """name -> parameter count of every function the header declares."""
    out = {}
    for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(mr_\w+)\s*\(([^)]*)\)\s*;", header_src(), re.M | re.S):
        args = m.group(2).strip()
        out[m.group(1)] = 0 if args in ("", "void") else len(args.split(","))
    return out


def rust_functions():
    src = _strip_rust_comments(open(FFI).read())
    block = re.search(r'extern "C"\s*\{(.*)\}', src, re.S).group(1)
    out = {}
    for m in re.finditer(r"pub fn (\w+)\s*\((.*?)\)\s*(?:->\s*[^;]+)?;", block, re.S):
        args = m.group(2).strip().rstrip(",")
        out[m.group(1)] = 0 if not args else len([a for a in args.split(",") if a.strip()])
    return out


def rust_consts():
    src = _strip_rust_comments(open(FFI).read())
    return {n: int(v) for n, v in re.findall(r"pub const (MR_\w+):\s*\w+\s*=\s*(-?\d+)\s*;", src)}


@pytest.fixture(scope="module")
def c_probe():
    """sizeof/offsetof of the header's structs and the values of its constants,
    as gcc compiles the header."""
    structs = rust_structs()
    consts = rust_consts()
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for s, fields in structs.items():
        lines.append(f'printf("S {s} %zu\\n", sizeof({s}));')
        for f, _ in fields:
            lines.append(f'printf("F {s} {f} %zu %zu\\n", offsetof({s}, {f}), sizeof((({s} *)0)->{f}));')
    for n in consts:
        lines.append(f'printf("C {n} %lld\\n", (long long)({n}));')
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "probe.c"), os.path.join(d, "probe")
        open(c, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c11", "-Wall", "-o", exe, c], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    sizes, offs, vals = {}, {}, {}
    for line in out.splitlines():
        t = line.split()
        if t[0] == "S":
            sizes[t[1]] = int(t[2])
        elif t[0] == "F":
            offs[(t[1], t[2])] = (int(t[3]), int(t[4]))
        else:
            vals[t[1]] = int(t[2])
    return sizes, offs, vals


def test_rust_structs_match_header_field_order():
    rs, hs = rust_structs(), header_structs()
    assert set(rs) == set(hs), (sorted(rs), sorted(hs))
    for name, fields in rs.items():
        assert [f for f, _ in fields] == hs[name], name


def test_rust_struct_layouts_match_c(c_probe):
    sizes, offs, _ = c_probe
    rs = rust_structs()
    for name in rs:
        size, _, fo = rust_layout(rs, name)
        assert size == sizes[name], name
        for f, (o, s) in fo.items():
            assert (o, s) == offs[(name, f)], (name, f)


def test_rust_constants_match_header(c_probe):
    _, _, vals = c_probe
    consts = rust_consts()
    assert len(consts) >= 25
    for n, v in consts.items():
        assert vals[n] == v, n


def test_rust_extern_block_is_the_header():
    hf, rf = header_functions(), rust_functions()
    assert set(rf) == set(hf), (sorted(set(hf) - set(rf)), sorted(set(rf) - set(hf)))
    for n, k in hf.items():
        assert rf[n] == k, n


def test_engine_uses_only_declared_items():
    src = _strip_rust_comments(open(ENGINE).read())
    fns = set(re.findall(r"ffi::(mr_[a-z]\w*)\s*\(", src))
    consts = set(re.findall(r"ffi::(MR_\w+)", src))
    types = set(re.findall(r"ffi::(mr_[a-z_]+)\b(?!\s*\()", src)) - fns
    assert {"mr_find_path", "mr_grid_create", "mr_grid_destroy"} <= fns
    assert fns <= set(rust_functions())
    assert consts <= set(rust_consts())
    assert types <= set(rust_structs()) | {"mr_grid", "mr_plan"}
    # FindPath's every field reaches mr_params (src/pathfinder.rs:183-196)
    for f in ("scroll_of_escape_cost", "scroll_of_escape_hq_cost", "scroll_of_escape_forum_cost", "use_soe",
              "use_sfm", "use_caravans", "hq_position", "route_guru", "fleetfoot", "sort_by", "homeland"):
        assert re.search(rf"{f}:\s*[^,\n]*fp\.{f}", src), f
