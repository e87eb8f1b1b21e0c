"""INTEGRATION.md's Rust `extern "C"` blocks, checked against include/odesat.h by the C compiler
(VERDICT r5 "the Rust host side is unverifiable": rustc is not in this image).

Every `pub fn` of the document's ```rust blocks becomes a C function-pointer type built from its Rust
signature (i64 -> int64_t, *const T -> const T *, ...), initialised with the header's function of that
name: gcc -Werror rejects any parameter, pointee qualifier or return type that differs.  Every
`pub const` must equal the header's macro, and every `#[repr(C)]` struct with fields must have the
size and the field offsets of the header's struct (OdesatParams -> odesat_params)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC = os.path.join(ROOT, "INTEGRATION.md")
HEADER = os.path.join(ROOT, "include", "odesat.h")

SCALARS = {"c_int": "int", "c_char": "char", "usize": "size_t", "i64": "int64_t", "i32": "int32_t",
           "u64": "uint64_t", "u8": "uint8_t", "f32": "float", "f64": "double", "std::ffi::c_void": "void"}
OPAQUE = {"OdesatCnf": "odesat_cnf", "OdesatSolver": "odesat_solver", "OdesatStoch": "odesat_stoch",
          "OdesatTrace": "odesat_trace", "OdesatPart": "odesat_part", "OdesatCtx": "odesat_ctx",
          "OdesatParams": "odesat_params"}


def rust_blocks():
    text = open(DOC).read()
    return re.findall(r"```rust\n(.*?)```", text, re.S)


def c_type(t):
    t = re.sub(r"/\*.*?\*/", "", t).strip()
    if t.startswith("*const "):
        inner = c_type(t[len("*const "):])
        return f"const {inner} *" if not inner.endswith("*") else f"{inner} const *"
    if t.startswith("*mut "):
        return f"{c_type(t[len('*mut '):])} *"
    if t in SCALARS:
        return SCALARS[t]
    if t in OPAQUE:
        return OPAQUE[t]
    raise ValueError(f"unmapped Rust type {t!r}")


def functions(code):
    out = []
    for block in re.findall(r'extern "C" \{(.*?)\n\}', code, re.S):
        body = re.sub(r"//[^\n]*", "", block)
        for name, params, ret in re.findall(r"pub fn (\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", body, re.S):
            args = []
            for p in (x.strip() for x in params.replace("\n", " ").split(",")):
                if p:
                    args.append(c_type(p.split(":", 1)[1]))
            out.append((name, args, c_type(ret) if ret else "void"))
    return out


def structs(code):
    return re.findall(r"#\[repr\(C\)\]\s*pub struct (\w+)\s*\{([^}]*)\}", code, re.S)


def consts(code):
    return re.findall(r"pub const (\w+):\s*\w+\s*=\s*(-?\d+);", code)


def test_rust_blocks_match_the_header(tmp_path):
    code = "\n".join(rust_blocks())
    fns = functions(code)
    assert len(fns) >= 34, len(fns)
    lines = ['#include <stddef.h>', '#include <stdint.h>', f'#include "{HEADER}"']
    for name, args, ret in fns:
        lines.append(f"typedef {ret} (*rs_{name}_t)({', '.join(args) or 'void'});")
        lines.append(f"rs_{name}_t rs_{name} = &{name};")
    for name, value in consts(code):
        lines.append(f'_Static_assert({name} == {value}, "{name}");')
    nfields = 0
    for name, body in structs(code):
        fields = [f.strip() for f in body.replace("\n", " ").split(",") if f.strip() and "_p:" not in f]
        if not fields:
            continue  # opaque handle
        members = []
        for f in fields:
            fname, ftype = (x.strip() for x in f.replace("pub ", "").split(":", 1))
            members.append((fname, c_type(ftype)))
        cname = OPAQUE[name]
        lines.append(f"struct rs_{name} {{ {' '.join(f'{t} {n};' for n, t in members)} }};")
        lines.append(f'_Static_assert(sizeof(struct rs_{name}) == sizeof({cname}), "{name} size");')
        for fname, _ in members:
            lines.append(f'_Static_assert(offsetof(struct rs_{name}, {fname}) == offsetof({cname}, {fname}), '
                         f'"{name}.{fname}");')
            nfields += 1
    assert nfields == 8  # OdesatParams
    src = tmp_path / "rust_block_check.c"
    src.write_text("\n".join(lines) + "\n")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-c", str(src), "-o", str(tmp_path / "x.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr + "\n" + src.read_text()


def test_the_checker_catches_a_mismatch(tmp_path):
    """The same machinery rejects a signature that differs from the header (one pointee qualifier)."""
    bad = 'extern "C" {\n    pub fn odesat_cnf_free(cnf: *const OdesatCnf);\n}'
    (name, args, ret), = functions(bad)
    src = tmp_path / "bad.c"
    src.write_text(f'#include "{HEADER}"\ntypedef {ret} (*t)({", ".join(args)});\nt x = &{name};\n')
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-c", str(src), "-o", str(tmp_path / "x.o")],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "incompatible" in r.stderr


@pytest.mark.parametrize("t,c", [("*mut *mut OdesatCnf", "odesat_cnf * *"), ("*const i64", "const int64_t *"),
                                 ("usize", "size_t"), ("*mut std::ffi::c_void", "void *")])
def test_type_mapping(t, c):
    assert c_type(t) == c
