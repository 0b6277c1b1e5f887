"""The Rust shim (rust/metabodecon-gpu/src/lib.rs) against the C ABI, without Rust.

There is no cargo/rustc in this image, so the crate cannot be compiled here.
This test pins the part a compiler would check at the boundary: every
`extern "C"` declaration of the shim's `ffi` module is translated mechanically
(Rust type -> C type) into a C prototype and compiled with gcc AFTER
`#include "mdgpu.h"` -- a redeclaration whose types differ from the header's is
a hard error in C -- together with shadow copies of the shim's `repr(C)` structs
whose size and field offsets are asserted equal to the header's, and the shim's
status/enum constants asserted equal to the header's. The resulting program is
linked against libmdgpu.so and calls the host-only entry points through those
prototypes. A mutated declaration must fail to compile (the check has power).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_RS = os.path.join(ROOT, "rust", "metabodecon-gpu", "src", "lib.rs")
INCLUDE = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "metabodecon-rust_amd", "metabodecon")

RUST_TO_C = {
    "c_int": "int", "i32": "int32_t", "u32": "uint32_t", "u64": "uint64_t", "i64": "int64_t",
    "usize": "size_t", "f64": "double", "c_void": "void", "c_char": "char",
    "MdgSettings": "mdg_settings", "MdgLorentzian": "mdg_lorentzian", "MdgCtx": "mdg_ctx",
    "MdgQueue": "mdg_queue",
}


def c_type(rt: str) -> str:
    rt = rt.strip()
    if rt.startswith("*const "):
        inner = c_type(rt[len("*const "):])
        # *const *const f64 -> const double* const*
        return inner + " const*" if inner.endswith("*") else "const " + inner + "*"
    if rt.startswith("*mut "):
        inner = c_type(rt[len("*mut "):])
        return inner + "*"
    return RUST_TO_C[rt]


def parse_externs(src: str):
    block = src[src.index('extern "C" {'):]
    block = block[: block.index("\n    }\n")]
    out = []
    for m in re.finditer(r"pub fn (\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", block, re.S):
        name, args, ret = m.group(1), m.group(2), m.group(3)
        params = []
        for a in [a.strip() for a in args.split(",") if a.strip()]:
            an, at = a.split(":", 1)
            params.append((an.strip(), at.strip()))
        out.append((name, params, (ret or "").strip()))
    return out


def parse_structs(src: str):
    structs = {}
    for m in re.finditer(r"#\[repr\(C\)\]\s*(?:#\[derive[^\]]*\]\s*)?pub struct (\w+) \{(.*?)\}",
                         src, re.S):
        fields = re.findall(r"pub (\w+): (\w+),", m.group(2))
        if fields:
            structs[m.group(1)] = fields
    return structs


def parse_consts(src: str):
    return re.findall(r"pub const (MDG_\w+): \w+ = (-?\d+);", src)


def c_program(externs, structs, consts):
    lines = ["#include <stddef.h>", "#include <stdint.h>", "#include <stdio.h>",
             "#include <string.h>", '#include "mdgpu.h"', ""]
    for name, params, ret in externs:
        cret = c_type(ret) if ret else "void"
        cparams = ", ".join(f"{c_type(t)} {n}" for n, t in params) or "void"
        lines.append(f"{cret} {name}({cparams});")
    lines.append("")
    for sname, fields in structs.items():
        cname = RUST_TO_C[sname]
        lines.append(f"struct shadow_{sname} {{")
        lines += [f"    {RUST_TO_C[t]} {f};" for f, t in fields]
        lines.append("};")
        lines.append(f"_Static_assert(sizeof(struct shadow_{sname}) == sizeof({cname}), "
                     f"\"size of {sname}\");")
        for f, _ in fields:
            lines.append(f"_Static_assert(offsetof(struct shadow_{sname}, {f}) == "
                         f"offsetof({cname}, {f}), \"offset of {sname}.{f}\");")
    for cname, val in consts:
        lines.append(f"_Static_assert({cname} == {val}, \"{cname}\");")
    lines += [
        "",
        "int main(void) {",
        "    if (mdg_abi_version() != MDG_ABI_VERSION) return 1;",
        "    mdg_settings s;",
        "    memset(&s, 0xff, sizeof(s));",
        "    mdg_settings_default(&s);",
        "    if (mdg_settings_validate(&s) != MDG_OK) return 2;",
        "    if (s.smooth_iterations != 3 || s.smooth_window != 3 || s.fit_iterations != 10 ||",
        "        s.threshold != 5.0) return 3;",
        "    s.fit_iterations = 0;",
        "    if (mdg_settings_validate(&s) != MDG_INVALID_FITTING) return 4;",
        "    double r[8] = {0};",
        "    size_t n = 0;",
        "    if (mdg_ignore_region_add(r, 0, 4, 4.8, 4.6, &n) || n != 1) return 5;",
        "    if (mdg_ignore_region_add(r, n, 4, 4.7, 5.0, &n) || n != 1) return 6;",
        "    if (r[0] != 4.6 || r[1] != 5.0) return 7;",
        "    if (mdg_ignore_region_add(r, n, 4, 1.0, 1.0, &n) != MDG_INVALID_IGNORE_REGION) return 8;",
        "    if (!mdg_strerror(MDG_NO_PEAKS_DETECTED)) return 9;",
        '    printf("shim abi ok: %d functions\\n", ' + str(len(externs)) + ");",
        "    return 0;",
        "}",
    ]
    return "\n".join(lines) + "\n"


def _compile(tmp_path, src, link=True):
    c = tmp_path / "shim_abi.c"
    c.write_text(src)
    exe = tmp_path / "shim_abi"
    cmd = ["gcc", "-std=c11", "-Wall", "-Werror", "-I", INCLUDE, str(c), "-o", str(exe)]
    if link:
        cmd += ["-L", LIBDIR, "-lmdgpu", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib"]
    else:
        cmd = cmd[:-2] + ["-c", "-o", str(tmp_path / "shim_abi.o")]
    return subprocess.run(cmd, capture_output=True, text=True), exe


@pytest.fixture(scope="module")
def shim():
    src = open(LIB_RS).read()
    return parse_externs(src), parse_structs(src), parse_consts(src)


def test_shim_declares_the_hot_path(shim):
    externs, structs, _ = shim
    names = {e[0] for e in externs}
    assert {"mdg_deconvolute", "mdg_deconvolute_batch", "mdg_deconvolute_rows",
            "mdg_deconvolute_batch_device", "mdg_superposition_vec", "mdg_optimize_settings", "mdg_ctx_create",
            "mdg_ctx_destroy"} <= names
    assert set(structs) == {"MdgSettings", "MdgLorentzian"}
    header = open(os.path.join(INCLUDE, "mdgpu.h")).read()
    for n in names:
        assert re.search(rf"\b{n}\(", header), n


def test_shim_signatures_compile_against_header_and_run(shim, tmp_path):
    externs, structs, consts = shim
    if not os.path.exists(os.path.join(LIBDIR, "libmdgpu.so")):
        pytest.skip("libmdgpu.so not built")
    res, exe = _compile(tmp_path, c_program(externs, structs, consts))
    assert res.returncode == 0, res.stderr
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", ""))
    run = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60, env=env)
    assert run.returncode == 0, (run.returncode, run.stdout, run.stderr)
    assert "shim abi ok" in run.stdout


@pytest.mark.parametrize("mutation", [
    ("mdg_deconvolute", "cap", "u32"),            # usize -> u32
    ("mdg_deconvolute_batch", "status", "*mut u64"),
    ("mdg_deconvolute_rows", "x_rows", "*const f64"),  # one row, not row pointers
    ("mdg_superposition_vec", "out", "*mut i32"),
])
def test_mutated_signature_fails_to_compile(shim, tmp_path, mutation):
    externs, structs, consts = shim
    fn, arg, new_type = mutation
    mutated = [(n, [(a, new_type if (n == fn and a == arg) else t) for a, t in p], r)
               for n, p, r in externs]
    assert mutated != externs
    res, _ = _compile(tmp_path, c_program(mutated, structs, consts), link=False)
    assert res.returncode != 0 and "conflicting types" in res.stderr, res.stderr


def test_mutated_struct_layout_fails_to_compile(shim, tmp_path):
    externs, structs, consts = shim
    bad = dict(structs)
    bad["MdgSettings"] = [(f, "f64" if f == "options" else t) for f, t in structs["MdgSettings"]]
    res, _ = _compile(tmp_path, c_program(externs, bad, consts), link=False)
    assert res.returncode != 0
