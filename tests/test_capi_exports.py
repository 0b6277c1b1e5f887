"""The C-ABI library loads on a CPU-only host and exports every symbol that
include/mdgpu.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re
import subprocess

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "mdgpu.h")
LIB = os.path.join(ROOT, "metabodecon-rust_amd", "metabodecon", "libmdgpu.so")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mdg_[a-z0-9_]+)\s*\(", text)))


def test_library_builds_and_loads():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "metabodecon-rust_amd")], check=True)
    ctypes.CDLL(LIB)


def test_every_declared_symbol_is_exported():
    syms = declared_symbols()
    assert len(syms) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (mdg_\w+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(LIB)
    for s in syms:
        getattr(lib, s)


def test_python_binding_covers_header():
    from metabodecon import _native
    assert sorted(_native.EXPORTS) == declared_symbols()


def test_abi_version_and_strerror():
    from metabodecon import _native
    L = _native.lib()
    assert L.mdg_abi_version() == 1
    assert _native.strerror(1) == "no peaks detected in the spectrum"
    assert _native.strerror(2) == "no peaks found in the signal region of the spectrum"
    assert _native.strerror(3) == "no peaks found in the signal-free region of the spectrum"


def test_library_built_from_the_tree_sources():
    """Build provenance: the hash compiled into libmdgpu.so (Makefile SRC_HASH) equals
    the sha256 of the engine sources in this tree, so the library the GPU tests load
    is the one these sources make."""
    from metabodecon import _native
    info = _native.build_info()
    assert info["tree"] is not None and len(info["src"]) == 16
    assert info["src"] == info["tree"], info
    assert info["flags"] == info["default_flags"] and len(info["flags"]) == 16, info
    mk = open(os.path.join(ROOT, "metabodecon-rust_amd", "Makefile")).read()
    m = re.search(r"^SRC = (.*)\nHDR = (.*)$", mk, re.M)
    assert (m.group(1).split() + m.group(2).split()) == _native.SOURCE_FILES


def test_stale_library_is_refused(monkeypatch):
    from metabodecon import _native
    L = _native.lib()
    monkeypatch.delenv("MDGPU_ALLOW_STALE", raising=False)
    monkeypatch.setattr(_native, "source_hash", lambda: "0" * 16)
    try:
        _native._check_provenance(L)
    except _native.NativeLibraryError as e:
        assert "rebuild" in str(e)
    else:
        raise AssertionError("stale library accepted")


def test_other_compile_flags_only_warn(monkeypatch):
    """Same sources built with other flags (make ARCH=..., an A/B -D override) load
    with a warning; only a source mismatch is refused."""
    import warnings
    from metabodecon import _native
    L = _native.lib()
    monkeypatch.delenv("MDGPU_ALLOW_STALE", raising=False)
    monkeypatch.setattr(_native, "flags_hash", lambda: "f" * 16)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        _native._check_provenance(L)
    assert any("non-default compile flags" in str(x.message) for x in w)


def _hipflags():
    mk = open(os.path.join(ROOT, "metabodecon-rust_amd", "Makefile")).read()
    m = re.search(r"^HIPFLAGS \?= (.*?)(?<!\\)\n", mk.replace("\\\n", " "), re.M | re.S)
    return m.group(1).replace("$(ARCH)", "gfx950").split()


def _device_outputs(flags, tmp, tag):
    """Device IR (after -O3) and device ISA of mdg_kernels.hip with `flags`, two
    hipcc processes in parallel."""
    src = os.path.join(ROOT, "metabodecon-rust_amd", "csrc", "mdg_kernels.hip")
    ll, s = os.path.join(tmp, f"{tag}.ll"), os.path.join(tmp, f"{tag}.s")
    hipcc = "/opt/rocm/bin/hipcc"
    procs = [subprocess.Popen([hipcc] + flags + ["--offload-device-only", "-emit-llvm", "-S", src,
                                                  "-o", ll], stderr=subprocess.DEVNULL),
             subprocess.Popen([hipcc] + flags + ["--offload-device-only", "-S", src, "-o", s],
                              stderr=subprocess.DEVNULL)]
    for p in procs:
        assert p.wait(timeout=600) == 0
    return open(ll).read(), open(s).read()


def _fma_budget(ir):
    """Per function: the f64 FMAs the source asks for -- explicit __builtin_fma
    (llvm.fma), FMAs written in inline asm (the DPP / +-1.0 folds), and the
    expansions of IEEE division (6 per fdiv: div_scale..div_fixup has 5, plus
    slack) and sqrt (4)."""
    out = {}
    for m in re.finditer(r"^define [^@]*@([\w.$]+)\((.*?)^\}", ir, re.S | re.M):
        body = m.group(0)
        explicit = (len(re.findall(r"call [^@\n]*double @llvm\.fma\.f64", body)) +
                    2 * len(re.findall(r"@llvm\.fma\.v2f64", body)))
        asm = sum(len(re.findall(r"v_fmac?_f64", a))
                  for a in re.findall(r'asm sideeffect "([^"]*)"', body))
        div = len(re.findall(r"= fdiv [a-z ]*double", body))
        sq = len(re.findall(r"@llvm\.sqrt\.f64", body))
        out[m.group(1)] = explicit + asm + 6 * div + 4 * sq
    return out


def _isa_fmas(isa):
    funcs = set(re.findall(r"\.type\s+([\w.$]+),@function", isa))
    out, cur = {}, None
    for line in isa.splitlines():
        m = re.match(r"^([\w.$]+):", line)
        if m and m.group(1) in funcs:
            cur = m.group(1)
            out.setdefault(cur, 0)
        elif cur and re.match(r"^\s+v_fmac?_f64", line):
            out[cur] += 1
    return out


def _contraction_report(ir, isa):
    contract = len(re.findall(r"= (?:fadd|fsub|fmul)[a-z ]* contract", ir))
    fmuladd = len(re.findall(r"@llvm\.fmuladd", ir))
    budget, fmas = _fma_budget(ir), _isa_fmas(isa)
    over = {f: (n, budget.get(f, 0)) for f, n in fmas.items() if n > budget.get(f, 0)}
    return contract, fmuladd, over, sum(fmas.values())


def test_no_fma_contraction_in_device_code(tmp_path):
    """rustc never fuses a*b+c (SURVEY 7 hard part 1), so the kernels must not
    either. Built with the Makefile's own HIPFLAGS: the optimised device IR has no
    `contract` flag and no llvm.fmuladd (so the backend may not fuse anything),
    and in the gfx950 ISA every v_fma_f64 / v_fmac_f64 of a function is accounted
    for by that function's explicit __builtin_fma calls, its inline-asm folds and
    its division/sqrt expansions. Power: the same sources built without
    -ffp-contract=off fail both checks."""
    flags = _hipflags()
    assert "-ffp-contract=off" in flags
    ir, isa = _device_outputs(flags, str(tmp_path), "real")
    contract, fmuladd, over, total = _contraction_report(ir, isa)
    assert total > 1000  # the kernels do use FMAs (divisions, folds)
    assert contract == 0 and fmuladd == 0, (contract, fmuladd)
    assert not over, over
    loose = [f for f in flags if f != "-ffp-contract=off"]
    ir2, isa2 = _device_outputs(loose, str(tmp_path), "loose")
    contract2, fmuladd2, over2, _ = _contraction_report(ir2, isa2)
    assert contract2 + fmuladd2 > 100
    fused = {f: n for f, (n, b) in _contraction_report(ir, isa2)[2].items()}
    assert len(fused) >= 3, fused  # contracted ISA exceeds the real budget
