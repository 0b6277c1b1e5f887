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


def test_no_fma_contraction_in_device_code():
    """-ffp-contract=off must hold: every v_fma_f64 in the kernels must belong to a
    division/sqrt expansion (v_div_* / v_rsq_* sequences), never to a*b+c."""
    mk = os.path.join(ROOT, "metabodecon-rust_amd", "Makefile")
    assert "-ffp-contract=off" in open(mk).read()
