"""Find the scale factors of tests/test_gpu_range_paths.py.

The fit and superposition_vec use div_rn (the IEEE division without its
div_scale/div_fixup wrappers) only when per-spectrum flags prove the operand ranges:
|sfhw|, hw2 in [2^-200, 2^200], |maxp| <= 2^100 for every parameter of the version an
iteration reads, and |x| <= 2^100. A spectrum's sfhw scale with its
intensities, so multiplying a spectrum by c moves log2 max|sfhw| of every parameter
version by log2 c. This tool traces max/min log2|sfhw| per version (the oracle's
mirror/solve/superposition, test infrastructure) and prints, for a threshold T between
two versions' values, c = 2^(200 - T) or 2^(-200 - T): a spectrum whose fast flag flips
at chosen iterations. The oracle's range_mask on the scaled spectrum is the check; the
test pins it.

    python tools/range_cases.py blood_01 sim_03
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]

import oracle  # noqa: E402  (test infrastructure)
from tests.golden.cases import load_case  # noqa: E402


def version_trace(x, y, sb, iters=10):
    """log2 of (max |sfhw|, min |sfhw|, max |maxp|) for parameter versions 0..iters."""
    st = oracle.default_settings()
    r = oracle.deconvolute(x, y, sb, st)
    assert r.status == 0
    sel = r.selected
    P = sel.shape[0]
    rx, ry = x[sel].reshape(-1), y[sel].reshape(-1)
    st6 = np.empty((P, 6))
    st6[:, :3], st6[:, 3:] = x[sel], y[sel]
    L = oracle.lib()
    params = np.empty((P, 3))

    def mirror_solve():
        for p in range(P):
            row = np.ascontiguousarray(st6[p])
            L.mdo_mirror_shoulder(oracle._ptr(row))
            st6[p] = row
            v = [oracle.ctypes.c_double() for _ in range(3)]
            L.mdo_solve_stencil(oracle._ptr(row), *[oracle.ctypes.byref(t) for t in v])
            params[p] = [t.value for t in v]

    out = []
    mirror_solve()
    for it in range(iters + 1):
        a = np.abs(params[:, 0])
        out.append((np.log2(a.max()), np.log2(a.min()), np.log2(np.abs(params[:, 2]).max())))
        if it == iters:
            break
        sup = oracle.superposition_vec(rx, params.copy())
        st6[:, 3:] *= (ry / sup).reshape(P, 3)
        mirror_solve()
    return np.array(out)


def main(names):
    for name in names:
        x, y, sb, _, _ = load_case(name)
        t = version_trace(x, y, sb)
        print(name)
        for v, row in enumerate(t):
            print(f"  version {v:2d}: log2 max|sfhw| {row[0]:.6f}  min {row[1]:.6f}  max|maxp| {row[2]:.6f}")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("names", nargs="*", default=["blood_01", "sim_03"], help="golden case names")
    main(ap.parse_args().names)
