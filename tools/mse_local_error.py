"""Accuracy of the local-expansion MSE (k_mse_local) restated in
numpy, against a long-double direct sum of the Lorentzians.

    python tools/mse_local_error.py [case ...]

For each golden case (oracle parameters from tests/golden/expected/*.npz) and
for the synthetic configs[1] spectrum it prints the largest relative error of
the superposition over the signal region and the relative error of the MSE,
for the kernel's tile shapes (512 and 1024 points, R = 3, 30 terms since round 5;
R = 5, 20 terms before) and neighbours.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd"), os.path.join(ROOT, "tests", "golden")]


def local_sup(xs, P, TP=256, R=5.0, p=20, rec=False):
    """The kernel's arithmetic per tile: near Lorentzians direct, far ones as the
    imaginary parts of -sum_k [sum_j a_j w_j (r w_j)^k] u^k. rec: the imaginary
    parts y_k = Im(c q^k) by the real second-order recurrence
    y_{k+2} = 2 Re(q) y_{k+1} - |q|^2 y_k (the roots q, conj(q) have one modulus,
    so an error decays like the terms themselves)."""
    f, h, m = P[:, 0], P[:, 1], P[:, 2]
    sig = np.sqrt(h)
    a = f / sig
    out = np.zeros(xs.size)
    for t0 in range(0, xs.size, TP):
        xt = xs[t0:t0 + TP]
        lo, hi = xt.min(), xt.max()
        t, r = 0.5 * lo + 0.5 * hi, 0.5 * hi - 0.5 * lo
        dz = (m - t) + 1j * sig
        far = np.abs(dz) > R * r
        w = 1.0 / dz[far]
        c, q = a[far] * w, r * w
        L = np.zeros(p)
        if rec:
            y0 = c.imag
            y1 = c.real * q.imag + c.imag * q.real
            a2, b = 2.0 * q.real, q.real * q.real + q.imag * q.imag
            L[0], L[1] = -np.sum(y0), -np.sum(y1)
            for k in range(2, p):
                y0, y1 = y1, a2 * y1 - b * y0
                L[k] = -np.sum(y1)
        else:
            for k in range(p):
                L[k] = -np.sum(c.imag)
                c = c * q
        u = (xt - t) / r if r > 0 else np.zeros_like(xt)
        S = np.zeros(xt.size)
        for k in range(p - 1, -1, -1):
            S = S * u + L[k]
        for j in np.nonzero(~far)[0]:
            d = xt - m[j]
            S += f[j] / (h[j] + d * d)
        out[t0:t0 + TP] = S
    return out


def direct(xv, P, dtype):
    xv = xv.astype(dtype)
    acc = np.zeros(xv.size, dtype=dtype)
    for j in range(P.shape[0]):
        d = xv - dtype(P[j, 2])
        acc += dtype(P[j, 0]) / (dtype(P[j, 1]) + d * d)
    return acc


def report(name, xs, ys, P, shapes):
    ref = direct(xs, P, np.longdouble)
    mref = float(np.mean((ref - ys) ** 2))
    d64 = direct(xs, P, np.float64)
    print(f"{name}: P={P.shape[0]} L={xs.size}  direct f64: MSE rel {float(np.mean((d64 - ys) ** 2)) / mref - 1:+.2e}")
    for TP, R, p, *rest in shapes:
        rec = bool(rest and rest[0])
        s = local_sup(xs, P, TP, R, p, rec)
        e = float(np.max(np.abs((s - ref) / ref)))
        print(f"   tile {TP} R={R} terms {p}{' rec' if rec else ''}: sup rel {e:.2e}  "
              f"MSE rel {float(np.mean((s - ys) ** 2)) / mref - 1:+.2e}")


def main():
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("cases", nargs="*", help="golden case names (default: five)")
    names_arg = ap.parse_args().cases
    from cases import load_case, synth_spectrum
    import oracle
    shapes = [(256, 5.0, 20), (256, 5.0, 20, True), (512, 5.0, 20), (512, 5.0, 20, True),
              (512, 4.0, 24, True), (512, 3.0, 30, True), (1024, 3.0, 30, True)]
    names = names_arg or ["blood_01", "blood_05", "blood_09", "sim_01", "synth"]
    for nm in names:
        if nm == "synth":
            x, y, _ = synth_spectrum(0)
            o = oracle.deconvolute(x, y, (11.8, -2.2), threads=8)
            P, (lo, hi) = o.params, o.sbi
        else:
            x, y, *_ = load_case(nm)
            g = np.load(os.path.join(ROOT, "tests", "golden", "expected", f"{nm}.npz"))
            P, (lo, hi) = g["params"], (int(v) for v in g["sbi"])
        x, y = np.asarray(x), np.asarray(y)
        report(nm, x[lo:hi], y[lo:hi], P, shapes)


if __name__ == "__main__":
    main()
