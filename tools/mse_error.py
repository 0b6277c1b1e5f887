"""Relative MSE deviation of every MSE kernel from the oracle's left-fold MSE
(compute_mse, deconvoluter.rs:828-862) over all golden cases and a few synthetic
spectra: python tools/mse_error.py  (GPU). Prints the max |rel| per kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]

import numpy as np  # noqa: E402

import oracle  # noqa: E402
from tests.golden.cases import CASES, load_case, synth_spectrum  # noqa: E402
from tests.test_gpu_parity import gpu_batch  # noqa: E402
from metabodecon import _native as nat  # noqa: E402


def main():
    ctx = nat.context(0)
    cases = []
    for name in CASES:
        x, y, sb, st, ign = load_case(name)
        g = np.load(os.path.join(ROOT, "tests", "golden", "expected", f"{name}.npz"))
        if int(g["status"]) == 0:
            cases.append((name, x, y, sb, st, ign, float(g["mse"])))
    for seed in (2, 3):
        x, y, _ = synth_spectrum(seed)
        o = oracle.deconvolute(x, y, (11.8, -2.2), threads=16)
        cases.append((f"synth_{seed}", x, y, (11.8, -2.2), oracle.default_settings(), (), o.mse))
    for kind in ("local", "local1", "quad", "n", "plain"):
        os.environ["MDG_MSE"] = "local" if kind.startswith("local") else kind
        os.environ["MDG_MSE_NPT"] = "1" if kind == "local1" else "2"
        worst, wname = 0.0, None
        for name, x, y, sb, st, ign, ref in cases:
            status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st, ign)
            assert status[0] == 0, (name, status[0])
            rel = abs(mse[0] - ref) / abs(ref)
            if rel > worst:
                worst, wname = rel, name
        print(f"MDG_MSE={kind}: max |rel err| {worst:.3e} ({wname}) over {len(cases)} spectra",
              flush=True)


if __name__ == "__main__":
    main()
