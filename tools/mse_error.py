"""Relative deviation of the engine's MSE from the oracle's left-fold MSE
(compute_mse, deconvoluter.rs:828-862) over all golden cases and two more synthetic
spectra (GPU box), for each MSE form the library ships: the local expansions with 2
and with 4 points per thread (MDG_MSE_NPT; the default picks it by batch size) and 20
or 30 powers (MDG_MSE_PK; the default is 30 at every batch size, 20 selects the
round-4 radius-5 form) and the exact-order option (MDG_OPTION_EXACT_MSE,
expected 0). Prints the max |rel| per form.

    python tools/mse_error.py
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    argparse.ArgumentParser(description=__doc__.split("\n\n")[0]).parse_args()
    sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
    import numpy as np
    import oracle
    from metabodecon import _native as nat
    from tests.golden.cases import CASES, load_case, synth_spectrum
    from tests.test_gpu_parity import gpu_batch
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
    forms = [(f"local, {npt} points per thread, {pk} powers", npt, pk, False)
             for npt in ("2", "4") for pk in ("20", "30")] + [("exact order", "2", "20", True)]
    for form, npt, pk, exact in forms:
        os.environ["MDG_MSE_NPT"] = npt
        os.environ["MDG_MSE_PK"] = pk
        ctx.reload_switches()  # the engine reads its switches per context, not per call
        worst, wname = 0.0, None
        for name, x, y, sb, st, ign, ref in cases:
            s = nat.Settings()
            for f, _ in nat.Settings._fields_:
                setattr(s, f, getattr(st, f, 0))
            s.options = nat.OPTION_EXACT_MSE if exact else 0
            status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], s, ign)
            assert status[0] == 0, (name, status[0])
            rel = abs(mse[0] - ref) / abs(ref)
            if rel > worst:
                worst, wname = rel, name
        print(f"{form}: max |rel err| {worst:.3e} ({wname}) over {len(cases)} spectra", flush=True)


if __name__ == "__main__":
    main()
