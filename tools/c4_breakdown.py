"""configs[4] host-side breakdown (GPU box): the 16 blood spectra through
Deconvoluter.par_deconvolute_spectra, and the parts of one batched call timed
separately (numpy stacking, the engine call with its copies, the results), then the
per-stage kernel times of one call at B = 1, 8 and 16.

    python tools/c4_breakdown.py [--reps R]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def med(f, k=10):
    import numpy as np
    f()
    ts = []
    for _ in range(k):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return 1e3 * float(np.median(ts))


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--torch-first", action="store_true", help="initialise torch's HIP runtime first")
    args = ap.parse_args()
    sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
    import numpy as np
    if args.torch_first:
        import torch
        torch.cuda.init()
    import metabodecon as md
    from metabodecon import _native as nat
    S = md.Spectrum.read_bruker_set(os.path.join(ROOT, "tests/golden/bruker/blood"), 10, 10, (-2.2, 11.8))
    dec = md.Deconvoluter()
    ctx = nat.context(nat.default_device())
    ign = dec._ignore_array()
    n = len(S[0])
    for rep in range(args.reps):
        print(f"rep {rep}: lanes {dec.LANES} par_deconvolute_spectra 16: "
              f"{med(lambda: dec.par_deconvolute_spectra(S)):.3f} ms")
        for b in (1, 8, 16):
            sub = S[:b]
            print(f"  B={b} stack x+y: %.3f ms" % med(lambda: (np.stack([s.chemical_shifts for s in sub]),
                                                             np.stack([s.intensities for s in sub]))))
            print(f"  B={b} _run_batch (one context): %.3f ms"
                  % med(lambda: dec._run_batch(ctx, sub, list(range(b)), n, ign)))
            print(f"  B={b} deconvolute_spectra: %.3f ms" % med(lambda: dec.deconvolute_spectra(sub)))
    for b in (1, 8, 16):
        sub = S[:b]
        ctx.reset_stage_times()
        ctx.set_profiling(True)
        for _ in range(3):
            dec._run_batch(ctx, sub, list(range(b)), n, ign)
        st = ctx.stage_times()
        ctx.set_profiling(False)
        print(f"B={b} stages ms per call:", {k: round(v[0] / 3, 3) for k, v in st.items() if v[1]})
        print("   kernels:", ctx.stage_kernels())


if __name__ == "__main__":
    main()
