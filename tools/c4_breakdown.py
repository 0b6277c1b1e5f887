"""configs[4] host-side breakdown (GPU box): the 16 blood spectra through
Deconvoluter.par_deconvolute_spectra, and the parts of one lane's batched call
timed separately (numpy stacking, the engine call with its copies, result rows).

    python tools/c4_breakdown.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
import numpy as np  # noqa: E402

if os.environ.get("C4_TORCH"):
    import torch  # noqa: F401
    torch.cuda.init()

import metabodecon as md  # noqa: E402
from metabodecon import _native as nat  # noqa: E402


def med(f, k=10):
    f()
    ts = []
    for _ in range(k):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return 1e3 * float(np.median(ts))


S = md.Spectrum.read_bruker_set(os.path.join(ROOT, "tests/golden/bruker/blood"), 10, 10, (-2.2, 11.8))
dec = md.Deconvoluter()
ctx = nat.context(nat.default_device())
ign = dec._ignore_array()
n = len(S[0])
for rep in range(3):
    print(f"rep {rep}: lanes {dec.LANES} par_deconvolute_spectra 16: %.3f ms" % med(lambda: dec.par_deconvolute_spectra(S)))
    for b in (1, 8, 16):
        sub = S[:b]
        print(f"  B={b} stack x+y: %.3f ms" % med(lambda: (np.stack([s.chemical_shifts for s in sub]),
                                                         np.stack([s.intensities for s in sub]))))
        print(f"  B={b} _run_batch (one context): %.3f ms" % med(lambda: dec._run_batch(ctx, sub, list(range(b)), n, ign)))
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
