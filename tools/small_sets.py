"""Small same-length sets through Deconvoluter.par_deconvolute_spectra: one batch
(ONE_LANE_UPTO) against two lanes, for k = 2, 4, 8, 16 blood spectra (GPU box; default
4 hardware queues). Median ms per set over 20 calls, alternating the settings.

    python tools/small_sets.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]

import numpy as np  # noqa: E402

import metabodecon as md  # noqa: E402


def main():
    import argparse
    argparse.ArgumentParser(description=__doc__.split("\n\n")[0]).parse_args()
    spectra = md.Spectrum.read_bruker_set(os.path.join(ROOT, "tests", "golden", "bruker", "blood"),
                                          10, 10, (-2.2, 11.8))
    D = md.Deconvoluter
    D.LANES = 2
    for k in (2, 4, 8, 16):
        sub = spectra[:k]
        res = {}
        for rnd in range(2):
            for name, upto in (("one batch", 16), ("two lanes", 0)):
                D.ONE_LANE_UPTO = upto
                dec = D()
                for _ in range(3):
                    dec.par_deconvolute_spectra(sub)
                ts = []
                for _ in range(20):
                    t = time.perf_counter()
                    dec.par_deconvolute_spectra(sub)
                    ts.append(time.perf_counter() - t)
                res.setdefault(name, []).append(1e3 * float(np.median(ts)))
        print(f"k={k:2d}: " + ", ".join(f"{n} {min(v):.3f}-{max(v):.3f} ms ({k / (1e-3 * min(v)):.0f}/s)"
                                         for n, v in res.items()), flush=True)


if __name__ == "__main__":
    main()
