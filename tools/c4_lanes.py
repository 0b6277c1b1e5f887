"""configs[4] experiment: the 16 blood spectra through
Deconvoluter.par_deconvolute_spectra with L lanes (one spectrum per engine context,
concurrently) against one batched call (L = 1 -> B = 16), host buffers in and out.

    GPU box: python tools/c4_lanes.py   (prints one line per setting)
"""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "32")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]

import numpy as np  # noqa: E402

import metabodecon as md  # noqa: E402


def main():
    spectra = md.Spectrum.read_bruker_set(os.path.join(ROOT, "tests", "golden", "bruker", "blood"),
                                          10, 10, (-2.2, 11.8))
    ref = None
    for lanes in (16, 1, 16, 1):  # 16 lanes, or (any L < 16) one batched call of 16
        md.Deconvoluter.LANES = lanes
        dec = md.Deconvoluter()
        for _ in range(2):
            res = dec.par_deconvolute_spectra(spectra)
        ts = []
        for _ in range(10):
            t = time.perf_counter()
            res = dec.par_deconvolute_spectra(spectra)
            ts.append(time.perf_counter() - t)
        params = [d.params for d in res]
        if ref is None:
            ref = params
        same = all(np.array_equal(a, b) for a, b in zip(ref, params))
        med = float(np.median(ts))
        print(f"lanes={lanes:2d}: {len(spectra) / med:7.0f} spectra/s, median {med * 1e3:.2f} ms "
              f"per set (min {min(ts) * 1e3:.2f}), identical={same}", flush=True)


if __name__ == "__main__":
    main()
