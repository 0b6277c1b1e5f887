"""configs[4] experiment: the 16 blood spectra through
Deconvoluter.par_deconvolute_spectra with L lanes (engine contexts running
concurrently, one spectrum each at L = 16) against one batched call of 16, host
buffers in and out; results compared bit for bit between the settings.

    GPU box: python tools/c4_lanes.py [--lanes 16 1 ...]   (prints one line per setting)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--lanes", type=int, nargs="+", default=[16, 1, 16, 1])
    args = ap.parse_args()
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "32")
    sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
    import numpy as np
    import metabodecon as md
    spectra = md.Spectrum.read_bruker_set(os.path.join(ROOT, "tests", "golden", "bruker", "blood"),
                                          10, 10, (-2.2, 11.8))
    ref = None
    for lanes in args.lanes:
        md.Deconvoluter.LANES = lanes
        # one batch below ONE_LANE_UPTO spectra unless lanes are asked for
        md.Deconvoluter.ONE_LANE_UPTO = 16 if lanes == 1 else 0
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
