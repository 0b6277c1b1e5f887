"""Wall time of Deconvoluter.optimize_settings (810 settings) on blood_01."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "metabodecon-rust_amd")]
import metabodecon as md  # noqa: E402

spec = md.Spectrum.read_bruker(os.path.join(ROOT, "tests", "golden", "bruker", "blood", "blood_01"),
                               10, 10, (-2.2, 11.8))
d = md.Deconvoluter()
d.optimize_settings(spec)  # warm-up (allocations, module load)
t = time.perf_counter()
mse = d.optimize_settings(spec)
dt = time.perf_counter() - t
s = d.settings
print(f"optimize_settings blood_01: {dt:.3f} s, mse {mse!r}, MA({s.smooth_iterations},"
      f"{s.smooth_window}) thr {s.threshold!r} fit {s.fit_iterations}")
