"""Named parity cases shared by the golden generator and the tests.

Each case returns (x, y, sb, settings, ignore) with sb already ordered as the
reference's Spectrum stores it (spectrum.rs:854-863).
"""
import functools
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BRUKER = os.path.join(HERE, "bruker")


def _spectrum(kind: str, idx: int, sb):
    from metabodecon import Spectrum
    s = Spectrum.read_bruker(os.path.join(BRUKER, kind, f"{kind}_{idx:02d}"), 10, 10, sb)
    return np.array(s.chemical_shifts), np.array(s.intensities), s.signal_boundaries


def synth_spectrum(seed: int, n: int = 131072, n_peaks: int = 2048, xmax: float = 14.8,
                   width: float = 20.0, lo: float = -1.8, hi: float = 11.4,
                   sigma: float = 1.0e3, hw_scale: float = 1.0, threads: int | None = None):
    """CPU twin of mdg_synth_batch_device (bit-identical): shared axis, in-order
    superposition of mdg_synth_lorentzians(seed) plus mdg_synth_noise(seed)."""
    import ctypes
    import oracle
    from metabodecon import _native as nat
    i = np.arange(n, dtype=np.float64)
    x = xmax - (i * width) / (float(n) - 1.0)
    params = np.empty((n_peaks, 3))
    nat.lib().mdg_synth_lorentzians_hw(seed, n_peaks, lo, hi, hw_scale, nat.ptr(params))
    noise = np.empty(n)
    nat.lib().mdg_synth_noise(seed, n, sigma, nat.ptr(noise))
    y = oracle.superposition_vec(x, params, threads=threads or host_threads()) + noise
    return x, y, params


def host_threads() -> int:
    """CPUs this process may use: affinity, capped by the cgroup v2 CPU quota (the
    GPU box shows 256 CPUs under a 16-CPU quota)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(p)))
    except (OSError, ValueError):
        pass
    return n


def _settings(**kw):
    import oracle
    return oracle.make_settings(**kw)


CASES = [f"sim_{i:02d}" for i in range(1, 17)] + [f"blood_{i:02d}" for i in range(1, 17)] + [
    "blood_01_water", "blood_02_two_regions_increasing", "sim_01_detector_only",
    "sim_01_identity", "sim_01_ma5x2_thr3", "synth_128k_2k_s0", "synth_128k_2k_s1",
] + [f"sim_{i:02d}_harness" for i in range(1, 17)]
# "_harness": the sim spectra with the signal boundaries of the reference's own
# benchmark harness, (3.34, 3.56) (benches/deconvoluter.rs:17-19, 40-44; the
# integration test, tests/deconvoluter.rs, uses (3.35, 3.55) as the plain sim cases)


@functools.lru_cache(maxsize=None)
def _load(name: str):
    ign = ()
    st = _settings()
    if name.startswith("sim_") and len(name) == 6:
        x, y, sb = _spectrum("sim", int(name[4:]), (3.35, 3.55))
    elif name.startswith("blood_") and len(name) == 8:
        x, y, sb = _spectrum("blood", int(name[6:]), (-2.2, 11.8))
    elif name.startswith("sim_") and name.endswith("_harness"):
        x, y, sb = _spectrum("sim", int(name[4:6]), (3.34, 3.56))
    elif name == "blood_01_water":
        x, y, sb = _spectrum("blood", 1, (-2.2, 11.8))
        ign = ((4.7, 4.9),)
    elif name == "blood_02_two_regions_increasing":
        # axis reversed to increasing so two ignore regions are legal in compute_mse
        x, y, sb = _spectrum("blood", 2, (-2.2, 11.8))
        x, y = x[::-1].copy(), y[::-1].copy()
        sb = (-2.2, 11.8)
        ign = ((1.0, 1.5), (4.7, 4.9))
    elif name == "sim_01_detector_only":
        x, y, sb = _spectrum("sim", 1, (3.35, 3.55))
        st = _settings(selector="detector_only")
    elif name == "sim_01_identity":
        x, y, sb = _spectrum("sim", 1, (3.35, 3.55))
        st = _settings(smoother="identity")
    elif name == "sim_01_ma5x2_thr3":
        x, y, sb = _spectrum("sim", 1, (3.35, 3.55))
        st = _settings(smooth_iterations=2, smooth_window=5, threshold=3.0, fit_iterations=15)
    elif name.startswith("synth_128k_2k_s"):
        x, y, _ = synth_spectrum(int(name.rsplit("s", 1)[1]))
        sb = (11.8, -2.2)
    else:
        raise KeyError(name)
    return x, y, sb, st, ign


def load_case(name: str):
    x, y, sb, st, ign = _load(name)
    return x, y, sb, st, ign
