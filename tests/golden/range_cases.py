"""Spectra outside the engine's fast-division ranges.

The fit and superposition_vec use div_rn -- the IEEE division without its
div_scale/div_fmas/div_fixup wrappers, bit-identical by construction only inside
|sfhw|, hw2 in [2^-200, 2^200], |maxp| <= 2^100, |x| <= 2^100 -- when per-spectrum
flags prove those ranges for the parameter version an iteration reads; otherwise the
plain `/`. Scaling a spectrum's intensities by c scales every sfhw by
c, so the factors below (found by ``tools/range_cases.py``, which traces log2 max/min
|sfhw| per parameter version) put one spectrum's largest (or smallest) sfhw just
across a range bound at chosen iterations: the fast flag flips in the middle of the
fit, both ways, and in both flag protocols (the ping-pong slots of k_fit_sup /
k_fit_update and the three-slot rotation of the term folds).

Each case: (name, golden spectrum, y factor, x factor, expected oracle range_mask over
parameter versions 0..10 as a string, bit v left to right, expected unsafe_kept > 0).
The masks are pinned by ``tests/test_range_cases_oracle.py`` (CPU) and compared with
the engine's own record of its slow launches by ``tests/test_gpu_range_paths.py``.
"""
import numpy as np

# (case id, spectrum, y scale, x scale, oracle range mask v0..v10, retained outside)
RANGE_CASES = [
    # every version out (sfhw > 2^200), MSE direct too
    ("up200_blood01", "blood_01", 2.0 ** 200, 1.0, "11111111111", True),
    # slow at iterations 0 and 2 only: the flag raised for one iteration mid-fit
    ("flip_blood01", "blood_01", 2.0 ** (200.0 - 8.2238), 1.0, "10100000000", False),
    # slow 0-4, fast at 5, slow again 6-10 (the largest sfhw dips under 2^200 once)
    ("dip_blood05", "blood_05", 2.0 ** (200.0 - 8.2535), 1.0, "11111011111", True),
    # slow at 0, fast 1-3, slow from 4 on
    ("late_sim03", "sim_03", 2.0 ** (200.0 - 3.8630), 1.0, "10001111111", True),
    # lower bound: the smallest |sfhw| falls under 2^-200 at version 2, back at 3, under from 4
    ("low_blood05", "blood_05", 2.0 ** (-200.0 + 43.8), 1.0, "00101111111", False),
    # lower bound: fast 0-4, slow from iteration 5
    ("low_blood01", "blood_01", 2.0 ** (-200.0 + 62.0), 1.0, "00000111111", False),
    # axis and signal boundaries past 2^100: x_ok false, every launch slow
    ("x101_blood01", "blood_01", 1.0, 2.0 ** 101, "11111111111", True),
]


def range_case(case):
    """(x, y, sb, settings, ignore) of a RANGE_CASES entry."""
    from tests.golden.cases import load_case
    _, name, yc, xc, _, _ = case
    x, y, sb, st, ign = load_case(name)
    return x * xc, y * yc, (sb[0] * xc, sb[1] * xc), st, ign


def mask_bits(s: str) -> int:
    return sum(1 << v for v, ch in enumerate(s) if ch == "1")


def mixed_superposition_inputs(seed=5, n=20000, p=300):
    """superposition_vec operands with a few parameters and points outside the fast
    ranges among in-range ones (lorentzian.rs:631-663 takes any finite values)."""
    rng = np.random.default_rng(seed)
    x = np.sort(rng.uniform(-5, 15, n))[::-1].copy()
    params = np.stack([rng.uniform(1e-3, 1e3, p), rng.uniform(1e-8, 1e-5, p),
                       rng.uniform(-2, 12, p)], axis=1)
    params[7] = (2.0 ** 210, 3e-6, 4.2)       # |sfhw| > 2^200
    params[100] = (2.0 ** -205, 2e-6, 7.5)    # |sfhw| < 2^-200
    params[150] = (12.0, 2.0 ** -210, 9.1)    # hw2 < 2^-200
    params[151] = (12.0, 2.0 ** 205, 1.0)     # hw2 > 2^200
    params[299] = (-3.0, 5e-6, 2.0 ** 101)    # |maxp| > 2^100
    x_far = x.copy()
    x_far[[0, 17, n - 1]] = (2.0 ** 101, -(2.0 ** 102), 2.0 ** 100 * 1.5)  # |x| > 2^100 points
    return x, x_far, params
