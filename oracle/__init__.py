"""ctypes wrapper around the C restatement in ``oracle/md_oracle.c``.

TEST INFRASTRUCTURE ONLY. Import this from ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg -- never from the product package
(``metabodecon-rust_amd/metabodecon``), which must fail loudly without its HIP
library instead of falling back to this CPU code.

Parity status: pinned by the reference's own known-answer unit/doc tests
(``tests/test_oracle_known_answers.py``), which are restated from
metabodecon/src/**/*.rs ``#[cfg(test)]`` modules and doc tests. The Rust
reference itself cannot be built here (no cargo/rustc), so end-to-end outputs
are pinned only through those unit-level answers (see DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MDO_LIB selects another build of the same source (the sanitizer build, tests only)
_LIB_PATH = os.environ.get("MDO_LIB", os.path.join(_HERE, "libmd_oracle.so"))

STATUS = {
    0: "Ok",
    1: "NoPeaksDetected",
    2: "EmptySignalRegion",
    3: "EmptySignalFreeRegion",
    10: "InvalidSmoothingSettings",
    11: "InvalidSelectionSettings",
    12: "InvalidFittingSettings",
    13: "InvalidIgnoreRegion",
    20: "InvalidArgument",
    21: "Capacity",
    30: "ReferencePanic",
}


class Settings(ctypes.Structure):
    _fields_ = [
        ("smoother", ctypes.c_int32),
        ("smooth_iterations", ctypes.c_uint32),
        ("smooth_window", ctypes.c_uint32),
        ("selector", ctypes.c_int32),
        ("scoring", ctypes.c_int32),
        ("fit_iterations", ctypes.c_uint32),
        ("fitter", ctypes.c_int32),
        ("options", ctypes.c_int32),  # mdgpu.h layout (the oracle always sums in the reference order)
        ("threshold", ctypes.c_double),
    ]


class Diag(ctypes.Structure):
    _fields_ = [
        ("n_detected", ctypes.c_int64),
        ("n_selected", ctypes.c_int64),
        ("n_kept", ctypes.c_int64),
        ("sbi0", ctypes.c_int64),
        ("sbi1", ctypes.c_int64),
        ("sfr_mean", ctypes.c_double),
        ("sfr_sd", ctypes.c_double),
        ("sel_left", ctypes.POINTER(ctypes.c_int64)),
        ("sel_center", ctypes.POINTER(ctypes.c_int64)),
        ("sel_right", ctypes.POINTER(ctypes.c_int64)),
        ("sel_cap", ctypes.c_size_t),
        ("range_mask", ctypes.c_uint64),
        ("unsafe_kept", ctypes.c_int64),
        ("x_ok", ctypes.c_int32),
    ]


def build() -> str:
    """Compile the oracle with its Makefile (gcc, no GPU needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _declare(_lib)
    return _lib


_dp = ctypes.POINTER(ctypes.c_double)
_i64p = ctypes.POINTER(ctypes.c_int64)
_szp = ctypes.POINTER(ctypes.c_size_t)


def _declare(L):
    L.mdo_default_settings.argtypes = [ctypes.POINTER(Settings)]
    L.mdo_validate_settings.argtypes = [ctypes.POINTER(Settings)]
    L.mdo_moving_average.argtypes = [_dp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
    L.mdo_second_derivative.argtypes = [_dp, ctypes.c_size_t, _dp]
    L.mdo_second_derivative.restype = None
    L.mdo_find_peak_centers.argtypes = [_dp, ctypes.c_size_t, _i64p, ctypes.c_size_t]
    L.mdo_find_peak_centers.restype = ctypes.c_size_t
    L.mdo_find_right_border.argtypes = [_dp, ctypes.c_size_t]
    L.mdo_find_right_border.restype = ctypes.c_size_t
    L.mdo_find_left_border.argtypes = [_dp, ctypes.c_size_t]
    L.mdo_find_left_border.restype = ctypes.c_size_t
    L.mdo_detect_peaks.argtypes = [_dp, ctypes.c_size_t, _i64p, _i64p, _i64p, ctypes.c_size_t]
    L.mdo_detect_peaks.restype = ctypes.c_size_t
    L.mdo_score_minimum_sum.argtypes = [_dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
    L.mdo_score_minimum_sum.restype = ctypes.c_double
    L.mdo_peak_region_boundaries.argtypes = [_i64p, ctypes.c_size_t, ctypes.c_size_t,
                                             ctypes.c_size_t, _szp, _szp]
    L.mdo_peak_region_boundaries.restype = None
    L.mdo_mean_sd.argtypes = [_dp, ctypes.c_size_t, _dp, _dp]
    L.mdo_mean_sd.restype = None
    L.mdo_mirror_shoulder.argtypes = [_dp]
    L.mdo_mirror_shoulder.restype = None
    L.mdo_solve_stencil.argtypes = [_dp, _dp, _dp, _dp]
    L.mdo_solve_stencil.restype = None
    L.mdo_superposition.argtypes = [ctypes.c_double, _dp, ctypes.c_size_t]
    L.mdo_superposition.restype = ctypes.c_double
    L.mdo_superposition_vec.argtypes = [_dp, ctypes.c_size_t, _dp, ctypes.c_size_t, _dp,
                                        ctypes.c_int]
    L.mdo_superposition_vec.restype = None
    L.mdo_ignore_region_indices.argtypes = [_dp, ctypes.c_size_t, ctypes.c_double,
                                            ctypes.c_double, _dp, ctypes.c_size_t, _i64p]
    L.mdo_ignore_region_indices.restype = ctypes.c_long
    L.mdo_add_ignore_region.argtypes = [_dp, ctypes.c_size_t, ctypes.c_size_t,
                                        ctypes.c_double, ctypes.c_double]
    L.mdo_add_ignore_region.restype = ctypes.c_long
    L.mdo_deconvolute.argtypes = [_dp, _dp, ctypes.c_size_t, ctypes.c_double, ctypes.c_double,
                                  ctypes.POINTER(Settings), _dp, ctypes.c_size_t, _dp,
                                  ctypes.c_size_t, _szp, _dp, ctypes.c_int,
                                  ctypes.POINTER(Diag)]
    L.mdo_deconvolute_batch.argtypes = [ctypes.c_size_t, ctypes.c_size_t, _dp, ctypes.c_size_t,
                                        _dp, _dp, ctypes.POINTER(Settings), _dp,
                                        ctypes.c_size_t, _dp, ctypes.c_size_t, _szp, _dp,
                                        ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.mdo_deconvolute_batch_nested.argtypes = L.mdo_deconvolute_batch.argtypes + [ctypes.c_int]


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def _ptr(a: np.ndarray, t=_dp):
    return a.ctypes.data_as(t)


def default_settings() -> Settings:
    s = Settings()
    lib().mdo_default_settings(ctypes.byref(s))
    return s


def make_settings(smoother="moving_average", smooth_iterations=3, smooth_window=3,
                  selector="noise_score", threshold=5.0, fit_iterations=10) -> Settings:
    s = default_settings()
    s.smoother = 1 if smoother == "moving_average" else 0
    s.smooth_iterations = smooth_iterations
    s.smooth_window = smooth_window
    s.selector = 1 if selector == "noise_score" else 0
    s.threshold = threshold
    s.fit_iterations = fit_iterations
    return s


def moving_average(values, iterations: int, window_size: int) -> np.ndarray:
    v = _f64(values).copy()
    rc = lib().mdo_moving_average(_ptr(v), v.size, iterations, window_size)
    if rc:
        raise RuntimeError(STATUS.get(rc, rc))
    return v


def second_derivative(y) -> np.ndarray:
    y = _f64(y)
    out = np.empty(max(y.size - 2, 0))
    lib().mdo_second_derivative(_ptr(y), y.size, _ptr(out))
    return out


def find_peak_centers(sd) -> list[int]:
    sd = _f64(sd)
    cap = sd.size + 1
    out = np.empty(cap, dtype=np.int64)
    n = lib().mdo_find_peak_centers(_ptr(sd), sd.size, _ptr(out, _i64p), cap)
    return out[:n].tolist()


def find_right_border(sd_right) -> int:
    s = _f64(sd_right)
    return int(lib().mdo_find_right_border(_ptr(s), s.size))


def find_left_border(sd_left) -> int:
    s = _f64(sd_left)
    return int(lib().mdo_find_left_border(_ptr(s), s.size))


def detect_peaks(sd):
    sd = _f64(sd)
    cap = sd.size + 1
    l, c, r = (np.empty(cap, dtype=np.int64) for _ in range(3))
    n = lib().mdo_detect_peaks(_ptr(sd), sd.size, _ptr(l, _i64p), _ptr(c, _i64p),
                               _ptr(r, _i64p), cap)
    return l[:n], c[:n], r[:n]


def score_minimum_sum(abs_sd, left, center, right) -> float:
    a = _f64(abs_sd)
    return float(lib().mdo_score_minimum_sum(_ptr(a), left, center, right))


def peak_region_boundaries(centers, sb) -> tuple[int, int]:
    c = np.ascontiguousarray(centers, dtype=np.int64)
    lo, hi = ctypes.c_size_t(), ctypes.c_size_t()
    lib().mdo_peak_region_boundaries(_ptr(c, _i64p), c.size, sb[0], sb[1], ctypes.byref(lo),
                                     ctypes.byref(hi))
    return lo.value, hi.value


def mean_sd(scores) -> tuple[float, float]:
    s = _f64(scores)
    m, d = ctypes.c_double(), ctypes.c_double()
    lib().mdo_mean_sd(_ptr(s), s.size, ctypes.byref(m), ctypes.byref(d))
    return m.value, d.value


def mirror_shoulder(stencil) -> np.ndarray:
    st = _f64(stencil).copy()
    lib().mdo_mirror_shoulder(_ptr(st))
    return st


def solve_stencil(stencil) -> tuple[float, float, float]:
    st = _f64(stencil)
    a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    lib().mdo_solve_stencil(_ptr(st), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return a.value, b.value, c.value


def superposition_vec(x, params, threads: int = 1) -> np.ndarray:
    x = _f64(x)
    p = _f64(params).reshape(-1, 3)
    out = np.empty(x.size)
    lib().mdo_superposition_vec(_ptr(x), x.size, _ptr(p), p.shape[0], _ptr(out), threads)
    return out


def ignore_region_indices(x, sb, regions) -> list[tuple[int, int]]:
    x = _f64(x)
    r = _f64(regions).reshape(-1)
    pairs = np.empty(r.size + 2, dtype=np.int64)
    n = lib().mdo_ignore_region_indices(_ptr(x), x.size, sb[0], sb[1], _ptr(r), r.size // 2,
                                        _ptr(pairs, _i64p))
    return [(int(pairs[2 * i]), int(pairs[2 * i + 1])) for i in range(n)]


def add_ignore_region(regions: list[tuple[float, float]], new) -> list[tuple[float, float]]:
    cap = len(regions) + 1
    buf = np.zeros(2 * cap)
    for i, (a, b) in enumerate(regions):
        buf[2 * i], buf[2 * i + 1] = a, b
    n = lib().mdo_add_ignore_region(_ptr(buf), len(regions), cap, new[0], new[1])
    if n < 0:
        raise ValueError("InvalidIgnoreRegion")
    return [(float(buf[2 * i]), float(buf[2 * i + 1])) for i in range(n)]


@dataclass
class OracleResult:
    status: int
    params: np.ndarray  # (P_kept, 3) = sfhw, hw2, maxp
    mse: float
    n_detected: int
    n_selected: int
    selected: np.ndarray  # (P_sel, 3) = left, center, right
    sbi: tuple[int, int]
    sfr_mean: float
    sfr_sd: float
    # the engine's fast-division ranges (mdo_diag): bit v = parameter version v has a
    # peak outside them; retained Lorentzians outside them; axis ends inside them
    range_mask: int = 0
    unsafe_kept: int = 0
    x_ok: int = 1


def deconvolute(x, y, sb, settings: Settings | None = None, ignore=(), threads: int = 1,
                cap: int | None = None) -> OracleResult:
    x, y = _f64(x), _f64(y)
    if settings is None:
        settings = default_settings()
    ign = _f64(np.asarray(ignore, dtype=np.float64).reshape(-1))
    n = y.size
    if cap is None:
        cap = n // 2 + 2
    out = np.empty((cap, 3))
    cnt = ctypes.c_size_t(0)
    mse = ctypes.c_double(0.0)
    sel = [np.empty(cap, dtype=np.int64) for _ in range(3)]
    d = Diag()
    d.sel_left, d.sel_center, d.sel_right = (_ptr(a, _i64p) for a in sel)
    d.sel_cap = cap
    rc = lib().mdo_deconvolute(_ptr(x), _ptr(y), n, sb[0], sb[1], ctypes.byref(settings),
                               _ptr(ign) if ign.size else None, ign.size // 2, _ptr(out), cap,
                               ctypes.byref(cnt), ctypes.byref(mse), threads, ctypes.byref(d))
    k = cnt.value if rc == 0 else 0
    ns = max(int(d.n_selected), 0) if rc == 0 else 0
    return OracleResult(rc, out[:k].copy(), mse.value, int(d.n_detected), int(d.n_selected),
                        np.stack([a[:ns] for a in sel], axis=1), (int(d.sbi0), int(d.sbi1)),
                        d.sfr_mean, d.sfr_sd, int(d.range_mask), int(d.unsafe_kept), int(d.x_ok))


def deconvolute_batch(x, y, sb, settings: Settings | None = None, ignore=(), threads: int = 1,
                      cap: int = 4096, inner_threads: int = 1):
    """x: (n,) shared axis or (b, n); y: (b, n); sb: (b, 2). Returns (status, counts, params, mse).
    ``threads`` workers over spectra, ``inner_threads`` per spectrum's superpositions."""
    y = _f64(y)
    b, n = y.shape
    x = _f64(x)
    x_stride = 0 if x.ndim == 1 else n
    sbv = _f64(np.broadcast_to(np.asarray(sb, dtype=np.float64), (b, 2)))
    if settings is None:
        settings = default_settings()
    ign = _f64(np.asarray(ignore, dtype=np.float64).reshape(-1))
    out = np.zeros((b, cap, 3))
    counts = np.zeros(b, dtype=np.uintp)
    mse = np.zeros(b)
    status = np.zeros(b, dtype=np.int32)
    lib().mdo_deconvolute_batch_nested(b, n, _ptr(x), x_stride, _ptr(y), _ptr(sbv),
                                       ctypes.byref(settings), _ptr(ign) if ign.size else None,
                                       ign.size // 2, _ptr(out), cap, _ptr(counts, _szp),
                                       _ptr(mse),
                                       status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                       threads, inner_threads)
    return status, counts.astype(np.int64), out, mse


def optimize_settings_grid():
    """The reference's grid in its order (deconvoluter.rs:762-788): smoothing
    (iterations 2..=10 x window 3, 5, 7) outermost, then the 10 noise-score
    thresholds 5 + c * 3 / 9, then the analytical fit iterations 5, 10, 15."""
    grid = []
    for it in range(2, 11):
        for ws in (3, 5, 7):
            for c in range(10):
                thr = 5.0 + (c * (8.0 - 5.0)) / 9.0
                for fit in (5, 10, 15):
                    grid.append((it, ws, thr, fit))
    return grid


def optimize_settings(x, y, sb, ignore=(), threads: int = 1):
    """Deconvoluter::optimize_settings (deconvoluter.rs:762-825): every grid setting
    deconvolutes the reference spectrum; a failing one returns its status (the
    reference's `?`; the first in grid order here); otherwise the FIRST minimum MSE
    in grid order wins (Iterator::min_by). Returns (status, (iterations, window,
    threshold, fit_iterations) or None, mse). The 810 deconvolutions run on
    ``threads`` worker threads (ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    grid = optimize_settings_grid()
    x, y = _f64(x), _f64(y)

    def one(g):
        it, ws, thr, fit = g
        st = make_settings(smooth_iterations=it, smooth_window=ws, threshold=thr,
                           fit_iterations=fit)
        r = deconvolute(x, y, sb, st, ignore=ignore)
        return r.status, r.mse

    with ThreadPoolExecutor(max_workers=max(1, threads)) as pool:
        res = list(pool.map(one, grid))
    for st, _ in res:
        if st:
            return st, None, None
    best = 0
    for k in range(1, len(res)):
        if res[k][1] < res[best][1]:
            best = k
    return 0, grid[best], res[best][1]
