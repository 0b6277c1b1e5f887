"""``Deconvoluter`` / ``Deconvolution`` / ``Lorentzian`` over the C ABI.

Mirrors metabodecon-python/src/bindings/{deconvoluter,deconvolution,lorentzian}.rs
(method names, argument meaning and exceptions). Every ``deconvolute_*`` and
``*superposition_vec`` call runs the HIP path in libmdgpu.so; scalar helpers
(``evaluate``, ``superposition`` at one point) are evaluated on the host with
the same operation order as lorentzian.rs:546-611.
"""
from __future__ import annotations

import ctypes
import os
import math

import numpy as np

from . import _native as nat
from . import _serde as serde
from . import exceptions as exc
from ._spectrum import Spectrum

_sz = ctypes.c_size_t


# =====================================================================================
# Lorentzian (bindings/lorentzian.rs:24-113, lorentzian.rs:138-663)
# =====================================================================================
class Lorentzian:
    __slots__ = ("sfhw", "hw2", "_maxp")

    def __init__(self, sf: float, hw: float, maxp: float):
        # bindings/lorentzian.rs:26-31: untransformed parameters
        self.sfhw = float(sf) * float(hw)
        self.hw2 = float(hw) * float(hw)
        self._maxp = float(maxp)

    @staticmethod
    def from_transformed(sfhw: float, hw2: float, maxp: float) -> "Lorentzian":
        lz = Lorentzian.__new__(Lorentzian)
        lz.sfhw, lz.hw2, lz._maxp = float(sfhw), float(hw2), float(maxp)
        return lz

    @property
    def hw(self) -> float:
        return math.sqrt(self.hw2)  # lorentzian.rs:428

    @hw.setter
    def hw(self, hw: float):  # lorentzian.rs:501-504
        self.sfhw = self.sf * hw
        self.hw2 = hw * hw

    @property
    def sf(self) -> float:
        return self.sfhw / self.hw  # lorentzian.rs:406

    @sf.setter
    def sf(self, sf: float):  # lorentzian.rs:477-479
        self.sfhw = sf * self.hw

    @property
    def maxp(self) -> float:
        return self._maxp

    @maxp.setter
    def maxp(self, v: float):
        self._maxp = float(v)

    def parameters(self) -> tuple[float, float, float]:
        return self.sfhw, self.hw2, self._maxp

    def evaluate(self, x: float) -> float:
        d = float(x) - self._maxp
        return self.sfhw / (self.hw2 + d * d)

    def evaluate_vec(self, x) -> np.ndarray:
        x = np.asarray(x, dtype=np.float64)
        d = x - self._maxp
        return self.sfhw / (self.hw2 + d * d)

    def integral(self) -> float:
        return math.pi * self.sf

    @staticmethod
    def superposition(x: float, lorentzians) -> float:
        acc = -0.0
        for lz in lorentzians:
            acc += lz.evaluate(x)
        return acc

    @staticmethod
    def superposition_vec(x, lorentzians) -> np.ndarray:
        return superposition_vec(x, _params_of(lorentzians))

    @staticmethod
    def par_superposition_vec(x, lorentzians) -> np.ndarray:
        return superposition_vec(x, _params_of(lorentzians))

    def __repr__(self) -> str:
        return f"Lorentzian(sfhw={self.sfhw!r}, hw2={self.hw2!r}, maxp={self._maxp!r})"


def _params_of(lorentzians) -> np.ndarray:
    if isinstance(lorentzians, np.ndarray):
        return np.ascontiguousarray(lorentzians, dtype=np.float64).reshape(-1, 3)
    return np.array([lz.parameters() for lz in lorentzians], dtype=np.float64).reshape(-1, 3)


def superposition_vec(x, params: np.ndarray, device: int | None = None) -> np.ndarray:
    """Lorentzian::superposition_vec on the GPU (lorentzian.rs:631-663)."""
    xa = np.asarray(x, dtype=np.float64)
    if xa.ndim != 1 or not xa.flags.c_contiguous:
        # the reference's `as_slice().unwrap()` panics on non-contiguous input
        # (bindings/deconvolution.rs:63-75); we accept it and copy instead.
        xa = np.ascontiguousarray(xa.reshape(-1))
    params = np.ascontiguousarray(params, dtype=np.float64).reshape(-1, 3)
    out = np.empty(xa.size)
    ctx = nat.context(device)
    with ctx.lock:
        st = nat.lib().mdg_superposition_vec(ctx.handle, nat.ptr(xa), xa.size, nat.ptr(params),
                                             params.shape[0], nat.ptr(out))
    if st:
        raise exc.UnexpectedError(f"superposition_vec failed: {nat.strerror(st)}")
    return out


# =====================================================================================
# settings serialisation (serde forms of smoother.rs:21-56, selector.rs:26-58,
# scorer.rs:15-29, fitter.rs:28-57: internally tagged on "method", camelCase fields)
# =====================================================================================
_U32_MAX = (1 << 32) - 1


def _settings_serde(s: nat.Settings, as_array: bool) -> list:
    if as_array:  # rmp_serde: [tag, fields...]
        sm = (["MovingAverage", s.smooth_iterations, s.smooth_window] if s.smoother == 1
              else ["Identity"])
        se = (["NoiseScoreFilter", ["MinimumSum"], s.threshold] if s.selector == 1
              else ["DetectorOnly"])
        return [sm, se, ["Analytical", s.fit_iterations]]
    sm = ({"method": "MovingAverage", "iterations": s.smooth_iterations,
           "windowSize": s.smooth_window} if s.smoother == 1 else {"method": "Identity"})
    se = ({"method": "NoiseScoreFilter", "scoringMethod": {"method": "MinimumSum"},
           "threshold": s.threshold} if s.selector == 1 else {"method": "DetectorOnly"})
    return [sm, se, {"method": "Analytical", "iterations": s.fit_iterations}]


def _engine_u32(v: int, what: str) -> int:
    if v > _U32_MAX:
        raise serde.SerdeError(f"{what} = {v} exceeds the engine's u32 settings field")
    return v


def _settings_from_serde(sm, se, fi) -> nat.Settings:
    s = nat.default_settings()
    tag, rest = serde.tagged(sm, "SmoothingSettings")
    if tag == "Identity":
        s.smoother = 0
    elif tag == "MovingAverage":
        f = serde.fields(rest, ("iterations", "windowSize"), "SmoothingSettings::MovingAverage")
        s.smoother = 1
        s.smooth_iterations = _engine_u32(serde.usize(f["iterations"], "iterations"),
                                          "iterations")
        s.smooth_window = _engine_u32(serde.usize(f["windowSize"], "windowSize"), "windowSize")
    else:
        raise serde.SerdeError(f"unknown variant `{tag}`, expected `Identity` or `MovingAverage`")
    tag, rest = serde.tagged(se, "SelectionSettings")
    if tag == "DetectorOnly":
        s.selector = 0
    elif tag == "NoiseScoreFilter":
        f = serde.fields(rest, ("scoringMethod", "threshold"),
                         "SelectionSettings::NoiseScoreFilter")
        stag, _ = serde.tagged(f["scoringMethod"], "ScoringMethod")
        if stag != "MinimumSum":
            raise serde.SerdeError(f"unknown variant `{stag}`, expected `MinimumSum`")
        s.selector = 1
        s.threshold = serde.f64(f["threshold"], "threshold")
    else:
        raise serde.SerdeError(
            f"unknown variant `{tag}`, expected `DetectorOnly` or `NoiseScoreFilter`")
    tag, rest = serde.tagged(fi, "FittingSettings")
    if tag != "Analytical":
        raise serde.SerdeError(f"unknown variant `{tag}`, expected `Analytical`")
    f = serde.fields(rest, ("iterations",), "FittingSettings::Analytical")
    s.fit_iterations = _engine_u32(serde.usize(f["iterations"], "iterations"), "iterations")
    # TryFrom<SerializedDeconvolution> validates (serialized_deconvolution.rs:34-49)
    st = nat.validate(s)
    if st:
        raise serde.SerdeError(str(exc.from_status(st)))
    return s


# =====================================================================================
# Deconvolution (bindings/deconvolution.rs:45-116, deconvolution.rs:45-115)
# =====================================================================================
class Deconvolution:
    def __init__(self, params: np.ndarray, mse: float, settings: nat.Settings):
        self._params = np.ascontiguousarray(params, dtype=np.float64).reshape(-1, 3)
        self._params.setflags(write=False)
        self._mse = float(mse)
        self._settings = settings.copy()

    @classmethod
    def _of(cls, params: np.ndarray, mse: float, settings: nat.Settings) -> "Deconvolution":
        """The engine's results: `params` a fresh (P, 3) float64 array owned by the
        result, `settings` a snapshot no one mutates (shared by one call's results)."""
        d = cls.__new__(cls)
        params.setflags(write=False)
        d._params = params
        d._mse = mse
        d._settings = settings
        return d

    @property
    def lorentzians(self) -> list[Lorentzian]:
        return [Lorentzian.from_transformed(*row) for row in self._params.tolist()]

    @property
    def params(self) -> np.ndarray:
        """(P, 3) array of transformed parameters (sfhw, hw2, maxp)."""
        return self._params

    @property
    def mse(self) -> float:
        return self._mse

    def superposition(self, x: float) -> float:
        acc = -0.0
        for sfhw, hw2, maxp in self._params.tolist():
            d = float(x) - maxp
            acc += sfhw / (hw2 + d * d)
        return acc

    def superposition_vec(self, x) -> np.ndarray:
        return superposition_vec(x, self._params)

    def par_superposition_vec(self, x) -> np.ndarray:
        return superposition_vec(x, self._params)

    # ---- serialisation (bindings/deconvolution.rs:77-116) ------------------------------
    def _serialized(self, as_array: bool):
        """SerializedDeconvolution (serialized_deconvolution.rs:9-31) with
        SerializedLorentzian {sf, hw, maxp} = (sfhw / sqrt(hw2), sqrt(hw2), maxp)
        (serialized_lorentzian.rs:5-21, lorentzian.rs:406-430)."""
        sm, se, fi = _settings_serde(self._settings, as_array)
        lz = []
        for sfhw, hw2, maxp in self._params.tolist():
            hw = math.sqrt(hw2)
            sf = sfhw / hw
            lz.append([sf, hw, maxp] if as_array else {"sf": sf, "hw": hw, "maxp": maxp})
        if as_array:
            return [sm, se, fi, self._mse, lz]
        return {"smoothingSettings": sm, "selectionSettings": se, "fittingSettings": fi,
                "mse": self._mse, "lorentzians": lz}

    def to_json_dict(self) -> dict:
        return self._serialized(as_array=False)

    @staticmethod
    def _from_serialized(v) -> "Deconvolution":
        d = serde.fields(v, ("smoothingSettings", "selectionSettings", "fittingSettings", "mse",
                             "lorentzians"), "Deconvolution")
        s = _settings_from_serde(d["smoothingSettings"], d["selectionSettings"],
                                 d["fittingSettings"])
        mse = serde.f64(d["mse"], "mse")
        if not isinstance(d["lorentzians"], list):
            raise serde.SerdeError("invalid type for lorentzians: expected a sequence")
        rows = []
        for l in d["lorentzians"]:
            f = serde.fields(l, ("sf", "hw", "maxp"), "Lorentzian")
            sf, hw, maxp = (serde.f64(f[k], k) for k in ("sf", "hw", "maxp"))
            # Lorentzian::new(sf * hw, hw.powi(2), maxp) (serialized_lorentzian.rs:23-27)
            rows.append((sf * hw, hw * hw, maxp))
        return Deconvolution(np.array(rows, dtype=np.float64).reshape(-1, 3), mse, s)

    def write_json(self, path: str) -> None:
        text = serde.to_string_pretty(self._serialized(as_array=False))
        with open(path, "wb") as f:
            f.write(text.encode("utf-8"))

    @staticmethod
    def read_json(path: str) -> "Deconvolution":
        with open(path, "rb") as f:
            raw = f.read()
        try:
            text = raw.decode("utf-8")
        except UnicodeDecodeError as e:
            raise OSError("stream did not contain valid UTF-8") from e
        try:
            return Deconvolution._from_serialized(serde.from_str(text))
        except serde.SerdeError as e:
            raise serde.serialization_error(e) from None

    def write_bin(self, path: str) -> None:
        with open(path, "wb") as f:
            f.write(serde.to_msgpack(self._serialized(as_array=True)))

    @staticmethod
    def read_bin(path: str) -> "Deconvolution":
        with open(path, "rb") as f:
            raw = f.read()
        try:
            return Deconvolution._from_serialized(serde.from_msgpack(raw))
        except serde.SerdeError as e:
            raise serde.serialization_error(e) from None

    def __repr__(self) -> str:
        return f"Deconvolution(lorentzians={self._params.shape[0]}, mse={self._mse!r})"


# =====================================================================================
# Deconvoluter (bindings/deconvoluter.rs:17-165, deconvoluter.rs:118-905)
# =====================================================================================
_pool = None


def _lane_pool(n: int):
    global _pool
    if _pool is None:
        from concurrent.futures import ThreadPoolExecutor
        _pool = ThreadPoolExecutor(max_workers=n, thread_name_prefix="mdgpu-lane")
    return _pool


class Deconvoluter:
    def __init__(self):
        self._s = nat.default_settings()
        self._ignore: list[tuple[float, float]] | None = None
        self._threads: int | None = None
        self.device: int | None = None

    # ---- settings -----------------------------------------------------------------
    def _apply(self, s: nat.Settings):
        st = nat.validate(s)
        if st:
            raise exc.from_status(st)
        self._s = s

    def set_identity_smoother(self) -> None:
        s = self._s.copy()
        s.smoother = 0
        self._apply(s)

    def set_moving_average_smoother(self, iterations: int, window_size: int) -> None:
        if iterations < 0 or window_size < 0:
            raise OverflowError("can't convert negative int to unsigned")
        s = self._s.copy()
        s.smoother, s.smooth_iterations, s.smooth_window = 1, iterations, window_size
        self._apply(s)

    def set_detector_only(self) -> None:
        s = self._s.copy()
        s.selector = 0
        self._apply(s)

    def set_noise_score_selector(self, threshold: float) -> None:
        s = self._s.copy()
        s.selector, s.scoring, s.threshold = 1, 0, float(threshold)
        self._apply(s)

    def set_analytical_fitter(self, iterations: int) -> None:
        if iterations < 0:
            raise OverflowError("can't convert negative int to unsigned")
        s = self._s.copy()
        s.fitter, s.fit_iterations = 0, iterations
        self._apply(s)

    @property
    def settings(self) -> nat.Settings:
        return self._s.copy()

    @property
    def exact_mse(self) -> bool:
        """Engine option (not a reference setting): compute each Deconvolution's MSE in
        the reference's summation order (compute_mse, deconvoluter.rs:828-862), so
        ``Deconvolution.mse`` and the serialized files' ``mse`` equal the reference's
        bit for bit. Off (the default) the engine's MSE is within 1e-12 relative of it
        and cheaper; Lorentzians are bit-identical either way (mdgpu.h
        MDG_OPTION_EXACT_MSE)."""
        return bool(self._s.options & nat.OPTION_EXACT_MSE)

    @exact_mse.setter
    def exact_mse(self, on: bool) -> None:
        s = self._s.copy()
        s.options = (s.options | nat.OPTION_EXACT_MSE) if on else (s.options & ~nat.OPTION_EXACT_MSE)
        self._apply(s)

    def add_ignore_region(self, boundaries) -> None:
        a, b = float(boundaries[0]), float(boundaries[1])
        cur = self._ignore or []
        cap = len(cur) + 1
        buf = np.zeros(2 * cap)
        for i, (lo, hi) in enumerate(cur):
            buf[2 * i], buf[2 * i + 1] = lo, hi
        n = _sz(0)
        st = nat.lib().mdg_ignore_region_add(nat.ptr(buf), len(cur), cap, a, b, ctypes.byref(n))
        if st:
            raise exc.InvalidIgnoreRegion(
                f"ignore region boundaries [{a}, {b}] are invalid")
        self._ignore = [(float(buf[2 * i]), float(buf[2 * i + 1])) for i in range(n.value)]

    def clear_ignore_regions(self) -> None:
        self._ignore = None

    @property
    def ignore_regions(self) -> list[tuple[float, float]] | None:
        return None if self._ignore is None else list(self._ignore)

    def set_threads(self, threads: int) -> None:
        # bindings/deconvoluter.rs:92-106; the GPU engine has no CPU pool to size
        if threads <= 1:
            raise ValueError("number of threads must be greater than 1")
        self._threads = threads

    def clear_threads(self) -> None:
        self._threads = None

    # ---- hot path -------------------------------------------------------------------
    def _ignore_array(self) -> np.ndarray:
        if not self._ignore:
            return np.zeros(0)
        return np.array(self._ignore, dtype=np.float64).reshape(-1)

    # Engine contexts (own HIP stream and workspace each) a call spreads its spectra
    # over, concurrently: a set of one length is cut into contiguous chunks (at least
    # one per lane, at most CHUNK spectra each), dealt round-robin to the lanes, each
    # chunk one batched pipeline; each lane's sequential smoother overlaps the other
    # lane's fit. (Round 3 measured two lanes best for the 16 blood spectra, 2.65-2.72
    # ms per set against 9.3-9.9 for one batch of 16; since round 4's small-batch fit
    # and in-launch decode, one batch wins for such sets: ONE_LANE_UPTO.) HIP maps streams
    # round-robin onto GPU_MAX_HW_QUEUES hardware queues and two busy streams on one
    # queue serialise, so the lanes also stay below that count (one queue is left
    # for the caller's own stream). MDGPU_LANES overrides the count.
    LANES = max(1, min(16, int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) - 1,
                       int(os.environ.get("MDGPU_LANES", "2") or 2)))
    CHUNK = 256  # spectra per batched call (the host staging of one call stays bounded)
    # Sets of up to this many spectra of one length run as one batch on one context
    # (unless MDGPU_LANES is set): since the pipeline decodes page-locked compact rows
    # while the smoother runs (round 4), one batch of the 16 blood spectra takes
    # 13.6-13.7k spectra/s in three rounds against 12.4-13.0k for two lanes of 8
    # (tools/gpu_run.sh c4lanes, 4 and 32 hardware queues alike).
    ONE_LANE_UPTO = 0 if os.environ.get("MDGPU_LANES") else 16

    def _run_one(self, ctx, sp: Spectrum, n: int, ign):
        """_run_batch for one spectrum with the ctypes arguments cached: the
        spectrum's row pointers on the spectrum (its rows never change), the result
        scratch and its pointers on the context. A single call's Python cost fell from
        ~42 to ~7 us (configs[0], one deconvolute_spectrum at a time; stubbed engine)."""
        f = sp.__dict__.get("_ffi_one")
        if f is None:
            raw = sp._raw
            if raw is not None:
                yr = np.array([raw[0].ctypes.data], dtype=np.uintp)
                axes = np.array([raw[2]], dtype=np.float64)
                scale = np.array([raw[1]], dtype=np.float64)
                f = (True, (yr, axes, scale), (axes.ctypes.data, yr.ctypes.data, scale.ctypes.data))
            else:
                xr = np.array([sp.chemical_shifts.ctypes.data], dtype=np.uintp)
                yr = np.array([sp.intensities.ctypes.data], dtype=np.uintp)
                f = (False, (xr, yr), (xr.ctypes.data, yr.ctypes.data))
            sp.__dict__["_ffi_one"] = f
        cap = n // 2 + 2
        with ctx.lock:
            one = ctx.__dict__.get("_one")
            out = ctx.host_rows("out", (1, cap, 3))
            if one is None or one[0] is not out:
                counts = np.zeros(1, dtype=np.uintp)
                mse = np.zeros(1)
                status = np.zeros(1, dtype=np.intc)
                sb = np.zeros(2)
                one = (out, counts, mse, status, sb,
                       (out.ctypes.data, cap, counts.ctypes.data, mse.ctypes.data, status.ctypes.data),
                       sb.ctypes.data)
                ctx.__dict__["_one"] = one
            out, counts, mse, status, sb, tail, sbp = one
            if tail[1] != cap:
                tail = (tail[0], cap) + tail[2:]
            sb[0], sb[1] = sp.signal_boundaries
            ig = (ign.ctypes.data if ign.size else None, ign.size // 2)
            if f[0]:
                rc = nat.lib().mdg_deconvolute_rows_i32(ctx.handle, 1, n, *f[2], sbp, ctypes.byref(self._s),
                                                        *ig, *tail)
            else:
                rc = nat.lib().mdg_deconvolute_rows(ctx.handle, 1, n, *f[2], sbp, ctypes.byref(self._s), *ig,
                                                    *tail)
            if rc >= 100 or rc == nat.INVALID_ARGUMENT:
                raise exc.UnexpectedError(f"GPU engine failure: {nat.strerror(rc)}")
            return int(status[0]), out[0, : int(counts[0])].copy(), float(mse[0])

    @staticmethod
    def _ffi_rows(sp: Spectrum):
        """A spectrum's row addresses and axis operands for the batched call, kept on
        the spectrum (its rows never change): (compact, y or sample row address, axis
        triple, scale, x row address)."""
        f = sp.__dict__.get("_ffi_b")
        if f is None:
            raw = sp._raw
            if raw is not None:
                f = (True, raw[0].ctypes.data, tuple(raw[2]), float(raw[1]), 0)
            else:
                f = (False, sp.intensities.ctypes.data, (), 0.0, sp.chemical_shifts.ctypes.data)
            sp.__dict__["_ffi_b"] = f
        return f

    def _run_batch(self, ctx, spectra: list[Spectrum], idx: list[int], n: int, ign):
        """One batched call on one context: the rows by address (no stacking copy;
        page-locked rows go by DMA straight from where they are), the per-call
        descriptors in the context's own small arrays (kept with their addresses), the
        result rows in the context's host buffer. Plain integer addresses throughout:
        the Python side of a 16-spectrum call fell from ~140 to ~25 us (stub engine)."""
        b = len(idx)
        cap = n // 2 + 2
        rows = [self._ffi_rows(spectra[i]) for i in idx]
        compact = all(r[0] for r in rows)
        with ctx.lock:  # ctypes drops the GIL for the call: lanes run concurrently
            scr = ctx.__dict__.get("_bscr")
            if scr is None or scr[0] < b:
                m = max(b, 16)
                arrs = (np.zeros(m, dtype=np.uintp), np.zeros(m, dtype=np.uintp), np.zeros((m, 3)),
                        np.zeros(m), np.zeros((m, 2)), np.zeros(m, dtype=np.uintp), np.zeros(m),
                        np.zeros(m, dtype=np.intc))
                scr = (m, arrs, tuple(a.ctypes.data for a in arrs))
                ctx.__dict__["_bscr"] = scr
            (yr, xr, axes, scale, sb, counts, mse, status), (a_yr, a_xr, a_ax, a_sc, a_sb, a_cnt, a_mse,
                                                              a_st) = scr[1], scr[2]
            sb[:b] = [spectra[i].signal_boundaries for i in idx]
            if compact:
                yr[:b] = [r[1] for r in rows]
                axes[:b] = [r[2] for r in rows]
                scale[:b] = [r[3] for r in rows]
            else:  # a compact spectrum in a mixed batch sends its f64 rows
                yr[:b] = [spectra[i].intensities.ctypes.data if r[0] else r[1] for i, r in zip(idx, rows)]
                xr[:b] = [spectra[i].chemical_shifts.ctypes.data if r[0] else r[4] for i, r in zip(idx, rows)]
            # the result rows: the context's own host buffer, kept across calls
            out = ctx.host_rows("out", (b, cap, 3))
            ig = (ign.ctypes.data if ign.size else None, ign.size // 2)
            tail = (out.ctypes.data, cap, a_cnt, a_mse, a_st)
            if compact:
                rc = nat.lib().mdg_deconvolute_rows_i32(ctx.handle, b, n, a_ax, a_yr, a_sc, a_sb,
                                                        ctypes.byref(self._s), *ig, *tail)
            else:
                rc = nat.lib().mdg_deconvolute_rows(ctx.handle, b, n, a_xr, a_yr, a_sb,
                                                    ctypes.byref(self._s), *ig, *tail)
            if rc >= 100 or rc == nat.INVALID_ARGUMENT:
                raise exc.UnexpectedError(f"GPU engine failure: {nat.strerror(rc)}")
            # copied out while the rows are still this call's
            cl, sl, ml = counts[:b].tolist(), status[:b].tolist(), mse[:b].tolist()
            return [(sl[k], out[k, : cl[k]].copy(), ml[k]) for k in range(b)]

    def _run(self, spectra: list[Spectrum]) -> list[tuple[int, np.ndarray, float]]:
        """GPU results per spectrum, (status, params, mse) in input order: the
        spectra of one length are cut into contiguous chunks (at least one per lane,
        at most CHUNK spectra), dealt round-robin to min(LANES, count) lane contexts
        that run concurrently, one batched pipeline per chunk."""
        results: list = [None] * len(spectra)
        by_n: dict[int, list[int]] = {}
        for i, sp in enumerate(spectra):
            if not isinstance(sp, Spectrum):
                raise TypeError("expected metabodecon.Spectrum")
            by_n.setdefault(len(sp), []).append(i)
        ign = self._ignore_array()
        from .distributed import shard_range
        for n, idx in by_n.items():
            lanes_n = 1 if len(idx) <= self.ONE_LANE_UPTO else min(self.LANES, len(idx))
            k = max(lanes_n, -(-len(idx) // self.CHUNK))
            chunks = [idx[lo:hi] for lo, hi in (shard_range(len(idx), r, k) for r in range(k))]
            if lanes_n <= 1:
                for c in chunks:
                    for i, r in zip(c, self._run_batch(nat.context(self.device), spectra, c, n, ign)):
                        results[i] = r
                continue
            lanes = nat.lane_contexts(self.device, lanes_n)
            pool = _lane_pool(self.LANES)

            def lane_work(j):  # lane j runs chunks j, j + lanes_n, ... one after another
                out = []
                for c in chunks[j::lanes_n]:
                    out.append((c, self._run_batch(lanes[j], spectra, c, n, ign)))
                return out
            # the last lane runs in the calling thread (one pool hand-off fewer)
            futs = [pool.submit(lane_work, j) for j in range(lanes_n - 1)]
            mine = lane_work(lanes_n - 1)
            for part in [f.result() for f in futs] + [mine]:
                for c, res in part:
                    for i, r in zip(c, res):
                        results[i] = r
        return results

    def _collect(self, results) -> list[Deconvolution]:
        out = []
        snap = self._s.copy()  # one snapshot of the settings for the call's results
        for st, params, mse in results:  # fail-fast Result collect (deconvoluter.rs:655-658)
            if st:
                raise exc.from_status(st)
            out.append(Deconvolution._of(params, mse, snap))
        return out

    def deconvolute_spectrum(self, spectrum: Spectrum) -> Deconvolution:
        if not isinstance(spectrum, Spectrum):
            raise TypeError("expected metabodecon.Spectrum")
        ign = self._ign_cache()
        return self._collect([self._run_one(nat.context(self.device), spectrum, len(spectrum), ign)])[0]

    def par_deconvolute_spectrum(self, spectrum: Spectrum) -> Deconvolution:
        return self.deconvolute_spectrum(spectrum)

    def _ign_cache(self) -> np.ndarray:
        """_ignore_array(), kept while the regions are unchanged."""
        c = self.__dict__.get("_ign_c")
        if c is None or c[0] is not self._ignore:
            c = (self._ignore, self._ignore_array())
            self.__dict__["_ign_c"] = c
        return c[1]

    def deconvolute_spectra(self, spectra) -> list[Deconvolution]:
        spectra = list(spectra)
        if not spectra:
            return []
        return self._collect(self._run(spectra))

    def par_deconvolute_spectra(self, spectra) -> list[Deconvolution]:
        return self.deconvolute_spectra(spectra)

    def optimize_settings(self, reference: Spectrum) -> float:
        """Deconvoluter::optimize_settings (deconvoluter.rs:762-825): grid of 27
        smoothing x 10 noise-score x 3 analytical-fit settings on ``reference``;
        keeps the first setting of minimum MSE and returns that MSE. Runs as 27
        batched GPU pipelines (mdg_optimize_settings); near-ties of the batched
        MSE are settled with the reference's exact summation order."""
        if not isinstance(reference, Spectrum):
            raise TypeError("expected metabodecon.Spectrum")
        ign = self._ignore_array()
        ctx = nat.context(self.device)
        best = nat.Settings()
        mse = ctypes.c_double(0.0)
        sb0, sb1 = reference.signal_boundaries
        with ctx.lock:
            rc = nat.lib().mdg_optimize_settings(
                ctx.handle, nat.ptr(np.ascontiguousarray(reference.chemical_shifts)),
                nat.ptr(np.ascontiguousarray(reference.intensities)), len(reference), sb0, sb1,
                nat.ptr(ign) if ign.size else None, ign.size // 2, ctypes.byref(best),
                ctypes.byref(mse))
        if rc >= 100 or rc == nat.INVALID_ARGUMENT:
            raise exc.UnexpectedError(f"GPU engine failure: {nat.strerror(rc)}")
        if rc:
            raise exc.from_status(rc)
        self.set_moving_average_smoother(int(best.smooth_iterations), int(best.smooth_window))
        self.set_noise_score_selector(float(best.threshold))
        self.set_analytical_fitter(int(best.fit_iterations))
        return float(mse.value)
