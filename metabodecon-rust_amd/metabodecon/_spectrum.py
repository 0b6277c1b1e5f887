"""Python ``Spectrum`` mirroring metabodecon-python/src/bindings/spectrum.rs:29-232.

Construction enforces the invariants of spectrum/spectrum.rs:120-150 and
:779-890 (lengths, uniform spacing, finite intensities, boundaries ordered per
monotonicity and inside the axis), so every spectrum handed to the GPU engine
is one the reference would also accept.
"""
from __future__ import annotations

import math

import numpy as np

from . import exceptions as exc
from ._bruker import MetadataError, bruker_set_paths, read_bruker_arrays

CHECK_PRECISION = 1.0e3 * 2.220446049250313e-16  # lib.rs:277


def _monotonicity(first: float, second: float) -> str | None:
    # spectrum/meta/monotonicity.rs:29-38
    d = first - second
    if abs(d) < CHECK_PRECISION or not math.isfinite(d):
        return None
    if first < second:
        return "increasing"
    if first > second:
        return "decreasing"
    return None


class Spectrum:
    def __init__(self, chemical_shifts, intensities, signal_boundaries):
        cs = np.array(chemical_shifts, dtype=np.float64, copy=True).reshape(-1)
        it = np.array(intensities, dtype=np.float64, copy=True).reshape(-1)
        # validate_lengths (spectrum.rs:779-799)
        if cs.size == 0 or it.size == 0:
            raise exc.EmptyData(
                f"input data is empty: chemical shifts {cs.size}, intensities {it.size}")
        if cs.size != it.size:
            raise exc.DataLengthMismatch(
                f"input lengths differ: chemical shifts {cs.size}, intensities {it.size}")
        if cs.size < 2:
            raise exc.NonUniformSpacing("at least two chemical shifts are required")
        # validate_spacing (spectrum.rs:801-822)
        step = cs[1] - cs[0]
        if abs(step) < CHECK_PRECISION:
            raise exc.NonUniformSpacing(f"step size {step} at positions (0, 1)")
        diffs = cs[1:] - cs[:-1]
        bad = np.nonzero((np.abs(diffs - step) > CHECK_PRECISION) | ~np.isfinite(diffs))[0]
        if bad.size:
            p = int(bad[0])
            raise exc.NonUniformSpacing(f"step size {step} at positions ({p}, {p + 1})")
        # validate_intensities (spectrum.rs:824-838)
        nonfinite = np.nonzero(~np.isfinite(it))[0]
        if nonfinite.size:
            raise exc.InvalidIntensities(f"non-finite intensities at {nonfinite[:10].tolist()}")
        mono = _monotonicity(float(cs[0]), float(cs[1]))
        if mono is None:  # pragma: no cover - excluded by validate_spacing
            raise exc.NonUniformSpacing("chemical shifts are not monotonic")
        # validate_boundaries (spectrum.rs:840-890)
        sb = (float(signal_boundaries[0]), float(signal_boundaries[1]))
        width = sb[0] - sb[1]
        rng = (float(cs[0]), float(cs[-1]))
        if abs(width) < CHECK_PRECISION or not math.isfinite(width):
            raise exc.InvalidSignalBoundaries(f"signal boundaries {sb} invalid for range {rng}")
        if mono == "increasing":
            sb = (min(sb), max(sb))
            if sb[0] < rng[0] or sb[1] > rng[1]:
                raise exc.InvalidSignalBoundaries(f"signal boundaries {sb} outside range {rng}")
        else:
            sb = (max(sb), min(sb))
            if sb[0] > rng[0] or sb[1] < rng[1]:
                raise exc.InvalidSignalBoundaries(f"signal boundaries {sb} outside range {rng}")
        cs.setflags(write=False)
        it.setflags(write=False)
        self._cs = cs
        self._it = it
        self._sb = sb
        self._mono = mono
        self.nucleus = "1H"
        self.frequency = 1.0
        self.reference_compound = {"chemical_shift": float(cs[0]), "index": 0, "name": None,
                                   "method": None}

    # ---- accessors (spectrum.rs:225-260, :633-635, :741-746) ------------------------
    @property
    def chemical_shifts(self) -> np.ndarray:
        return self._cs

    @property
    def intensities(self) -> np.ndarray:
        return self._it

    @property
    def signal_boundaries(self) -> tuple[float, float]:
        return self._sb

    @property
    def monotonicity(self) -> str:
        return self._mono

    def __len__(self) -> int:
        return int(self._cs.size)

    def step(self) -> float:
        return float(self._cs[1] - self._cs[0])

    def signal_boundaries_indices(self) -> tuple[int, int]:
        def as_usize(v):
            return 0 if not (v > 0.0) else int(v)
        st = self.step()
        x0 = float(self._cs[0])
        return (as_usize(math.floor((self._sb[0] - x0) / st)),
                as_usize(math.ceil((self._sb[1] - x0) / st)))

    # ---- readers (bindings/spectrum.rs:90-120) ----------------------------------------
    @staticmethod
    def read_bruker(path: str, experiment: int, processing: int,
                    signal_boundaries) -> "Spectrum":
        try:
            cs, it, meta = read_bruker_arrays(path, experiment, processing)
        except MetadataError as e:
            raise getattr(exc, e.kind, exc.SpectrumError)(str(e)) from None
        s = Spectrum(cs, it, signal_boundaries)
        s.nucleus = meta["nucleus"]
        s.frequency = meta["frequency"]
        return s

    @staticmethod
    def read_bruker_set(path: str, experiment: int, processing: int,
                        signal_boundaries) -> list["Spectrum"]:
        return [Spectrum.read_bruker(p, experiment, processing, signal_boundaries)
                for p in bruker_set_paths(path)]

    def __repr__(self) -> str:
        return (f"Spectrum(n={self._cs.size}, range=({self._cs[0]}, {self._cs[-1]}), "
                f"signal_boundaries={self._sb})")
