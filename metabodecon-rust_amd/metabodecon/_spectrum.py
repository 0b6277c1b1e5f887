"""Python ``Spectrum`` mirroring metabodecon-python/src/bindings/spectrum.rs:29-232.

Construction enforces the invariants of spectrum/spectrum.rs:120-150 and
:779-890 (lengths, uniform spacing, finite intensities, boundaries ordered per
monotonicity and inside the axis), so every spectrum handed to the GPU engine
is one the reference would also accept. Metadata follows spectrum/meta/
(nucleus.rs, reference.rs): the nucleus is normalised through ``Nucleus::from``
and shown with its ``Display`` string; the reference compound is validated as
the binding's setter does (bindings/spectrum.rs:155-191). Serialisation is the
reference's ``SerializedSpectrum`` (serialized_spectrum.rs:7-55) through
``_serde``.
"""
from __future__ import annotations

import math
import operator

import numpy as np

from . import _native
from . import _serde as serde
from . import exceptions as exc
from ._bruker import MetadataError, bruker_set_paths, read_bruker_arrays
from ._jcampdx import RUST_WS, JcampError, jcampdx_set_paths, read_jcampdx_arrays

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


# spectrum/meta/nucleus.rs:20-73: accepted spellings -> Display string
_NUCLEI = {
    "1H": "1H", "PROTON": "1H", "HYDROGEN1": "1H",
    "11B": "11B", "BORON11": "11B",
    "13C": "13C", "CARBON13": "13C",
    "15N": "15N", "NITROGEN15": "15N",
    "19F": "19F", "FLUORINE19": "19F",
    "29SI": "29Si", "SILICON29": "29Si",
    "31P": "31P", "PHOSPHORUS31": "31P",
}
_RUST_WS = RUST_WS  # char::is_whitespace, for str::trim


def nucleus_display(value: str) -> str:
    """``Nucleus::from(value).to_string()`` (nucleus.rs:22-46, :57-72)."""
    key = value.strip(_RUST_WS)
    for ch in " ^-_":
        key = key.replace(ch, "")
    return _NUCLEI.get(key.upper(), value)


def referencing_method(value: str) -> str | None:
    """``ReferencingMethod::from_str`` (reference.rs:15-35) as its Display string."""
    return {"INTERNAL": "internal", "EXTERNAL": "external"}.get(value.strip(_RUST_WS).upper())


def _extract_f64(v, what: str) -> float:
    # pyo3 f64 extraction: floats and ints (anything with __float__/__index__), not str
    if isinstance(v, (str, bytes)):
        raise TypeError(f"'{type(v).__name__}' object cannot be converted to 'PyFloat' ({what})")
    return float(v)


def _extract_usize(v, what: str) -> int:
    i = operator.index(v)  # TypeError for floats / str, as pyo3
    if i < 0:
        raise OverflowError(f"can't convert negative int to unsigned ({what})")
    if i >= 1 << 64:
        raise OverflowError(f"int too big to convert ({what})")
    return i


def _validate_boundaries(sb, cs: np.ndarray, mono: str) -> tuple[float, float]:
    """validate_boundaries (spectrum.rs:840-890): ordered per monotonicity, inside the axis."""
    sb = (float(sb[0]), float(sb[1]))
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
    return sb


class Spectrum:
    def __init__(self, chemical_shifts, intensities, signal_boundaries):
        # the spectrum's own rows, page-locked when the engine can give such memory:
        # the host-buffer calls then DMA straight from them (mdg_host_alloc)
        self._init(_native.pinned_copy(chemical_shifts), _native.pinned_copy(intensities),
                   signal_boundaries)

    @classmethod
    def _adopt(cls, cs: np.ndarray, it: np.ndarray, signal_boundaries) -> "Spectrum":
        """A Spectrum that takes `cs` / `it` as its own rows (fresh f64 arrays the
        caller gives up), validated like the constructor; no copy."""
        s = cls.__new__(cls)
        s._init(cs, it, signal_boundaries)
        return s

    def _set_raw(self, row: np.ndarray, scale: float, axis: tuple) -> None:
        """The compact form the Bruker reader built the rows from: intensities =
        row * scale, chemical shifts = axis[0] - (i * axis[1]) / axis[2] (bruker.rs:
        278-280, :459-470). The host-buffer calls send it instead of the f64 rows."""
        row.setflags(write=False)
        self._raw = (row, float(scale), tuple(float(v) for v in axis))

    def _init(self, cs: np.ndarray, it: np.ndarray, signal_boundaries) -> None:
        self._raw = None
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
        sb = _validate_boundaries(signal_boundaries, cs, mono)
        cs.setflags(write=False)
        it.setflags(write=False)
        self._cs = cs
        self._it = it
        self._sb = sb
        self._mono = mono
        # defaults of Spectrum::new (spectrum.rs:140-150): 1H, 1.0, (x_0, index 0)
        self._nucleus = "1H"
        self._frequency = 1.0
        self._reference = (float(cs[0]), 0, None, None)

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

    @signal_boundaries.setter
    def signal_boundaries(self, signal_boundaries) -> None:
        # bindings/spectrum.rs:134-143 -> Spectrum::set_signal_boundaries
        self._sb = _validate_boundaries(signal_boundaries, self._cs, self._mono)

    @property
    def nucleus(self) -> str:
        return self._nucleus

    @nucleus.setter
    def nucleus(self, nucleus: str) -> None:
        if not isinstance(nucleus, str):
            raise TypeError(f"'{type(nucleus).__name__}' object cannot be converted to 'PyString'")
        self._nucleus = nucleus_display(nucleus)

    @property
    def frequency(self) -> float:
        return self._frequency

    @frequency.setter
    def frequency(self, frequency: float) -> None:
        self._frequency = _extract_f64(frequency, "frequency")

    @property
    def reference_compound(self) -> dict:
        cs, index, name, method = self._reference
        return {"chemical_shift": cs, "index": index, "name": name, "method": method}

    @reference_compound.setter
    def reference_compound(self, reference: dict) -> None:
        # bindings/spectrum.rs:155-191
        if not isinstance(reference, dict):
            raise TypeError(f"'{type(reference).__name__}' object cannot be converted to 'PyDict'")
        cs = _extract_f64(reference["chemical_shift"], "chemical_shift")
        index = _extract_usize(reference["index"], "index")
        name = reference.get("name")
        if name is not None and not isinstance(name, str):
            raise TypeError("reference compound name must be a string")
        method = reference.get("method")
        if method is not None:
            if not isinstance(method, str):
                raise TypeError("referencing method must be a string")
            parsed = referencing_method(method)
            if parsed is None:
                raise ValueError("referencing method must be either 'external' or 'internal'")
            method = parsed
        self._reference = (cs, index, name, method)

    def range(self) -> tuple[float, float]:
        """(first, last) chemical shift (spectrum.rs:633-635)."""
        return (float(self._cs[0]), float(self._cs[-1]))

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
        raw = meta.get("raw")
        if raw is not None:  # the GPU reads the compact rows: x / y stay ordinary memory
            s = Spectrum._adopt(np.asarray(cs, dtype=np.float64), np.asarray(it, dtype=np.float64),
                                signal_boundaries)
            row = _native.pinned_empty(raw[0].shape, np.int32)
            if row is None:
                row = np.array(raw[0], dtype=np.int32)
            else:
                row[...] = raw[0]
            s._set_raw(row, raw[1], raw[2])
        else:
            s = Spectrum(cs, it, signal_boundaries)
        s.nucleus = meta["nucleus"]
        s.frequency = meta["frequency"]
        return s

    @staticmethod
    def read_bruker_set(path: str, experiment: int, processing: int,
                        signal_boundaries) -> list["Spectrum"]:
        # the files are read by a few threads at once (the reads and the int32
        # decode release the GIL); the first error in directory order is raised,
        # as the reference's sequential collect does (bruker.rs:300-321)
        paths = bruker_set_paths(path)

        def one(p):
            try:
                return read_bruker_arrays(p, experiment, processing)
            except Exception as e:  # noqa: BLE001 -- raised below, in directory order
                return e
        if len(paths) > 1:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(max_workers=min(8, len(paths))) as pool:
                arrays = list(pool.map(one, paths))
        else:
            arrays = [one(p) for p in paths]
        # The reference reads and validates one spectrum at a time (read_spectrum, then
        # Spectrum::new, then the next directory: bruker.rs:360-373), so the first
        # failure in directory order wins, whether a read error or a validation error:
        # the spectra before the first failed read are validated first.
        bad = next((i for i, a in enumerate(arrays) if isinstance(a, BaseException)), None)
        if bad is not None:
            _set_of_rows(arrays[:bad], signal_boundaries)  # raises an earlier validation error
            e = arrays[bad]
            if isinstance(e, MetadataError):
                raise getattr(exc, e.kind, exc.SpectrumError)(str(e)) from None
            raise e
        return _set_of_rows(arrays, signal_boundaries)


    @staticmethod
    def read_jcampdx(path: str, signal_boundaries) -> "Spectrum":
        """bindings/spectrum.rs:69-75 -> JcampDx::read_spectrum (jcampdx.rs:555-590)."""
        try:
            cs, it, header = read_jcampdx_arrays(path)
        except JcampError as e:
            if e.kind == "UnsupportedJcampDxFile":  # not mapped by error.rs
                raise exc.UnexpectedError(f"unexpected error: {e}") from None
            raise getattr(exc, e.kind, exc.SpectrumError)(str(e)) from None
        except UnicodeDecodeError as e:  # read_to_string -> io::Error -> PyIOError
            raise OSError(f"stream did not contain valid UTF-8: {path}") from e
        s = Spectrum(cs, it, signal_boundaries)
        s.nucleus = header["nucleus"]
        s.frequency = header["frequency"]
        ref = header["reference"]
        if ref is not None:
            s._reference = (ref["chemical_shift"], ref["index"], ref["name"], ref["method"])
        return s

    @staticmethod
    def read_jcampdx_set(path: str, signal_boundaries) -> list["Spectrum"]:
        return [Spectrum.read_jcampdx(p, signal_boundaries) for p in jcampdx_set_paths(path)]

    # ---- serialisation (bindings/spectrum.rs:193-232, serialized_spectrum.rs) --------
    def _serialized(self, as_array: bool):
        cs, index, name, method = self._reference
        if as_array:  # rmp_serde: structs as arrays, skipped Options omitted
            ref = [cs, index] + ([name] if name is not None else []) \
                + ([method] if method is not None else [])
            return [list(self.range()), list(self._sb), int(self._cs.size), self._nucleus,
                    self._frequency, ref, self._it.tolist()]
        ref = {"chemicalShift": cs, "index": index}
        if name is not None:
            ref["name"] = name
        if method is not None:
            ref["method"] = method
        return {"spectrumBoundaries": list(self.range()), "signalBoundaries": list(self._sb),
                "size": int(self._cs.size), "nucleus": self._nucleus,
                "frequency": self._frequency, "referenceCompound": ref,
                "intensities": self._it.tolist()}

    @staticmethod
    def _from_serialized(v) -> "Spectrum":
        d = serde.fields(v, ("spectrumBoundaries", "signalBoundaries", "size", "nucleus",
                             "frequency", "referenceCompound", "intensities"), "Spectrum")

        def pair(x, what):
            if not isinstance(x, list) or len(x) != 2:
                raise serde.SerdeError(f"invalid value for {what}: expected a tuple of size 2")
            return (serde.f64(x[0], what), serde.f64(x[1], what))

        start, end = pair(d["spectrumBoundaries"], "spectrumBoundaries")
        sb = pair(d["signalBoundaries"], "signalBoundaries")
        size = serde.usize(d["size"], "size")
        nucleus = serde.string(d["nucleus"], "nucleus")
        frequency = serde.f64(d["frequency"], "frequency")
        r = serde.fields(d["referenceCompound"], ("chemicalShift", "index", "name", "method"),
                         "ReferenceCompound", optional=("name", "method"))
        ref_cs = serde.f64(r["chemicalShift"], "chemicalShift")
        ref_index = serde.usize(r["index"], "index")
        name = None if r["name"] is None else serde.string(r["name"], "name")
        method = None
        if r["method"] is not None:
            method = serde.string(r["method"], "method")
            if method not in ("internal", "external"):  # rename_all = "camelCase"
                raise serde.SerdeError(f"unknown variant `{method}`, expected `internal` or "
                                       "`external`")
        if not isinstance(d["intensities"], list):
            raise serde.SerdeError("invalid type for intensities: expected a sequence")
        it = [serde.f64(x, "intensities") for x in d["intensities"]]
        # TryFrom<SerializedSpectrum> (serialized_spectrum.rs:35-55)
        step = (end - start) / (float(size) - 1.0)
        cs = start + np.arange(size, dtype=np.float64) * step
        try:
            s = Spectrum(cs, it, sb)
        except exc.SpectrumError as e:
            raise serde.SerdeError(str(e)) from None
        s._nucleus = nucleus_display(nucleus)
        s._frequency = frequency
        s._reference = (ref_cs, ref_index, name, method)
        return s

    def write_json(self, path: str) -> None:
        text = serde.to_string_pretty(self._serialized(as_array=False))
        with open(path, "wb") as f:
            f.write(text.encode("utf-8"))

    @staticmethod
    def read_json(path: str) -> "Spectrum":
        with open(path, "rb") as f:
            raw = f.read()
        try:
            text = raw.decode("utf-8")
        except UnicodeDecodeError as e:
            raise OSError("stream did not contain valid UTF-8") from e
        try:
            return Spectrum._from_serialized(serde.from_str(text))
        except serde.SerdeError as e:
            raise serde.serialization_error(e) from None

    def write_bin(self, path: str) -> None:
        with open(path, "wb") as f:
            f.write(serde.to_msgpack(self._serialized(as_array=True)))

    @staticmethod
    def read_bin(path: str) -> "Spectrum":
        with open(path, "rb") as f:
            raw = f.read()
        try:
            return Spectrum._from_serialized(serde.from_msgpack(raw))
        except serde.SerdeError as e:
            raise serde.serialization_error(e) from None

    def __repr__(self) -> str:
        return (f"Spectrum(n={self._cs.size}, range=({self._cs[0]}, {self._cs[-1]}), "
                f"signal_boundaries={self._sb})")


def _set_of_rows(arrays, signal_boundaries) -> list[Spectrum]:
    """Spectra of a set read together ((chemical shifts, intensities, meta) each),
    their rows laid out in one page-locked block per length, so consecutive spectra
    of a batch are adjacent rows and travel in one DMA (mdg_deconvolute_rows[_i32]):
    the int32 sample rows of Bruker data [r_0 .. r_k-1] (the f64 rows then stay
    ordinary memory), else [x_0 .. x_k-1][y_0 .. y_k-1]. Ordinary copies without
    the engine's memory."""
    by_n: dict[tuple, list[int]] = {}
    for i, (cs, it, meta) in enumerate(arrays):
        if cs.ndim == 1 and cs.size == it.size and cs.size > 0:
            by_n.setdefault((cs.size, meta.get("raw") is not None), []).append(i)
    rows: dict[int, tuple] = {}  # spectrum -> its rows in a shared block
    for (n, compact), idx in by_n.items():
        if len(idx) < 2:
            continue
        blk = _native.pinned_empty((len(idx), n), np.int32) if compact else \
            _native.pinned_empty((2, len(idx), n))
        if blk is not None:
            for r, i in enumerate(idx):
                rows[i] = (blk[r],) if compact else (blk[0, r], blk[1, r])
    out = []
    for i, (cs, it, meta) in enumerate(arrays):  # in order: the first error is raised
        raw = meta.get("raw")
        if raw is not None:
            s = Spectrum._adopt(np.asarray(cs, dtype=np.float64), np.asarray(it, dtype=np.float64),
                                signal_boundaries)
            if i in rows:
                row = rows[i][0]
                row[...] = raw[0]
            else:
                row = _native.pinned_empty(raw[0].shape, np.int32)
                if row is None:
                    row = np.array(raw[0], dtype=np.int32)
                else:
                    row[...] = raw[0]
            s._set_raw(row, raw[1], raw[2])
        elif i in rows:
            xr, yr = rows[i]
            xr[...] = cs
            yr[...] = it
            s = Spectrum._adopt(xr, yr, signal_boundaries)
        else:
            s = Spectrum(cs, it, signal_boundaries)
        s.nucleus = meta["nucleus"]
        s.frequency = meta["frequency"]
        out.append(s)
    return out
