"""Bruker TopSpin reader (host side, feeds the GPU path).

Restates spectrum/formats/bruker.rs:260-490 of the reference: the same header
regexes (``##$SW``, ``##$SFO1``, ``##$NUC1`` in ``acqus``; ``##$OFFSET``,
``##$NC_proc``, ``##$BYTORDP``, ``##$DTYPP``, ``##$SI`` in ``procs``), the
axis ``maximum - (i * width) / (SI - 1)`` evaluated in that operation order
(bruker.rs:278-280), and ``1r`` decoded as int32 (scaled by ``2^NC_proc``) or
f64, little/big endian (bruker.rs:459-489). The data is NOT reversed, exactly
as the reference code (its doc comment says otherwise).
"""
from __future__ import annotations

import os
import re

import numpy as np

_ACQUS = {
    "width": (re.compile(r"^(##\$SW=\s*)(?P<v>\d+(\.\d+)?)", re.M), "SW", float),
    "frequency": (re.compile(r"^(##\$SFO1=\s*)(?P<v>\d+(\.\d+)?)", re.M), "SFO1", float),
    "nucleus": (re.compile(r"^(##\$NUC1=\s*<)(?P<v>\w+)", re.M), "NUC1", str),
}
_PROCS = {
    "maximum": (re.compile(r"^(##\$OFFSET=\s*)(?P<v>\d+(\.\d+)?)", re.M), "OFFSET", float),
    "exponent": (re.compile(r"^(##\$NC_proc=\s*)(?P<v>-?\d+)", re.M), "NC_proc", int),
    "endian": (re.compile(r"^(##\$BYTORDP=\s*)(?P<v>\d)", re.M), "BYTORDP", int),
    "data_type": (re.compile(r"^(##\$DTYPP=\s*)(?P<v>\d)", re.M), "DTYPP", int),
    "data_size": (re.compile(r"^(##\$SI=\s*)(?P<v>\d+)", re.M), "SI", int),
}


class MetadataError(Exception):
    def __init__(self, kind: str, path: str, key: str, details: str = ""):
        self.kind, self.path, self.key = kind, path, key
        super().__init__(f"{kind}: key {key} in {path} {details}".strip())


def _extract(spec: dict, text: str, path: str) -> dict:
    out = {}
    for name, (rx, key, conv) in spec.items():
        m = rx.search(text)
        if m is None:
            raise MetadataError("MissingMetadata", path, key)
        try:
            out[name] = conv(m.group("v"))
        except ValueError as e:  # pragma: no cover - regex already constrains
            raise MetadataError("MalformedMetadata", path, key, str(e))
    return out


def read_bruker_arrays(path: str, experiment: int, processing: int):
    """Returns (chemical_shifts f64[SI], intensities f64[SI], meta dict)."""
    acqus_path = os.path.join(path, f"{experiment}", "acqus")
    procs_path = os.path.join(path, f"{experiment}", "pdata", f"{processing}", "procs")
    one_r_path = os.path.join(path, f"{experiment}", "pdata", f"{processing}", "1r")
    with open(acqus_path, "r", errors="replace") as f:
        acqus = _extract(_ACQUS, f.read(), acqus_path)
    with open(procs_path, "r", errors="replace") as f:
        procs = _extract(_PROCS, f.read(), procs_path)
    si = procs["data_size"]
    i = np.arange(si, dtype=np.float64)
    # bruker.rs:278-280: maximum - (i as f64) * width / (SI as f64 - 1.0)
    chemical_shifts = procs["maximum"] - (i * acqus["width"]) / (float(si) - 1.0)
    endian = "<" if procs["endian"] == 0 else ">"
    if procs["data_type"] == 0:
        raw = np.fromfile(one_r_path, dtype=np.dtype(endian + "i4"), count=si)
        if raw.size != si:
            raise MetadataError("MissingData", one_r_path, "1r")
        intensities = raw.astype(np.float64) * float(2.0 ** procs["exponent"])
    else:
        raw = np.fromfile(one_r_path, dtype=np.dtype(endian + "f8"), count=si)
        if raw.size != si:
            raise MetadataError("MissingData", one_r_path, "1r")
        intensities = raw.astype(np.float64)
    meta = {"nucleus": acqus["nucleus"], "frequency": acqus["frequency"]}
    if procs["data_type"] == 0:
        # the compact form the rows were built from (mdg_deconvolute_rows_i32 decodes
        # it on the device bit for bit): int32 samples, their power-of-two scale, and
        # the axis operands (maximum, width, SI - 1) of the formula above
        meta["raw"] = (raw.astype(np.int32, copy=False), float(2.0 ** procs["exponent"]),
                       (float(procs["maximum"]), float(acqus["width"]), float(si) - 1.0))
    return chemical_shifts, intensities, meta


def bruker_set_paths(path: str) -> list[str]:
    """bruker.rs:300-321 iterates ``read_dir`` (directory order); we sort by name
    so results are reproducible across file systems."""
    return sorted(
        os.path.join(path, e) for e in os.listdir(path) if os.path.isdir(os.path.join(path, e))
    )
