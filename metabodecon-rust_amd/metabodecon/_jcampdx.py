"""JCAMP-DX reader (§8 row f4, host side, feeds the GPU path).

Restates spectrum/formats/jcampdx.rs of the reference:

* header (jcampdx.rs:404-436, :666-714): version 5.x/6.x, DATA TYPE ``NMR
  SPECTRUM``, DATA CLASS ``XYDATA``/``NTUPLES``, ``.OBSERVE FREQUENCY``,
  ``.OBSERVE NUCLEUS``, and the reference compound from ``.SHIFT REFERENCE``
  (method, name, 1-based index, shift) or else ``.SOLVENT NAME`` /
  ``.SOLVENT REFERENCE``;
* data blocks (jcampdx.rs:458-498, :726-884): XYDATA (``XUNITS``, ``YFACTOR``,
  ``FIRSTX``, ``LASTX``, ``NPOINTS``, ``XYDATA=(X++(Y..Y))``) and NTUPLES
  (per-column ``SYMBOL``/``VAR_DIM``/``UNITS``/``FIRST``/``LAST``/``FACTOR`` rows
  and the first ``DATA TABLE``);
* the axis (jcampdx.rs:566-577): ``step = (last - first) * conversion /
  (n - 1)``, ``offset = shift - index * step`` with a reference compound, else
  ``first * conversion``, ``x_i = offset + i * step``;
* the decoders (jcampdx.rs:892-1091): AFFN directly; anything containing an
  ASDF character goes through the reference's rewriting passes -- PAC/ASDF
  separation, SQZ digits, removal of the DIF y-checkpoints at line ends, then
  DIF and DUP rewrites repeated until neither pattern matches. This is the
  reference's own decoding (a DUP after a DIF repeats the decoded value, not
  the difference); results follow the reference, not the JCAMP-DX spec, where
  the two differ.

The regexes are the reference's, evaluated with Python's backtracking engine
(leftmost-first, the same match the Rust ``regex`` crate reports). Rust's
``str::lines``/``split_whitespace``/``trim`` and ``FromStr`` rules are
restated where Python's built-ins differ. Where the reference would panic on
malformed data (an unparsable DIF base value), this reader raises
``MalformedData`` instead.
"""
from __future__ import annotations

import os
import re

import numpy as np

# Rust char::is_whitespace (Unicode White_Space)
RUST_WS = _WS = ("\t\n\x0b\x0c\r \x85\xa0\u1680" + "".join(chr(c) for c in range(0x2000, 0x200B))
       + "\u2028\u2029\u202f\u205f\u3000")
_WS_RUN = re.compile("[" + re.escape(_WS) + "]+")
_RUST_F64 = re.compile(r"[+-]?(?:(?:[0-9]+\.?[0-9]*|\.[0-9]+)(?:[eE][+-]?[0-9]+)?|"
                       r"(?i:inf|infinity|nan))\Z")
_RUST_USIZE = re.compile(r"\+?[0-9]+\Z")
_RUST_I64 = re.compile(r"[+-]?[0-9]+\Z")
_U64 = 1 << 64


class JcampError(Exception):
    def __init__(self, kind: str, path: str, key: str = "", details: str = ""):
        self.kind, self.path, self.key = kind, path, key
        msg = f"{kind}: {path}"
        if key:
            msg += f" (key {key})"
        if details:
            msg += f": {details}"
        super().__init__(msg)


def rust_trim(s: str) -> str:
    return s.strip(_WS)


def rust_lines(s: str) -> list[str]:
    """str::lines: split on '\\n', strip one trailing '\\r', no final empty line."""
    if not s:
        return []
    parts = s.split("\n")
    if parts[-1] == "":
        parts.pop()
    return [p[:-1] if p.endswith("\r") else p for p in parts]


def rust_split_whitespace(s: str) -> list[str]:
    return [t for t in _WS_RUN.split(s) if t]


def _parse(kind: str, text: str):
    """<T as FromStr>::from_str for f64 / usize / String; ValueError on failure."""
    if kind == "f64":
        if not _RUST_F64.match(text):
            raise ValueError("invalid float literal")
        return float(text)
    if kind == "usize":
        if not _RUST_USIZE.match(text):
            raise ValueError("invalid digit found in string")
        v = int(text)
        if v >= _U64:
            raise ValueError("number too large to fit in target type")
        return v
    return text


def _capture(rx: re.Pattern, name: str, text: str, path: str, key: str, kind: str = "str"):
    """extract_capture.rs:8-44: first match, named group, parsed."""
    m = rx.search(text)
    if m is None or m.group(name) is None:
        raise JcampError("MissingMetadata", path, key)
    try:
        return _parse(kind, m.group(name))
    except ValueError as e:
        raise JcampError("MalformedMetadata", path, key, str(e)) from None


def _row(rx: re.Pattern, name: str, text: str, path: str, key: str, kind: str):
    """extract_capture.rs:49-81: comma separated row, every value trimmed and parsed."""
    raw = _capture(rx, name, text, path, key)
    try:
        return [_parse(kind, rust_trim(v)) for v in raw.split(",")]
    except ValueError as e:
        raise JcampError("MalformedMetadata", path, key, str(e)) from None


def _opt(fn, *a, **k):
    try:
        return fn(*a, **k)
    except JcampError:
        return None


# ---- jcampdx.rs:404-513 -------------------------------------------------------------
_M = re.M
HEADER_RE = [
    re.compile(r"^(##JCAMP(\s*|_|-)DX=\s*)(?P<version>\d+(\.\d+)?)", _M),
    re.compile(r"^(##DATA(\s|_)TYPE=\s*)(?P<type>\w+\s\w+)", _M),
    re.compile(r"^(##DATA(\s|_)CLASS=\s*)(?P<format>\w+(\s\w+)?)", _M),
    re.compile(r"^(##\.OBSERVE(\s|_)FREQUENCY=\s*)(?P<frequency>\d+(\.\d+)?)", _M),
    re.compile(r"^(##\.OBSERVE(\s|_)NUCLEUS=\s*)(?P<nucleus>\^\w+)", _M),
    re.compile(r"^(##\.SOLVENT(\s|_)NAME=\s*)(?P<name>.*)", _M),
    re.compile(r"^(##\.SOLVENT(\s|_)REFERENCE=\s*)(?P<shift>\d+(\.\d+))?", _M),
    re.compile(r"^(##\.SHIFT(\s|_)REFERENCE=\s*)(?P<method>[^,]*)", _M),
    re.compile(r"^(##\.SHIFT(\s|_)REFERENCE=[^,]*,\s*)(?P<name>[^,]*)", _M),
    re.compile(r"^(##\.SHIFT(\s|_)REFERENCE=[^,]*,[^,]*,\s*)(?P<index>\d+)", _M),
    re.compile(r"^(##\.SHIFT(\s|_)REFERENCE=[^,]*,[^,]*,[^,]*,\s*)(?P<shift>\d+(\.\d+)?)", _M),
]
HEADER_KEYS = ["JCAMPDX", "DATA_TYPE", "DATA_CLASS", ".OBSERVE FREQUENCY", ".OBSERVE NUCLEUS",
               ".SOLVENT NAME", ".SOLVENT REFERENCE", ".SHIFT REFERENCE [METHOD]",
               ".SHIFT REFERENCE [COMPOUND]", ".SHIFT REFERENCE [INDEX]",
               ".SHIFT REFERENCE [SHIFT]"]
XY_DATA_RE = [
    re.compile(r"^(##XUNITS=\s*)(?P<xunits>\w+)", _M),
    re.compile(r"^(##YFACTOR=\s*)(?P<factor>\d+(\.\d+)?)", _M),
    re.compile(r"^(##FIRSTX=\s*)(?P<first>\d+(\.\d+)?)", _M),
    re.compile(r"^(##LASTX=\s*)(?P<last>\d+(\.\d+)?)", _M),
    re.compile(r"^(##NPOINTS=\s*)(?P<data_size>\d+(\.\d+)?)", _M),
    re.compile(r"^(##XYDATA=\s*\(X\+\+\([RY]\.\.[RY]\)\)(.*)?)(?P<data>[^#$]*)", _M),
]
XY_DATA_KEYS = ["XUNITS", "YFACTOR", "FIRSTX", "LASTX", "NPOINTS", "XYDATA"]
N_TUPLES_RE = [
    re.compile(r"^(##SYMBOL=\s*)(?P<symbols>.*)(\r\n|\n|\r)", _M),
    re.compile(r"^(##VAR(\s*|_)DIM=\s*)(?P<data_sizes>.*)(\r\n|\n|\r)", _M),
    re.compile(r"^(##UNITS=\s*)(?P<units>.*)(\r\n|\n|\r)", _M),
    re.compile(r"^(##FIRST=\s*)(?P<first>.*)(\r\n|\n|\r)", _M),
    re.compile(r"^(##LAST=\s*)(?P<last>.*)(\r\n|\n|\r)", _M),
    re.compile(r"^(##FACTOR=\s*)(?P<factor>.*)(\r\n|\n|\r)", _M),
    re.compile(r"^(##DATA(\s|_)TABLE=\s*\(X\+\+\(([RY])\.\.[RY]\)\)(.*)?)(?P<data>[^#$]*)", _M),
]
N_TUPLES_KEYS = ["SYMBOL", "VAR DIM", "UNITS", "FIRST", "LAST", "FACTOR", "DATA TABLE"]
ENCODING = [
    re.compile(r"(?P<asdf>[@%A-Za-z+-])"),
    re.compile(r"(?P<pac>[+-]\d)"),
    re.compile(r"(?P<sqz>[@A-Ia-i])"),
    re.compile(r"\s+(?P<dif>[%J-Rj-r]\d*)\s*(?P<dup>([S-Zs]\d*)?)\s*((\r\n|\n|\r)\s*(?P<next>\d+))"),
    re.compile(r"\s+(?P<val>[+-]*\d*)\s+(?P<dif>[%J-Rj-r]\d*)"),
    re.compile(r"\s+(?P<val>[+-]*\d+)\s+(?P<dup>[S-Zs]\d*)"),
]

_SQZ = {c: str(i) for i, c in enumerate("@ABCDEFGHI")}
_SQZ.update({c: str(-(i + 1)) for i, c in enumerate("abcdefghi")})
_DIF = {c: str(i) for i, c in enumerate("%JKLMNOPQR")}
_DIF.update({c: str(-(i + 1)) for i, c in enumerate("jklmnopqr")})
_DUP = {c: str(i + 1) for i, c in enumerate("STUVWXYZs")}
_DUP_INV = {v: k for k, v in _DUP.items()}


# ---- header / blocks ----------------------------------------------------------------
def read_header(dx: str, path: str) -> dict:
    """jcampdx.rs:666-714."""
    re_, k = HEADER_RE, HEADER_KEYS
    version = _capture(re_[0], "version", dx, path, k[0], "f64")
    if int(version) not in (5, 6):
        raise JcampError("UnsupportedJcampDxFile", path)
    if _capture(re_[1], "type", dx, path, k[1]).upper() != "NMR SPECTRUM":
        raise JcampError("UnsupportedJcampDxFile", path)
    fmt = _capture(re_[2], "format", dx, path, k[2]).upper()
    if fmt not in ("XYDATA", "NTUPLES"):
        raise JcampError("UnsupportedJcampDxFile", path)
    frequency = _capture(re_[3], "frequency", dx, path, k[3], "f64")
    nucleus = _capture(re_[4], "nucleus", dx, path, k[4])
    method = _opt(_capture, re_[7], "method", dx, path, k[7])
    if method is not None:  # .parse::<ReferencingMethod>().ok()
        method = {"INTERNAL": "internal", "EXTERNAL": "external"}.get(rust_trim(method).upper())
    name = _opt(_capture, re_[8], "name", dx, path, k[8])
    index = _opt(_capture, re_[9], "index", dx, path, k[9], "usize")
    shift = _opt(_capture, re_[10], "shift", dx, path, k[10], "f64")
    if shift is not None and index is not None:
        # ReferenceCompound::new(shift, index - 1, ...): usize arithmetic wraps
        reference = {"chemical_shift": shift, "index": (index - 1) % _U64, "name": name,
                     "method": method}
    else:
        name = _opt(_capture, re_[5], "name", dx, path, k[5])
        shift = _opt(_capture, re_[6], "shift", dx, path, k[6], "f64")
        reference = (None if shift is None else
                     {"chemical_shift": shift, "index": 0, "name": name, "method": None})
    return {"format": fmt, "frequency": frequency, "nucleus": nucleus, "reference": reference}


def _x_units(u: str, path: str, key: str, ntuples: bool) -> str:
    u = u.upper()
    if u in ("HZ", "PPM"):
        return u
    if ntuples:
        raise JcampError("MalformedMetadata", path, key, f"Unsupported x unit: {u.lower()}")
    raise JcampError("UnsupportedJcampDxFile", path)


def read_xydata(dx: str, path: str) -> dict:
    """jcampdx.rs:726-762."""
    re_, k = XY_DATA_RE, XY_DATA_KEYS
    x_units = _x_units(_capture(re_[0], "xunits", dx, path, k[0]), path, k[0], False)
    factor = _capture(re_[1], "factor", dx, path, k[1], "f64")
    first = _capture(re_[2], "first", dx, path, k[2], "f64")
    last = _capture(re_[3], "last", dx, path, k[3], "f64")
    data_size = _capture(re_[4], "data_size", dx, path, k[4], "usize")
    data = rust_trim(_capture(re_[5], "data", dx, path, k[5]))
    if not data:
        raise JcampError("MissingData", path)
    return {"x_units": x_units, "factor": factor, "first": first, "last": last,
            "data_size": data_size, "data": data}


def read_ntuples(dx: str, path: str) -> dict:
    """jcampdx.rs:774-884."""
    re_, k = N_TUPLES_RE, N_TUPLES_KEYS
    symbols = [rust_trim(s) for s in _capture(re_[0], "symbols", dx, path, k[0]).split(",")]
    up = [s.upper() for s in symbols]
    if "X" not in up:
        raise JcampError("MissingMetadata", path, k[0])
    x_col = up.index("X")
    r_col = next((i for i, s in enumerate(up) if s in ("R", "Y")), None)
    if r_col is None:
        raise JcampError("MissingMetadata", path, k[0])

    def col(row, c, key, what):
        if c >= len(row):
            raise JcampError("MalformedMetadata", path, key, f"Could not find {what} column")
        return row[c]

    data_size = col(_row(re_[1], "data_sizes", dx, path, k[1], "usize"), x_col, k[1], "X")
    units = col(_row(re_[2], "units", dx, path, k[2], "str"), x_col, k[2], "X")
    x_units = _x_units(units, path, k[2], True)
    first = col(_row(re_[3], "first", dx, path, k[3], "f64"), x_col, k[3], "X")
    last = col(_row(re_[4], "last", dx, path, k[4], "f64"), x_col, k[4], "X")
    factor = col(_row(re_[5], "factor", dx, path, k[5], "f64"), r_col, k[5], "R")
    data = rust_trim(_capture(re_[6], "data", dx, path, k[6]))
    if not data:
        raise JcampError("MissingData", path)
    return {"x_units": x_units, "factor": factor, "first": first, "last": last,
            "data_size": data_size, "data": data}


# ---- decoders -----------------------------------------------------------------------
def decode_affn(data: str, factor: float, path: str) -> np.ndarray:
    """jcampdx.rs:892-916: every line minus its first (abscissa) token."""
    out = []
    for line in rust_lines(data):
        for v in rust_split_whitespace(line)[1:]:
            try:
                out.append(_parse("f64", v))
            except ValueError as e:
                raise JcampError("MalformedData", path, details=f"{v} ({e})") from None
    return np.array(out, dtype=np.float64) * factor


def _dup_count(encoded: str) -> int:
    return int(_DUP[encoded[0]] + encoded[1:])


def decrement_dup(encoded: str) -> str:
    """jcampdx.rs:1055-1091."""
    dec = str(_dup_count(encoded) - 1)
    return ("" if dec[0] == "0" else _DUP_INV[dec[0]]) + dec[1:]


def _undo_dif(value: str, encoded: str, path: str) -> str:
    """jcampdx.rs:1020-1049: ' value value+difference'."""
    if not _RUST_I64.match(value):
        raise JcampError("MalformedData", path, details=f"DIF base value {value!r}")
    v = int(value)
    return f" {v} {v + int(_DIF[encoded[0]] + encoded[1:])}"


def decode_asdf(data: str, factor: float, path: str) -> np.ndarray:
    """jcampdx.rs:925-966."""
    re_ = ENCODING
    data = re_[0].sub(r" \g<asdf>", data)
    data = re_[1].sub(r" \g<pac>", data)
    data = re_[2].sub(lambda m: _SQZ[m.group("sqz")], data)

    def checkpoint(m):
        dif, dup, nxt = m.group("dif"), m.group("dup"), m.group("next")
        if dup in ("", "S"):
            return f" \n{nxt}"
        return f" {dif} {decrement_dup(dup)} \n{nxt}"

    data = re_[3].sub(checkpoint, data)
    while True:
        data = re_[4].sub(lambda m: _undo_dif(m.group("val"), m.group("dif"), path), data)
        data = re_[5].sub(lambda m: f" {m.group('val')}" * _dup_count(m.group("dup")), data)
        if not re_[4].search(data) and not re_[5].search(data):
            break
    return decode_affn(data, factor, path)


# ---- jcampdx.rs:555-656 -------------------------------------------------------------
def read_jcampdx_arrays(path: str):
    """Returns (chemical_shifts, intensities, header) of one file."""
    path = os.fspath(path)
    with open(path, "r", encoding="utf-8", newline="") as f:
        dx = f.read()
    header = read_header(dx, path)
    block = read_xydata(dx, path) if header["format"] == "XYDATA" else read_ntuples(dx, path)
    conversion = 1.0 / header["frequency"] if block["x_units"] == "HZ" else 1.0
    n = block["data_size"]
    step = (block["last"] - block["first"]) * conversion / (float(n) - 1.0)
    ref = header["reference"]
    if ref is not None:
        offset = ref["chemical_shift"] - float(ref["index"]) * step
    else:
        offset = block["first"] * conversion
    # (i as f64) * step, then offset + that: two roundings, as the reference
    chemical_shifts = offset + np.arange(n, dtype=np.float64) * step
    intensities = decode_native(block["data"], block["factor"], n)
    if intensities is None:  # left to the regex restatement (non-ASCII, or an error)
        if ENCODING[0].search(block["data"]):
            intensities = decode_asdf(block["data"], block["factor"], path)
        else:
            intensities = decode_affn(block["data"], block["factor"], path)
    return chemical_shifts, intensities, header


def decode_native(data: str, factor: float, hint: int) -> np.ndarray | None:
    """The block through the engine library's decoder (mdg_jcampdx_decode: the same
    passes in C++, ~100x faster than the regex passes); None for the blocks it leaves
    to decode_asdf / decode_affn (non-ASCII text, data the reference rejects), and
    when the engine library is missing or stale (reading a file needs no GPU: the regex
    restatement then decodes it)."""
    from . import _native as nat
    import ctypes
    if not data.isascii():
        return None
    raw = data.encode("ascii")
    try:
        L = nat.lib()
    except (nat.NativeLibraryError, OSError):
        return None
    n = ctypes.c_size_t(0)
    cap = max(1, int(hint))
    for _ in range(2):
        out = np.empty(cap, dtype=np.float64)
        st = L.mdg_jcampdx_decode(raw, len(raw), float(factor), nat.ptr(out), cap, ctypes.byref(n))
        if st == 0:
            return out[: n.value]
        if st != nat.CAPACITY:
            return None
        cap = n.value
    return None


def jcampdx_set_paths(path: str) -> list[str]:
    """jcampdx.rs:633-656 keeps the entries whose extension is ``dx`` (any case)
    in ``read_dir`` order; sorted here so results are reproducible across file
    systems (as the Bruker set reader)."""
    out = []
    for e in os.listdir(path):
        stem, ext = os.path.splitext(e)
        if ext[1:].lower() == "dx" and stem:
            out.append(os.path.join(path, e))
    return sorted(out)
