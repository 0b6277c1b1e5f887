"""Reference-compatible serialisation (§8 row f3, host side).

The reference Python bindings write JSON with ``serde_json::to_string_pretty``
and MessagePack with ``rmp_serde::to_vec`` (metabodecon-python/src/bindings/
spectrum.rs:194-232, deconvolution.rs:77-116; serde_json 1.0.140, rmp-serde
1.3.0, Cargo.toml:35-37). This module reproduces both encodings byte for byte
and both decoders value for value, so files move freely between this framework
and the reference:

* JSON writer -- serde_json's ``PrettyFormatter`` (two-space indent, ``": "``,
  empty containers as ``[]``/``{}``, no trailing newline), strings escaped like
  serde_json's ``ESCAPE`` table, floats in ryu's shortest round-trip layout
  (``1.0``, ``0.001234``, ``1e-7``, ``1.234e33``), non-finite floats as ``null``.
* JSON reader -- serde_json WITHOUT the ``float_roundtrip`` feature (the
  reference does not enable it): a decimal literal is read as a u64 significand
  (digits past u64 overflow dropped) times an exact power of ten, i.e.
  ``significand as f64`` then one multiply/divide by ``POW10[|e|]``. That is
  not always correctly rounded, so reading with Python's ``float()`` would give
  different bits than the reference for some 17-digit values.
* MessagePack -- rmp_serde's default config: structs as arrays in field order,
  ``skip_serializing_if`` fields omitted (so later fields shift left, exactly as
  the reference), internally tagged enums as ``[tag, fields...]``, unit
  variants of plain enums as their (renamed) name, f64 always as ``0xcb``,
  integers in the smallest unsigned form. The decoder accepts arrays or maps,
  as rmp_serde's ``deserialize_struct`` does.

No fixture of either format ships with the reference, so the byte layouts are
"parity unpinned"; the tests pin them structurally (tests/test_formats.py).
"""
from __future__ import annotations

import json
import math
import re

import msgpack

from . import exceptions as exc

__all__ = ["ryu_f64", "to_string_pretty", "from_str", "to_msgpack", "from_msgpack",
           "SerdeError"]


class SerdeError(ValueError):
    """Deserialisation failed (mapped to ``exceptions.SerializationError``)."""


# =====================================================================================
# ryu layout of a finite f64 (ryu 1.x pretty::format64)
# =====================================================================================
def ryu_f64(v: float) -> str:
    if v == 0.0:
        return "-0.0" if math.copysign(1.0, v) < 0 else "0.0"
    # Python's repr is the shortest round-trip digit string (correctly rounded,
    # closest to the exact value), the same digits ryu produces.
    r = repr(abs(v))
    mant, _, e = r.partition("e")
    exp = int(e) if e else 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    if fp == "0":
        fp = ""
    digits = (ip + fp).lstrip("0")
    exp -= len(fp)
    stripped = digits.rstrip("0")
    exp += len(digits) - len(stripped)
    digits = stripped
    length = len(digits)
    kk = length + exp          # 10^(kk-1) <= v < 10^kk
    sign = "-" if v < 0 else ""
    if 0 <= exp and kk <= 16:
        out = digits + "0" * (kk - length) + ".0"
    elif 0 < kk <= 16:
        out = digits[:kk] + "." + digits[kk:]
    elif -5 < kk <= 0:
        out = "0." + "0" * (-kk) + digits
    elif length == 1:
        out = digits + "e" + str(kk - 1)
    else:
        out = digits[0] + "." + digits[1:] + "e" + str(kk - 1)
    return sign + out


# =====================================================================================
# serde_json::to_string_pretty
# =====================================================================================
_ESC = {'"': '\\"', "\\": "\\\\", "\b": "\\b", "\t": "\\t", "\n": "\\n", "\f": "\\f",
        "\r": "\\r"}
_NEEDS_ESC = re.compile(r'["\\\x00-\x1f]')


def _json_str(s: str) -> str:
    return '"' + _NEEDS_ESC.sub(lambda m: _ESC.get(m.group(0), "\\u%04x" % ord(m.group(0))),
                                s) + '"'


def _pretty(v, indent: str, out: list) -> None:
    if v is None:
        out.append("null")
    elif v is True:
        out.append("true")
    elif v is False:
        out.append("false")
    elif isinstance(v, int):
        out.append(str(v))
    elif isinstance(v, float):
        out.append(ryu_f64(v) if math.isfinite(v) else "null")
    elif isinstance(v, str):
        out.append(_json_str(v))
    elif isinstance(v, dict):
        if not v:
            out.append("{}")
            return
        inner = indent + "  "
        out.append("{")
        first = True
        for k, x in v.items():
            out.append("\n" + inner if first else ",\n" + inner)
            first = False
            out.append(_json_str(k))
            out.append(": ")
            _pretty(x, inner, out)
        out.append("\n" + indent + "}")
    elif isinstance(v, (list, tuple)):
        if not v:
            out.append("[]")
            return
        inner = indent + "  "
        if all(type(x) is float for x in v):  # fast path: long f64 vectors
            sep = ",\n" + inner
            out.append("[\n" + inner)
            out.append(sep.join(ryu_f64(x) if math.isfinite(x) else "null" for x in v))
            out.append("\n" + indent + "]")
            return
        out.append("[")
        first = True
        for x in v:
            out.append("\n" + inner if first else ",\n" + inner)
            first = False
            _pretty(x, inner, out)
        out.append("\n" + indent + "]")
    else:
        raise TypeError(f"cannot serialise {type(v).__name__}")


def to_string_pretty(value) -> str:
    """serde_json::to_string_pretty of a value built from dict (struct, keys in
    field order), list/tuple (seq / tuple), str, int (u64/usize), float (f64)."""
    out: list = []
    _pretty(value, "", out)
    return "".join(out)


# =====================================================================================
# serde_json::from_str number parsing (no float_roundtrip)
# =====================================================================================
_U64_MAX = (1 << 64) - 1
_I32_MAX = (1 << 31) - 1
_POW10 = [float(f"1e{i}") for i in range(309)]


class _JsonF64(float):
    """A JSON number that serde_json parses as F64 (has '.', 'e' or overflowed)."""


def _f64_from_parts(positive: bool, significand: int, exponent: int) -> float:
    # de.rs f64_from_parts (cfg(not(feature = "float_roundtrip")))
    f = float(significand)
    while True:
        a = abs(exponent)
        if a < len(_POW10):
            if exponent >= 0:
                f *= _POW10[a]
                if math.isinf(f):
                    raise SerdeError("number out of range")
            else:
                f /= _POW10[a]
            break
        if f == 0.0:
            break
        if exponent >= 0:
            raise SerdeError("number out of range")
        f /= 1e308
        exponent += 308
    return f if positive else -f


def _parse_number(tok: str):
    """Value of one JSON number token the way serde_json's parser produces it:
    int for U64/I64, _JsonF64 for F64."""
    positive = not tok.startswith("-")
    s = tok if positive else tok[1:]
    i, n = 0, len(s)
    significand = 0
    exponent = 0
    # integer part: parse_integer, then parse_long_integer once the next digit
    # would overflow u64 (every further integer digit only bumps the exponent)
    long_int = False
    while i < n and s[i].isdigit():
        d = ord(s[i]) - 48
        if long_int:
            exponent += 1
        elif significand * 10 + d > _U64_MAX:
            long_int = True
            exponent += 1
        else:
            significand = significand * 10 + d
        i += 1
    is_float = long_int
    if i < n and s[i] == ".":
        # parse_decimal starts its own overflow check; after the first digit that
        # would overflow, parse_decimal_overflow drops the rest
        is_float = True
        i += 1
        dropped = False
        while i < n and s[i].isdigit():
            d = ord(s[i]) - 48
            if not dropped and significand * 10 + d > _U64_MAX:
                dropped = True
            if not dropped:
                significand = significand * 10 + d
                exponent -= 1
            i += 1
    if i < n and s[i] in "eE":
        is_float = True
        i += 1
        pos_exp = True
        if s[i] in "+-":
            pos_exp = s[i] == "+"
            i += 1
        e = 0
        while i < n:
            e = e * 10 + (ord(s[i]) - 48)
            if e > _I32_MAX:  # parse_exponent_overflow
                if significand != 0 and pos_exp:
                    raise SerdeError("number out of range")
                return _JsonF64(0.0 if positive else -0.0)
            i += 1
        exponent = exponent + e if pos_exp else exponent - e
        exponent = max(-(1 << 31), min(_I32_MAX, exponent))  # saturating_add/sub
    if is_float:
        return _JsonF64(_f64_from_parts(positive, significand, exponent))
    if positive:
        return significand
    neg = -significand
    if neg < -(1 << 63):  # (significand as i64).wrapping_neg() >= 0 -> F64
        return _JsonF64(-float(significand))
    if neg == 0:
        return _JsonF64(-0.0)
    return neg


def _reject_constant(name):
    raise SerdeError(f"invalid JSON value {name}")


def from_str(text: str):
    """serde_json::from_str into generic values (numbers as serde_json parses them)."""
    try:
        return json.loads(text, parse_float=_parse_number, parse_int=_parse_number,
                          parse_constant=_reject_constant)
    except json.JSONDecodeError as e:
        raise SerdeError(str(e)) from None


# =====================================================================================
# rmp_serde::to_vec / from_slice
# =====================================================================================
def to_msgpack(value) -> bytes:
    """rmp_serde::to_vec of a value already laid out as arrays (see module doc)."""
    return msgpack.packb(value, use_bin_type=True, use_single_float=False, strict_types=False)


def from_msgpack(data: bytes):
    try:
        return msgpack.unpackb(data, raw=False, strict_map_key=False, use_list=True)
    except (msgpack.ExtraData, msgpack.FormatError, msgpack.StackError, ValueError) as e:
        raise SerdeError(str(e)) from None


# =====================================================================================
# schema helpers shared by the Spectrum / Deconvolution codecs
# =====================================================================================
def f64(v, what: str) -> float:
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise SerdeError(f"invalid type for {what}: expected f64")
    return float(v)


def usize(v, what: str) -> int:
    if isinstance(v, bool) or isinstance(v, float) or not isinstance(v, int):
        raise SerdeError(f"invalid type for {what}: expected usize")
    if v < 0 or v > _U64_MAX:
        raise SerdeError(f"invalid value for {what}: expected usize")
    return int(v)


def string(v, what: str) -> str:
    if not isinstance(v, str):
        raise SerdeError(f"invalid type for {what}: expected a string")
    return v


def fields(v, names: tuple, what: str, optional: tuple = ()) -> dict:
    """Struct from a map (by name) or an array (by position, as rmp_serde writes
    it). Missing optional fields are None; unknown map keys are ignored."""
    if isinstance(v, dict):
        out = {}
        for k in names:
            if k in v:
                out[k] = v[k]
            elif k in optional:
                out[k] = None
            else:
                raise SerdeError(f"missing field `{k}` in {what}")
        return out
    if isinstance(v, list):
        need = len(names) - len(optional)
        if len(v) < need:
            raise SerdeError(f"invalid length {len(v)} for {what}, expected {need}")
        if len(v) > len(names):
            raise SerdeError(f"invalid length {len(v)} for {what}, expected {len(names)}")
        out = dict(zip(names, v))
        for k in names[len(v):]:
            out[k] = None
        return out
    raise SerdeError(f"invalid type for {what}: expected struct")


def tagged(v, what: str) -> tuple[str, object]:
    """Internally tagged enum (``#[serde(tag = "method")]``): (variant, rest)."""
    if isinstance(v, dict):
        if "method" not in v:
            raise SerdeError(f"missing field `method` in {what}")
        return string(v["method"], what), v
    if isinstance(v, list):
        if not v:
            raise SerdeError(f"missing tag in {what}")
        return string(v[0], what), v[1:]
    raise SerdeError(f"invalid type for {what}: expected enum")


def serialization_error(e: Exception) -> exc.SerializationError:
    return exc.SerializationError(str(e))
