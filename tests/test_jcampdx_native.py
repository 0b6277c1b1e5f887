"""The native JCAMP-DX decoder (mdg_jcampdx_decode, csrc/mdg_jcampdx.cpp; CPU, no
GPU) against the regex restatement it replaces on the hot read path
(metabodecon/_jcampdx.py decode_asdf / decode_affn, itself pinned by the reference's
decode vectors jcampdx.rs:1226-1299 and its data files in test_formats.py):
  * the reference's vectors and every committed .dx fixture: identical bits;
  * random blocks over the encodings' alphabet (PAC, SQZ, DIF, DUP, line breaks of
    every kind, blank lines, signs): whenever the native decoder returns values, the
    restatement returns the same bits; whenever the restatement raises, the native
    decoder declines (the reader then raises the restatement's error); it declines
    otherwise only on NaN tokens (left to Python for the sign of the NaN).
"""
import ctypes
import gzip
import os
import random

import numpy as np
import pytest

from metabodecon import _jcampdx as jdx
from metabodecon import _native as nat

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "jcampdx")


def native(data: str, factor: float = 1.0):
    raw = data.encode("ascii")
    n = ctypes.c_size_t(0)
    cap = max(16, 4 * len(raw))
    for _ in range(2):
        out = np.empty(cap)
        st = nat.lib().mdg_jcampdx_decode(raw, len(raw), factor, nat.ptr(out), cap, ctypes.byref(n))
        if st != nat.CAPACITY:
            break
        cap = n.value
    return out[: n.value].copy() if st == 0 else st


def python(data: str, factor: float = 1.0):
    try:
        if jdx.ENCODING[0].search(data):
            return jdx.decode_asdf(data, factor, "t")
        return jdx.decode_affn(data, factor, "t")
    except jdx.JcampError:
        return None


def same(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.int64), b.view(np.int64))


def test_reference_vectors_and_capacity():
    affn = "19 482 -763 215 -632\n15 -924 357 -678 841"
    vecs = [affn,
            "19 +482-763+215-632-924+357-678+841+512-194\n9  +321-467-689+278+278+732+835-619+247-193",
            "19 D82g63B15f32i24C57f78H41E12a94\n9  C21d67f89B78B78G32H35f19B47a93",
            "19 D82j245R78q47k92J281j035J519l29p06\n10 a94N15p88k22R67TM54J03j454Q66m40",
            "1 A T", "1 2 3\n"]
    for v in vecs:
        for f in (1.0, 2.5, 0.0078125):
            assert same(native(v, f), python(v, f)), v
    # capacity: the count is reported and nothing is written
    raw = affn.encode()
    n = ctypes.c_size_t(0)
    out = np.full(3, 7.0)
    assert nat.lib().mdg_jcampdx_decode(raw, len(raw), 1.0, nat.ptr(out), 3, ctypes.byref(n)) == nat.CAPACITY
    assert n.value == 8 and out.tolist() == [7.0, 7.0, 7.0]
    # malformed data and non-ASCII text are left to the restatement
    assert native("1 2 x") == nat.INVALID_ARGUMENT
    raw = "1 2 3 4".encode("utf-8")
    assert nat.lib().mdg_jcampdx_decode(raw, len(raw), 1.0, nat.ptr(out), 3, ctypes.byref(n)) == \
        nat.INVALID_ARGUMENT


@pytest.mark.parametrize("name", sorted(f for f in os.listdir(GOLD) if f.endswith(".dx.gz")))
def test_fixture_files_bit_identical(name):
    dx = gzip.open(os.path.join(GOLD, name), "rt", encoding="utf-8", newline="").read()
    hdr = jdx.read_header(dx, name)
    blk = jdx.read_xydata(dx, name) if hdr["format"] == "XYDATA" else jdx.read_ntuples(dx, name)
    got = jdx.decode_native(blk["data"], blk["factor"], blk["data_size"])
    ref = python(blk["data"], blk["factor"])
    assert got is not None and ref is not None and same(got, ref), name
    assert got.size == blk["data_size"]


ALPHABET = list("0123456789") * 4 + list("@ABCDEFGHIabcdefghi%JKLMNOPQRjklmnopqrSTUVWXYZs") + \
    list("+-.eE") + [" "] * 12 + ["\n"] * 4 + ["\r\n", "\r", "\t", "  \n", "\n\n"]


def _block(rng):
    lines = []
    for _ in range(rng.randint(1, 8)):
        toks = [str(rng.randint(0, 99))]
        for _ in range(rng.randint(0, 12)):
            kind = rng.random()
            if kind < 0.5:  # an encoded value
                toks.append(rng.choice("@ABCDEFGHIabcdefghi") + str(rng.randint(0, 999)))
            elif kind < 0.75:
                toks.append(rng.choice("%JKLMNOPQRjklmnopqr") + str(rng.randint(0, 99)))
            elif kind < 0.85:
                toks.append(rng.choice("STUVWXYZs") + str(rng.randint(0, 9) if rng.random() < 0.3 else ""))
            else:
                toks.append(rng.choice(["+", "-", ""]) + str(rng.randint(0, 9999)))
        sep = rng.choice(["", " ", "  "])
        lines.append(sep.join(toks))
    text = rng.choice(["\n", "\r\n", "\r", " \n", "\n\n"]).join(lines)
    if rng.random() < 0.3:  # noise characters
        k = rng.randrange(len(text) + 1)
        text = text[:k] + "".join(rng.choice(ALPHABET) for _ in range(rng.randint(1, 4))) + text[k:]
    return text


def test_random_blocks_agree_with_the_restatement():
    rng = random.Random(20261017)
    decoded = declined = 0
    for _ in range(3000):
        text = _block(rng)
        a, b = native(text), python(text)
        if isinstance(a, np.ndarray):
            assert b is not None and same(a, b), repr(text)
            decoded += 1
        else:
            assert a == nat.INVALID_ARGUMENT, (a, repr(text))
            declined += 1
            if b is not None:  # declined though the restatement decodes: NaN only
                assert "nan" in text.lower(), repr(text)
    assert decoded > 800, (decoded, declined)  # the rest: data both reject


def test_affn_floats_agree():
    rng = random.Random(7)
    toks = ["1.5", "-2.25e3", ".5", "5.", "1E-320", "1e400", "-0", "+7", "inf", "-Infinity",
            "123456789012345678901234567890", "0.1", "2.5e-5"]
    for _ in range(200):
        lines = [" ".join(["9"] + [rng.choice(toks) for _ in range(rng.randint(0, 6))])
                 for _ in range(rng.randint(1, 5))]
        text = "\n".join(lines)
        # AFFN only when no ASDF character is present (E/e exponents are ASDF characters)
        a, b = native(text), python(text)
        if isinstance(a, np.ndarray):
            assert b is not None and same(a, b), text
        else:
            assert b is None or "nan" in text.lower(), text


@pytest.mark.timeout(60)
def test_long_whitespace_runs_are_linear():
    """the DIF/DUP token matcher was quadratic in the length of a whitespace
    run that does not match. 400k blanks between values (and before a DIF token after
    an empty value, the shorter-first-run candidate) decode in well under a second,
    with the restatement's bits."""
    import time
    native("1 2")  # the library's first load is not the decoder's time
    shapes = (lambda k: "1 2" + " " * k + "3 4", lambda k: "5" + " " * k + "J2 7",
              lambda k: "@" + " " * k + "%1 " + " " * k + "A")
    for make in shapes:
        t = time.perf_counter()
        native(make(400_000))
        assert time.perf_counter() - t < 1.0, make(0)
        # the same shape, short enough for the regex restatement (itself quadratic
        # here: Python's backtracking), bit for bit
        got, want = native(make(100)), python(make(100))
        if isinstance(got, np.ndarray) and isinstance(want, np.ndarray):
            assert np.array_equal(got, want)
        else:
            assert not isinstance(got, np.ndarray) and not isinstance(want, np.ndarray)


def test_decode_native_declines_without_the_library(monkeypatch):
    """reading a JCAMP-DX file needs no engine library; when it is missing
    or stale the regex restatement decodes the block."""
    def missing():
        raise nat.NativeLibraryError("libmdgpu.so missing")
    monkeypatch.setattr(nat, "lib", missing)
    assert jdx.decode_native("1 2 3", 1.0, 3) is None
