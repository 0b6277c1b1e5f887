"""Host rows in page-locked memory (mdg_host_alloc, include/mdgpu.h).

A Spectrum keeps its rows in page-locked blocks when the engine can give them, and
mdg_deconvolute_rows then sends them by DMA straight from there instead of through
the context's ring. Every path must give the goldens' results: parameters and
counts bit-identical, MSE within 1e-12 relative.
"""
import ctypes
import os

import numpy as np
import pytest

from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu

MSE_RTOL = 1e-12

nat = pytest.importorskip("metabodecon._native")


def _pinned(a: np.ndarray) -> bool:
    b = a
    while b is not None:
        if isinstance(b, ctypes.Array):
            return True
        b = getattr(b, "base", None)
    return False


def _blood(md):
    return md.Spectrum.read_bruker_set(os.path.join(GOLDEN, "bruker", "blood"), 10, 10,
                                       (-2.2, 11.8))


def _check(decs, which):
    for k, d in zip(which, decs):
        g = np.load(os.path.join(GOLDEN, "expected", f"blood_{k + 1:02d}.npz"))
        assert np.array_equal(d.params, g["params"]), k
        assert abs(d.mse - float(g["mse"])) <= MSE_RTOL * abs(float(g["mse"]))


@pytest.mark.parametrize("lanes", [1, 2])
def test_pinned_pageable_and_mixed_rows_match_goldens(lanes, monkeypatch):
    """The 16 blood spectra three ways: every row page-locked (direct DMA), every
    row in ordinary memory (the ring), and the two mixed in one call (the ring);
    one batch of 16 (1 lane) and two concurrent lanes of 8."""
    import metabodecon as md
    monkeypatch.setattr(md.Deconvoluter, "LANES", lanes)
    pinned = _blood(md)
    assert all(_pinned(s.chemical_shifts) and _pinned(s.intensities) for s in pinned)
    _check(md.Deconvoluter().par_deconvolute_spectra(pinned), range(16))
    monkeypatch.setattr(nat, "_pinned_off", True)
    plain = _blood(md)
    assert not any(_pinned(s.intensities) for s in plain)
    _check(md.Deconvoluter().par_deconvolute_spectra(plain), range(16))
    mixed = [pinned[k] if k % 3 else plain[k] for k in range(16)]
    _check(md.Deconvoluter().par_deconvolute_spectra(mixed), range(16))
    # one spectrum through deconvolute_spectrum (mdg_deconvolute_rows with b = 1)
    _check([md.Deconvoluter().deconvolute_spectrum(pinned[5])], [5])


def test_pinned_blocks_are_reused_and_rows_released():
    """Released blocks go back to their size's free list: a block of the same size
    comes back at the same address; freeing an unknown pointer is refused."""
    import gc
    a = nat.pinned_empty((131072,))
    assert a is not None
    addr = a.ctypes.data
    a[:] = 1.5
    del a
    gc.collect()
    b = nat.pinned_empty((131072,))
    assert b.ctypes.data == addr
    assert nat.lib().mdg_host_free(ctypes.c_void_p(addr + 8)) == nat.INVALID_ARGUMENT
    assert nat.lib().mdg_host_free(None) == nat.OK


def test_pinned_rows_with_an_offset_into_a_block():
    """Rows that are views into one page-locked block (not block starts), adjacent
    rows sent as one DMA: the results equal the per-spectrum calls'."""
    import metabodecon as md
    spectra = _blood(md)[:4]
    n = len(spectra[0])
    blk = nat.pinned_empty((2 * 4 * n + 1,))
    xs = blk[1:1 + 4 * n].reshape(4, n)
    ys = blk[1 + 4 * n:].reshape(4, n)
    for k, s in enumerate(spectra):
        xs[k], ys[k] = s.chemical_shifts, s.intensities
    ctx = nat.context()
    dec = md.Deconvoluter()
    cap = n // 2 + 2
    out = np.zeros((4, cap, 3))
    counts = np.zeros(4, dtype=np.uintp)
    mse = np.zeros(4)
    status = np.zeros(4, dtype=np.intc)
    xr = np.array([xs[k].ctypes.data for k in range(4)], dtype=np.uintp)
    yr = np.array([ys[k].ctypes.data for k in range(4)], dtype=np.uintp)
    sb = np.array([s.signal_boundaries for s in spectra], dtype=np.float64)
    with ctx.lock:
        rc = nat.lib().mdg_deconvolute_rows(
            ctx.handle, 4, n, xr.ctypes.data_as(ctypes.POINTER(nat._dp)),
            yr.ctypes.data_as(ctypes.POINTER(nat._dp)), nat.ptr(sb), ctypes.byref(dec.settings),
            None, 0, nat.ptr(out), cap, nat.ptr(counts, nat._szp), nat.ptr(mse),
            status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    assert rc == 0 and not status.any()
    for k in range(4):
        g = np.load(os.path.join(GOLDEN, "expected", f"blood_{k + 1:02d}.npz"))
        assert np.array_equal(out[k, : int(counts[k])], g["params"]), k
        assert abs(mse[k] - float(g["mse"])) <= MSE_RTOL * abs(float(g["mse"]))
