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
def test_compact_pinned_pageable_and_mixed_rows_match_goldens(lanes, monkeypatch):
    """The 16 blood spectra four ways: as read (the int32 sample rows in one
    page-locked block, mdg_deconvolute_rows_i32 decoding them on the device), as f64
    rows in page-locked memory (direct DMA), as f64 rows in ordinary memory (the
    ring), and compact and f64 spectra mixed in one call (the f64 rows path); one
    batch of 16 (1 lane) and two concurrent lanes of 8."""
    import metabodecon as md
    monkeypatch.setattr(md.Deconvoluter, "LANES", lanes)
    monkeypatch.setattr(md.Deconvoluter, "ONE_LANE_UPTO", 0)
    read = _blood(md)
    assert all(s._raw is not None and _pinned(s._raw[0]) for s in read)
    _check(md.Deconvoluter().par_deconvolute_spectra(read), range(16))
    pinned = [md.Spectrum(s.chemical_shifts, s.intensities, s.signal_boundaries) for s in read]
    assert all(s._raw is None and _pinned(s.intensities) for s in pinned)
    _check(md.Deconvoluter().par_deconvolute_spectra(pinned), range(16))
    monkeypatch.setattr(nat, "_pinned_off", True)
    plain = [md.Spectrum(s.chemical_shifts, s.intensities, s.signal_boundaries) for s in read]
    assert not any(_pinned(s.intensities) for s in plain)
    _check(md.Deconvoluter().par_deconvolute_spectra(plain), range(16))
    mixed = [read[k] if k % 3 else plain[k] for k in range(16)]
    _check(md.Deconvoluter().par_deconvolute_spectra(mixed), range(16))
    # one spectrum through deconvolute_spectrum (b = 1), compact and f64
    _check([md.Deconvoluter().deconvolute_spectrum(read[5])], [5])
    _check([md.Deconvoluter().deconvolute_spectrum(plain[5])], [5])


def test_compact_rows_decode_bit_exact():
    """The device decode of the compact rows equals the reader's f64 rows: the
    smoothed rows of mdg_deconvolute_rows_i32 equal the oracle's moving average of
    the reader's intensities, and every result equals mdg_deconvolute_rows' on the
    reader's f64 rows (a shared axis in one call, distinct axes in another)."""
    import metabodecon as md
    import oracle
    read = _blood(md)
    single = md.Spectrum.read_bruker(os.path.join(GOLDEN, "bruker", "blood", "blood_03"), 10, 10,
                                     (-2.2, 11.8))
    assert single._raw is not None and np.array_equal(single.intensities, read[2].intensities)
    ctx = nat.context()
    s = md.Deconvoluter().settings
    n = len(read[0])
    cap = n // 2 + 2
    for group in ([0, 1, 2, 3], [2, 2, 2]):
        spectra = [read[k] for k in group]
        b = len(spectra)
        sb = np.array([sp.signal_boundaries for sp in spectra], dtype=np.float64)

        def run(compact):
            out = np.zeros((b, cap, 3))
            counts = np.zeros(b, dtype=np.uintp)
            mse = np.zeros(b)
            status = np.zeros(b, dtype=np.intc)
            tail = (nat.ptr(out), cap, nat.ptr(counts, nat._szp), nat.ptr(mse),
                    status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
            if compact:
                yr = np.array([sp._raw[0].ctypes.data for sp in spectra], dtype=np.uintp)
                axes = np.array([sp._raw[2] for sp in spectra], dtype=np.float64)
                scale = np.array([sp._raw[1] for sp in spectra], dtype=np.float64)
                rc = nat.lib().mdg_deconvolute_rows_i32(
                    ctx.handle, b, n, nat.ptr(axes), yr.ctypes.data_as(ctypes.POINTER(nat._i32p)),
                    nat.ptr(scale), nat.ptr(sb), ctypes.byref(s), None, 0, *tail)
            else:
                xr = np.array([sp.chemical_shifts.ctypes.data for sp in spectra], dtype=np.uintp)
                yr = np.array([sp.intensities.ctypes.data for sp in spectra], dtype=np.uintp)
                rc = nat.lib().mdg_deconvolute_rows(
                    ctx.handle, b, n, xr.ctypes.data_as(ctypes.POINTER(nat._dp)),
                    yr.ctypes.data_as(ctypes.POINTER(nat._dp)), nat.ptr(sb), ctypes.byref(s),
                    None, 0, *tail)
            assert rc == 0 and not status.any()
            return out, counts, mse
        with ctx.lock:
            c_out, c_counts, c_mse = run(True)
            smoothed = [ctx.last_smoothed(k, n) for k in range(b)]
            f_out, f_counts, f_mse = run(False)
        for k, sp in enumerate(spectra):
            assert np.array_equal(smoothed[k], oracle.moving_average(sp.intensities, s.smooth_iterations,
                                                                     s.smooth_window)), k
        assert np.array_equal(c_counts, f_counts) and np.array_equal(c_mse, f_mse)
        assert np.array_equal(c_out, f_out)


@pytest.mark.parametrize("env", ["", "MDG_DEC_OVERLAP=0", "MDG_SMOOTH=pipe", "MDG_PREP=separate",
                                 "MDG_CHAIN_EXCL=0"])
def test_compact_rows_decode_paths(env, monkeypatch, engine_env):
    """Page-locked compact rows are decoded from host memory by the pipeline: by the
    chain launch's decoders while pass 0 smooths the decoded chunks (default), or by
    a decode launch of their own before any other smoother / a separate prep
    (MDG_SMOOTH=pipe, MDG_PREP=separate); MDG_DEC_OVERLAP=0 sends them by DMA first.
    Every path: the smoothed rows equal the oracle's and the results equal
    mdg_deconvolute_rows' on the reader's f64 rows, at 1, 3 (distinct axes) and 16
    spectra (two decoders per XCD)."""
    import metabodecon as md
    import oracle
    if env:
        k, v = env.split("=")
        engine_env.setenv(k, v)
    read = _blood(md)
    ctx = nat.context()
    s = md.Deconvoluter().settings
    n = len(read[0])
    cap = n // 2 + 2
    for group in ([7], [0, 5, 9], list(range(16))):
        spectra = [read[k] for k in group]
        b = len(spectra)
        sb = np.array([sp.signal_boundaries for sp in spectra], dtype=np.float64)

        def run(compact):
            out = np.zeros((b, cap, 3))
            counts = np.zeros(b, dtype=np.uintp)
            mse = np.zeros(b)
            status = np.zeros(b, dtype=np.intc)
            tail = (nat.ptr(out), cap, nat.ptr(counts, nat._szp), nat.ptr(mse),
                    status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
            if compact:
                yr = np.array([sp._raw[0].ctypes.data for sp in spectra], dtype=np.uintp)
                axes = np.array([sp._raw[2] for sp in spectra], dtype=np.float64)
                scale = np.array([sp._raw[1] for sp in spectra], dtype=np.float64)
                rc = nat.lib().mdg_deconvolute_rows_i32(
                    ctx.handle, b, n, nat.ptr(axes), yr.ctypes.data_as(ctypes.POINTER(nat._i32p)),
                    nat.ptr(scale), nat.ptr(sb), ctypes.byref(s), None, 0, *tail)
            else:
                xr = np.array([sp.chemical_shifts.ctypes.data for sp in spectra], dtype=np.uintp)
                yr = np.array([sp.intensities.ctypes.data for sp in spectra], dtype=np.uintp)
                rc = nat.lib().mdg_deconvolute_rows(
                    ctx.handle, b, n, xr.ctypes.data_as(ctypes.POINTER(nat._dp)),
                    yr.ctypes.data_as(ctypes.POINTER(nat._dp)), nat.ptr(sb), ctypes.byref(s),
                    None, 0, *tail)
            assert rc == 0 and not status.any(), (rc, status)
            return out, counts, mse
        with ctx.lock:
            c_out, c_counts, c_mse = run(True)
            smoothed = [ctx.last_smoothed(k, n) for k in range(b)]
            f_out, f_counts, f_mse = run(False)
        for k, sp in enumerate(spectra):
            assert np.array_equal(smoothed[k], oracle.moving_average(sp.intensities, s.smooth_iterations,
                                                                     s.smooth_window)), (group, k)
        assert np.array_equal(c_counts, f_counts) and np.array_equal(c_mse, f_mse), group
        assert np.array_equal(c_out, f_out), group


@pytest.mark.parametrize("n,b,off", [(4099, 1, 1), (20001, 5, 3), (131071, 2, 0)])
def test_compact_rows_decode_odd_shapes(n, b, off):
    """The in-launch decode on rows that are not 16-byte aligned (an offset of off
    int32 into a page-locked block: the decoders' scalar path) and lengths that are
    not a multiple of 4 or of the chunk (the tails), 1-5 spectra (32 and 64
    decoders): results bit-equal to mdg_deconvolute_rows on the same rows built on
    the host with the decode's operations."""
    import metabodecon as md
    ctx = nat.context()
    s = md.Deconvoluter().settings
    rng = np.random.default_rng(n + b)
    blk = nat.pinned_empty((b * (n + 4) + 4,), np.int32)
    assert blk is not None
    rows, xs, ys, axes, scales = [], [], [], [], []
    for i in range(b):
        mx, wd, dv = 11.8 + 0.01 * i, 14.0, float(n - 1)
        x = mx - (np.arange(n, dtype=np.float64) * wd) / dv
        c = rng.uniform(1.0, 9.0, 40)
        hw = rng.uniform(0.002, 0.01, 40) ** 2
        a = rng.uniform(1e5, 1e7, 40) * hw
        y = (a[:, None] / (hw[:, None] + (x[None, :] - c[:, None]) ** 2)).sum(0) + rng.normal(0, 50, n)
        scale = 2.0 ** int(rng.integers(-2, 3))
        raw = np.round(y / scale).astype(np.int32)
        r = blk[off + i * (n + 4): off + i * (n + 4) + n]
        r[:] = raw
        rows.append(r)
        xs.append(nat.pinned_copy(x))
        ys.append(nat.pinned_copy(raw.astype(np.float64) * scale))
        axes.append((mx, wd, dv))
        scales.append(scale)
    cap = n // 2 + 2
    sb = np.array([[11.0, 0.5]] * b, dtype=np.float64)

    def run(compact):
        out = np.zeros((b, cap, 3))
        counts = np.zeros(b, dtype=np.uintp)
        mse = np.zeros(b)
        status = np.zeros(b, dtype=np.intc)
        tail = (nat.ptr(out), cap, nat.ptr(counts, nat._szp), nat.ptr(mse),
                status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        if compact:
            yr = np.array([r.ctypes.data for r in rows], dtype=np.uintp)
            ax = np.array(axes, dtype=np.float64)
            sc = np.array(scales, dtype=np.float64)
            rc = nat.lib().mdg_deconvolute_rows_i32(
                ctx.handle, b, n, nat.ptr(ax), yr.ctypes.data_as(ctypes.POINTER(nat._i32p)),
                nat.ptr(sc), nat.ptr(sb), ctypes.byref(s), None, 0, *tail)
        else:
            xr = np.array([v.ctypes.data for v in xs], dtype=np.uintp)
            yr = np.array([v.ctypes.data for v in ys], dtype=np.uintp)
            rc = nat.lib().mdg_deconvolute_rows(
                ctx.handle, b, n, xr.ctypes.data_as(ctypes.POINTER(nat._dp)),
                yr.ctypes.data_as(ctypes.POINTER(nat._dp)), nat.ptr(sb), ctypes.byref(s),
                None, 0, *tail)
        return rc, out, counts, mse, status
    with ctx.lock:
        c = run(True)
        f = run(False)
    assert c[0] == f[0]
    assert np.array_equal(c[4], f[4]) and np.array_equal(c[2], f[2]) and np.array_equal(c[3], f[3])
    assert np.array_equal(c[1], f[1])
    assert c[2].min() > 0  # every spectrum found its peaks


def _compact_set(n, b, seed, blk_off=0):
    """b synthetic compact rows of n points in one page-locked block (rows
    adjacent, as Spectrum.read_bruker_set places them), with their axes, scales and
    the f64 intensities the decode must produce."""
    rng = np.random.default_rng(seed)
    blk = nat.pinned_empty((b * n + blk_off + 4,), np.int32)
    assert blk is not None
    rows, axes, scales, ys = [], [], [], []
    for i in range(b):
        mx, wd, dv = 11.8 + 0.01 * i, 14.0, float(n - 1)
        x = mx - (np.arange(n, dtype=np.float64) * wd) / dv
        c = rng.uniform(1.0, 9.0, 40)
        hw = rng.uniform(0.002, 0.01, 40) ** 2
        a = rng.uniform(1e5, 1e7, 40) * hw
        y = (a[:, None] / (hw[:, None] + (x[None, :] - c[:, None]) ** 2)).sum(0) + rng.normal(0, 50, n)
        scale = 2.0 ** int(rng.integers(-2, 3))
        raw = np.round(y / scale).astype(np.int32)
        r = blk[blk_off + i * n: blk_off + (i + 1) * n]
        r[:] = raw
        rows.append(r)
        axes.append((mx, wd, dv))
        scales.append(scale)
        ys.append(raw.astype(np.float64) * scale)
    return blk, rows, np.array(axes, dtype=np.float64), np.array(scales, dtype=np.float64), ys


def _run_compact(ctx, s, n, rows, axes, scales):
    b = len(rows)
    cap = n // 2 + 2
    sb = np.array([[11.0, 0.5]] * b, dtype=np.float64)
    out = np.zeros((b, cap, 3))
    counts = np.zeros(b, dtype=np.uintp)
    mse = np.zeros(b)
    status = np.zeros(b, dtype=np.intc)
    yr = np.array([r.ctypes.data for r in rows], dtype=np.uintp)
    rc = nat.lib().mdg_deconvolute_rows_i32(
        ctx.handle, b, n, nat.ptr(axes), yr.ctypes.data_as(ctypes.POINTER(nat._i32p)),
        nat.ptr(scales), nat.ptr(sb), ctypes.byref(s), None, 0, nat.ptr(out), cap,
        nat.ptr(counts, nat._szp), nat.ptr(mse), status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    return rc, out, counts, mse, status


@pytest.mark.parametrize("n", [20001, 131071])
@pytest.mark.parametrize("b", [2, 5, 16])
def test_compact_rows_decode_poisoned_staging_under_load(n, b):
    """the in-launch decode's cross-XCD hand-off (chain_decode ->
    pass 0's feeder) under the conditions the microarchitecture guide says expose a
    stale read: the staging rows are poisoned by a call on the same context
    immediately before (other spectra of the same shape, so every staging line holds
    other values and was just read, warm, by that call's chains), the rows are an odd
    length (n % 16 != 0: before round 5 a 128-byte line straddled two chunks of two
    decoders; now the rows are padded to whole lines), 2-16 spectra (32 or 64
    decoders, rows on every XCD), and a second engine context runs batches on the
    same GPU the whole time (uneven load). Every smoothed word of every spectrum is
    checked against the oracle's moving average of the decoded intensities, three
    poisoned rounds in a row."""
    import threading

    import metabodecon as md
    import oracle
    ctx = nat.context()
    s = md.Deconvoluter().settings
    cur = _compact_set(n, b, seed=1000 + n + b)
    poison = _compact_set(n, b, seed=2000 + n + b, blk_off=3)
    other = nat.Context(0)
    busy_rows = _compact_set(65536, 8, seed=7)
    stop = threading.Event()
    busy_err = []

    def busy():  # the second lane: compact batches on another context until stopped
        try:
            while not stop.is_set():
                with other.lock:
                    rc = _run_compact(other, s, 65536, busy_rows[1], busy_rows[2], busy_rows[3])[0]
                if rc not in (0, 1, 2, 3):
                    busy_err.append(rc)
                    return
        except Exception as e:  # pragma: no cover - reported below
            busy_err.append(repr(e))
    t = threading.Thread(target=busy)
    t.start()
    try:
        ref = [oracle.moving_average(y, s.smooth_iterations, s.smooth_window) for y in cur[4]]
        for rnd in range(3):
            with ctx.lock:
                _run_compact(ctx, s, n, poison[1], poison[2], poison[3])
                rc, out, counts, mse, status = _run_compact(ctx, s, n, cur[1], cur[2], cur[3])
                assert rc in (0, 1, 2, 3), rc
                smoothed = [ctx.last_smoothed(k, n) for k in range(b)]
            for k in range(b):
                bad = np.flatnonzero(smoothed[k] != ref[k])
                assert bad.size == 0, (rnd, k, bad[:8], bad.size)
    finally:
        stop.set()
        t.join(timeout=120)
    assert not busy_err, busy_err
    other.close()


def test_compact_rows_reject_bad_descriptors():
    """A zero divisor, a non-finite axis operand or scale, or a null row: invalid
    argument, nothing run."""
    import metabodecon as md
    sp = _blood(md)[0]
    ctx = nat.context()
    n = len(sp)
    cap = n // 2 + 2
    out = np.zeros((1, cap, 3))
    counts = np.zeros(1, dtype=np.uintp)
    mse = np.zeros(1)
    status = np.zeros(1, dtype=np.intc)
    sb = np.array([sp.signal_boundaries], dtype=np.float64)
    good_ax = np.array([sp._raw[2]], dtype=np.float64)
    for ax, scale, row in ((good_ax * [1, 1, 0], 1.0, sp._raw[0].ctypes.data),
                           (good_ax * [np.nan, 1, 1], 1.0, sp._raw[0].ctypes.data),
                           (good_ax, np.inf, sp._raw[0].ctypes.data),
                           (good_ax, 1.0, 0)):
        yr = np.array([row], dtype=np.uintp)
        sc = np.array([scale])
        with ctx.lock:
            rc = nat.lib().mdg_deconvolute_rows_i32(
                ctx.handle, 1, n, nat.ptr(np.ascontiguousarray(ax)),
                yr.ctypes.data_as(ctypes.POINTER(nat._i32p)), nat.ptr(sc), nat.ptr(sb),
                ctypes.byref(md.Deconvoluter().settings), None, 0, nat.ptr(out), cap,
                nat.ptr(counts, nat._szp), nat.ptr(mse),
                status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        assert rc == nat.INVALID_ARGUMENT


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


def test_device_decode_equals_reader_rows():
    """mdg_decode_rows_i32_device rebuilds every blood spectrum's axis and
    intensities bit for bit as the reader computed them on the host
    (maximum - (i * width) / (SI - 1) and sample * 2^NC_proc)."""
    torch = pytest.importorskip("torch")
    import metabodecon as md
    read = _blood(md)
    n, b = len(read[0]), len(read)
    raw = torch.from_numpy(np.stack([s._raw[0] for s in read])).to("cuda")
    desc = torch.tensor([[*s._raw[2], s._raw[1]] for s in read], dtype=torch.float64,
                        device="cuda")
    x = torch.empty((b, n), dtype=torch.float64, device="cuda")
    y = torch.empty((b, n), dtype=torch.float64, device="cuda")
    ctx = nat.context()
    torch.cuda.synchronize()
    assert nat.lib().mdg_decode_rows_i32_device(ctx.handle, b, n, raw.data_ptr(), desc.data_ptr(),
                                                x.data_ptr(), y.data_ptr()) == 0
    ctx.synchronize()
    assert np.array_equal(x.cpu().numpy(), np.stack([s.chemical_shifts for s in read]))
    assert np.array_equal(y.cpu().numpy(), np.stack([s.intensities for s in read]))
    assert nat.lib().mdg_decode_rows_i32_device(ctx.handle, b, n, None, desc.data_ptr(),
                                                x.data_ptr(), y.data_ptr()) == nat.INVALID_ARGUMENT
