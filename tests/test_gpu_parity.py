"""GPU parity: the HIP path (through the C ABI) against the oracle and goldens.

Tolerances (north star: Lorentzians within 1e-6 relative, peak index sets
bit-identical): we require MORE -- peak index sets, Lorentzian parameters and
superposition vectors bit-identical (np.array_equal), and the MSE within
MSE_RTOL = 1e-12 relative (its residual sum is a fixed-order tree on the GPU
instead of the reference's left fold, deconvoluter.rs:850-856).
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
from tests.conftest import GOLDEN
from tests.golden.cases import CASES, load_case, synth_spectrum

pytestmark = pytest.mark.gpu

MSE_RTOL = 1e-12

nat = pytest.importorskip("metabodecon._native")


@pytest.fixture(scope="module")
def ctx():
    return nat.context(0)


def gpu_batch(ctx, xs, ys, sbs, settings, ignore=()):
    """Run mdg_deconvolute_batch on host arrays; returns status, counts, params, mse."""
    ys = np.ascontiguousarray(ys, dtype=np.float64)
    b, n = ys.shape
    xs = np.ascontiguousarray(xs, dtype=np.float64)
    x_stride = 0 if xs.ndim == 1 else n
    sbs = np.ascontiguousarray(np.broadcast_to(np.asarray(sbs, dtype=np.float64), (b, 2)))
    s = nat.Settings()
    for f, _ in nat.Settings._fields_:
        setattr(s, f, getattr(settings, f))
    ign = np.asarray(ignore, dtype=np.float64).reshape(-1)
    cap = n // 2 + 2
    out = np.zeros((b, cap, 3))
    counts = np.zeros(b, dtype=np.uintp)
    mse = np.zeros(b)
    status = np.zeros(b, dtype=np.intc)
    rc = nat.lib().mdg_deconvolute_batch(
        ctx.handle, b, n, nat.ptr(xs), x_stride, nat.ptr(ys), n, nat.ptr(sbs), ctypes.byref(s),
        nat.ptr(ign) if ign.size else None, ign.size // 2, nat.ptr(out), cap,
        nat.ptr(counts, nat._szp), nat.ptr(mse), status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    assert rc < 100, nat.strerror(rc)
    return status, counts.astype(int), out, mse


def check_against(golden_params, golden_mse, status, count, params, mse, gstatus=0):
    assert status == gstatus
    if gstatus:
        return
    assert count == golden_params.shape[0]
    assert np.array_equal(params[:count], golden_params), \
        np.max(np.abs(params[:count] - golden_params) / np.abs(golden_params))
    assert abs(mse - golden_mse) <= MSE_RTOL * abs(golden_mse)


@pytest.mark.parametrize("name", CASES)
def test_golden_case_bit_exact(ctx, name):
    g = np.load(os.path.join(GOLDEN, "expected", f"{name}.npz"))
    x, y, sb, st, ign = load_case(name)
    status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st, ign)
    check_against(g["params"], float(g["mse"]), status[0], counts[0], out[0], mse[0],
                  int(g["status"]))
    sel = ctx.last_peaks(0, "selected")
    assert np.array_equal(sel.astype(np.int64), g["selected"])


def test_blood_batch_all_16(ctx):
    names = [f"blood_{i:02d}" for i in range(1, 17)]
    data = [load_case(n) for n in names]
    xs = np.stack([d[0] for d in data])
    ys = np.stack([d[1] for d in data])
    sbs = [d[2] for d in data]
    status, counts, out, mse = gpu_batch(ctx, xs, ys, sbs, data[0][3])
    for k, n in enumerate(names):
        g = np.load(os.path.join(GOLDEN, "expected", f"{n}.npz"))
        check_against(g["params"], float(g["mse"]), status[k], counts[k], out[k], mse[k])
        assert np.array_equal(ctx.last_peaks(k, "selected").astype(np.int64), g["selected"])


def gpu_rows(ctx, x_rows, y_rows, sbs, settings):
    """mdg_deconvolute_rows: one pointer per spectrum row (as the Rust shim binds it)."""
    b, n = len(y_rows), len(y_rows[0])
    xr = np.array([r.ctypes.data for r in x_rows], dtype=np.uintp)
    yr = np.array([r.ctypes.data for r in y_rows], dtype=np.uintp)
    sbs = np.ascontiguousarray(np.asarray(sbs, dtype=np.float64).reshape(b, 2))
    s = nat.Settings()
    for f, _ in nat.Settings._fields_:
        setattr(s, f, getattr(settings, f))
    cap = n // 2 + 2
    out = np.zeros((b, cap, 3))
    counts = np.zeros(b, dtype=np.uintp)
    mse = np.zeros(b)
    status = np.zeros(b, dtype=np.intc)
    rc = nat.lib().mdg_deconvolute_rows(
        ctx.handle, b, n, xr.ctypes.data_as(ctypes.POINTER(nat._dp)),
        yr.ctypes.data_as(ctypes.POINTER(nat._dp)), nat.ptr(sbs), ctypes.byref(s), None, 0,
        nat.ptr(out), cap, nat.ptr(counts, nat._szp), nat.ptr(mse),
        status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    assert rc < 100, nat.strerror(rc)
    return status, counts.astype(int), out, mse


def test_rows_entry_blood_16_and_shared_axis(ctx):
    """mdg_deconvolute_rows (row pointers, no stacking) on the 16 blood spectra, in
    a scrambled order with every row its own array: the goldens bit for bit. Then
    spectrum 1's axis passed for every spectrum (one pointer repeated, uploaded
    once) against mdg_deconvolute_batch with x_stride 0 on the same inputs."""
    names = [f"blood_{i:02d}" for i in range(1, 17)]
    order = [5, 0, 15, 3, 9, 1, 12, 7, 2, 14, 8, 4, 11, 6, 13, 10]
    data = [load_case(names[k]) for k in order]
    xs = [np.array(d[0]) for d in data]
    ys = [np.array(d[1]) for d in data]
    sbs = [d[2] for d in data]
    status, counts, out, mse = gpu_rows(ctx, xs, ys, sbs, data[0][3])
    for j, k in enumerate(order):
        g = np.load(os.path.join(GOLDEN, "expected", f"{names[k]}.npz"))
        check_against(g["params"], float(g["mse"]), status[j], counts[j], out[j], mse[j])
    x0 = xs[0]
    st1, c1, o1, m1 = gpu_rows(ctx, [x0] * 16, ys, sbs, data[0][3])
    st2, c2, o2, m2 = gpu_batch(ctx, x0, np.stack(ys), sbs, data[0][3])
    assert np.array_equal(st1, st2) and np.array_equal(c1, c2) and np.array_equal(m1, m2)
    for j in range(16):
        assert np.array_equal(o1[j, : c1[j]], o2[j, : c2[j]])


def test_single_spectrum_entry(ctx):
    """mdg_deconvolute (the Rust shim's gpu_deconvolute_spectrum) on blood_01 and
    blood_02: the goldens bit for bit; a capacity below P_kept reports MDG_CAPACITY
    with the count (the shim's two-phase size query)."""
    for name in ("blood_01", "blood_02"):
        x, y, sb, st, _ = load_case(name)
        x, y = np.ascontiguousarray(x), np.ascontiguousarray(y)
        s = nat.Settings()
        for f, _ in nat.Settings._fields_:
            setattr(s, f, getattr(st, f))
        cap = len(y) // 2 + 2
        out = np.zeros((cap, 3))
        cnt = ctypes.c_size_t(0)
        mse = ctypes.c_double(0.0)
        rc = nat.lib().mdg_deconvolute(ctx.handle, nat.ptr(x), nat.ptr(y), len(y), sb[0], sb[1],
                                       ctypes.byref(s), None, 0, nat.ptr(out), cap,
                                       ctypes.byref(cnt), ctypes.byref(mse))
        g = np.load(os.path.join(GOLDEN, "expected", f"{name}.npz"))
        check_against(g["params"], float(g["mse"]), rc, cnt.value, out, mse.value)
        small = np.zeros((8, 3))
        rc = nat.lib().mdg_deconvolute(ctx.handle, nat.ptr(x), nat.ptr(y), len(y), sb[0], sb[1],
                                       ctypes.byref(s), None, 0, nat.ptr(small), 8,
                                       ctypes.byref(cnt), ctypes.byref(mse))
        assert rc == nat.CAPACITY and cnt.value == g["params"].shape[0]


@pytest.mark.parametrize("path", ["chain", "pipe", "generic"])
def test_detected_peaks_match_oracle(ctx, path, monkeypatch, engine_env):
    """Detected triples equal the oracle's; the selection (which reads the noise
    scores k_peaks computes for the peaks it writes) equals the golden, behind every
    smoother kernel (the chain smoother runs the set-up itself, the others after
    k_prep)."""
    engine_env.setenv("MDG_SMOOTH", path)
    x, y, sb, st, ign = load_case("blood_01")
    gpu_batch(ctx, x, y[None, :], [sb], st)
    det = ctx.last_peaks(0, "detected").astype(np.int64)
    sm = oracle.moving_average(y, 3, 3)
    l, c, r = oracle.detect_peaks(oracle.second_derivative(sm))
    assert np.array_equal(det, np.stack([l, c, r], axis=1))
    g = np.load(os.path.join(GOLDEN, "expected", "blood_01.npz"))
    assert np.array_equal(ctx.last_peaks(0, "selected").astype(np.int64), g["selected"])


def test_concurrent_lanes_and_release(monkeypatch):
    """The 16 blood spectra one per lane context (16 concurrent engine contexts, as
    bench.py's configs[4] runs them), bit-equal to the goldens; then the lanes are
    released and re-created by the next call."""
    import metabodecon as md
    from metabodecon import _native as nat
    monkeypatch.setattr(md.Deconvoluter, "LANES", 16)
    monkeypatch.setattr(md.Deconvoluter, "ONE_LANE_UPTO", 0)
    spectra = md.Spectrum.read_bruker_set(os.path.join(GOLDEN, "bruker", "blood"), 10, 10,
                                          (-2.2, 11.8))
    for rnd in range(2):
        decs = md.Deconvoluter().par_deconvolute_spectra(spectra)
        for k, d in enumerate(decs):
            g = np.load(os.path.join(GOLDEN, "expected", f"blood_{k + 1:02d}.npz"))
            assert np.array_equal(d.params, g["params"]), (rnd, k)
            assert abs(d.mse - float(g["mse"])) <= MSE_RTOL * abs(float(g["mse"]))
        assert len(nat._lanes.get(nat.default_device(), [])) == 16
        nat.release_lanes()
        assert not nat._lanes


def test_chunked_lanes_bit_exact(monkeypatch):
    """A set larger than a chunk: the 16 blood spectra in chunks of at most 3 (6
    chunks) dealt round-robin to 2 lanes, each lane running its chunks one after
    another; every result equals the golden."""
    import metabodecon as md
    monkeypatch.setattr(md.Deconvoluter, "LANES", 2)
    monkeypatch.setattr(md.Deconvoluter, "CHUNK", 3)
    monkeypatch.setattr(md.Deconvoluter, "ONE_LANE_UPTO", 0)
    spectra = md.Spectrum.read_bruker_set(os.path.join(GOLDEN, "bruker", "blood"), 10, 10,
                                          (-2.2, 11.8))
    decs = md.Deconvoluter().par_deconvolute_spectra(spectra)
    for k, d in enumerate(decs):
        g = np.load(os.path.join(GOLDEN, "expected", f"blood_{k + 1:02d}.npz"))
        assert np.array_equal(d.params, g["params"]), k
        assert abs(d.mse - float(g["mse"])) <= MSE_RTOL * abs(float(g["mse"]))


def test_python_api_end_to_end():
    import metabodecon as md
    spectra = md.Spectrum.read_bruker_set(os.path.join(GOLDEN, "bruker", "blood"), 10, 10,
                                          (-2.2, 11.8))
    decs = md.Deconvoluter().par_deconvolute_spectra(spectra)
    for k, d in enumerate(decs):
        g = np.load(os.path.join(GOLDEN, "expected", f"blood_{k + 1:02d}.npz"))
        assert np.array_equal(d.params, g["params"])
        assert abs(d.mse - float(g["mse"])) <= MSE_RTOL * abs(float(g["mse"]))
    # Deconvolution.par_superposition_vec == oracle superposition, bitwise
    sup = decs[0].par_superposition_vec(spectra[0].chemical_shifts)
    ref = oracle.superposition_vec(spectra[0].chemical_shifts, decs[0].params, threads=16)
    assert np.array_equal(sup, ref)
    dec = md.Deconvoluter()
    dec.add_ignore_region((4.7, 4.9))
    d = dec.deconvolute_spectrum(spectra[0])
    g = np.load(os.path.join(GOLDEN, "expected", "blood_01_water.npz"))
    assert np.array_equal(d.params, g["params"])


@pytest.mark.parametrize("n,p", [(1, 1), (1000, 0), (4097, 3), (131072, 766), (70001, 2048)])
def test_superposition_vec_bit_exact(ctx, n, p):
    rng = np.random.default_rng(n + p)
    x = np.sort(rng.uniform(-5, 15, n))[::-1].copy()
    params = np.stack([rng.uniform(1e-3, 1e3, p), rng.uniform(1e-8, 1e-5, p),
                       rng.uniform(-2, 12, p)], axis=1)
    import metabodecon as md
    got = md.superposition_vec(x, params)
    ref = oracle.superposition_vec(x, params, threads=16)
    assert np.array_equal(got, ref)


def test_reference_unit_superposition(ctx):
    # lorentzian.rs:741-788 through the GPU path
    import metabodecon as md
    L = [md.Lorentzian.from_transformed(1.0, 0.5, -2.0), md.Lorentzian.from_transformed(2.0, 0.75, 0.0),
         md.Lorentzian.from_transformed(1.0, 0.5, 2.0)]
    x = np.array([-5.0 + i for i in range(11)])
    got = md.Lorentzian.par_superposition_vec(x, L)
    assert np.array_equal(got, oracle.superposition_vec(x, [l.parameters() for l in L]))
    trip = [md.Lorentzian.from_transformed(0.03, 0.0009, 4.8),
            md.Lorentzian.from_transformed(0.02, 0.0004, 5.0),
            md.Lorentzian.from_transformed(0.03, 0.0009, 5.2)]
    assert abs(md.Lorentzian.superposition_vec(np.array([5.0]), trip)[0] - 51.466992) <= 1e-6


def test_fused_prep_after_failures_and_other_smoothers(monkeypatch, engine_env):
    """The chain smoother runs k_prep's work itself and never reads the status the
    previous run left; k_flags returns its progress counters to zero. On one
    context: a failing spectrum (NoPeaksDetected), then a good one, the same on
    the lane-pipelined smoother, on k_smooth_small (the 4096-point failing row; fused
    prep on its extra wave; blood_07 is longer and takes the chain), with
    k_prep launched separately, and the chain again --
    every result equal to the oracle."""
    c = nat.Context(0)
    st = oracle.default_settings()
    n = 4096
    xf = np.linspace(14.0, -6.0, n)
    flat = np.full(n, 7.0)
    x, y, sb, cst, _ = load_case("blood_07")
    o = oracle.deconvolute(x, y, sb, cst)
    for smooth, prep in [("chain", None), ("pipe", None), ("small", None), ("chain", "separate"),
                         ("chain", None)]:
        engine_env.setenv("MDG_SMOOTH", smooth)
        if prep:
            engine_env.setenv("MDG_PREP", prep)
        else:
            engine_env.delenv("MDG_PREP", raising=False)
        status, *_ = gpu_batch(c, xf, flat[None, :], [(11.8, -2.2)], st)
        assert status[0] == 1, (smooth, prep)
        status, counts, out, mse = gpu_batch(c, x, y[None, :], [sb], cst)
        assert status[0] == 0, (smooth, prep)
        assert np.array_equal(out[0, : counts[0]], o.params), (smooth, prep)
        assert abs(mse[0] - o.mse) <= MSE_RTOL * abs(o.mse)
    c.close()


def test_error_statuses(ctx):
    import metabodecon as md
    from metabodecon import exceptions as ex
    st = oracle.default_settings()
    n = 4096
    x = np.linspace(14.0, -6.0, n)
    # constant spectrum: no curvature anywhere -> NoPeaksDetected
    flat = np.full(n, 7.0)
    status, *_ = gpu_batch(ctx, x, flat[None, :], [(11.8, -2.2)], st)
    assert status[0] == oracle.deconvolute(x, flat, (11.8, -2.2)).status == 1
    with pytest.raises(ex.NoPeaksDetected):
        md.Deconvoluter().deconvolute_spectrum(md.Spectrum(x, flat, (-2.2, 11.8)))
    # peaks only outside a narrow signal region -> EmptySignalRegion
    rng = np.random.default_rng(1)
    noisy = rng.normal(0, 1, n)
    for sb in [(11.8, 11.79), (1.0, 0.99)]:
        o = oracle.deconvolute(x, noisy, sb)
        status, counts, out, mse = gpu_batch(ctx, x, noisy[None, :], [sb], st)
        assert status[0] == o.status
        if o.status == 0:
            assert np.array_equal(out[0, : counts[0]], o.params)
    # two ignore regions on a decreasing axis: the reference panics in compute_mse
    sim = load_case("sim_01")
    ign = ((3.40, 3.42), (3.45, 3.47))
    o = oracle.deconvolute(sim[0], sim[1], sim[2], st, ignore=ign)
    status, *_ = gpu_batch(ctx, sim[0], sim[1][None, :], [sim[2]], st, ign)
    assert status[0] == o.status == 30
    # detector-only may legitimately select nothing: Ok with zero Lorentzians
    dso = oracle.make_settings(selector="detector_only")
    o = oracle.deconvolute(x, noisy, (11.8, 11.79), dso)
    status, counts, out, mse = gpu_batch(ctx, x, noisy[None, :], [(11.8, 11.79)], dso)
    assert status[0] == o.status
    assert counts[0] == o.params.shape[0]
    if o.status == 0:
        assert abs(mse[0] - o.mse) <= MSE_RTOL * abs(o.mse)


def test_mixed_batch_statuses_are_per_spectrum(ctx):
    st = oracle.default_settings()
    x, y, sb, _, _ = load_case("sim_02")
    flat = np.full_like(y, 3.0)
    status, counts, out, mse = gpu_batch(ctx, x, np.stack([y, flat, y]), [sb] * 3, st)
    assert list(status) == [0, 1, 0]
    g = np.load(os.path.join(GOLDEN, "expected", "sim_02.npz"))
    for k in (0, 2):
        check_against(g["params"], float(g["mse"]), status[k], counts[k], out[k], mse[k])


def test_small_and_odd_shapes(ctx):
    st = oracle.default_settings()
    rng = np.random.default_rng(11)
    for n in [2, 3, 5, 17, 64, 65, 127, 1000, 1023]:
        x = np.linspace(12.0, -4.0, n)
        y = rng.normal(0, 1, n) + 50.0 * np.exp(-((x - 4.0) / 0.3) ** 2)
        sb = (11.8, -2.2) if n > 2 else (12.0, -4.0)
        o = oracle.deconvolute(x, y, sb, st)
        status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st)
        assert status[0] == o.status, n
        if o.status == 0:
            assert np.array_equal(out[0, : counts[0]], o.params)
            assert abs(mse[0] - o.mse) <= MSE_RTOL * abs(o.mse)


@pytest.mark.parametrize("path", ["chain", "pipe", "generic"])
@pytest.mark.parametrize("it,ws", [(1, 2), (2, 4), (3, 3), (5, 7), (8, 5), (10, 3), (3, 31),
                                   (4, 9), (2, 11)])
def test_smoother_settings_sweep(ctx, it, ws, path, monkeypatch, engine_env):
    """Every smoother kernel (chain, lane-pipelined, one lane per spectrum, forced by
    MDG_SMOOTH) against the oracle; (3, 31) and iterations > 8 exercise fallbacks."""
    engine_env.setenv("MDG_SMOOTH", path)
    x, y, sb, _, _ = load_case("blood_05")
    st = oracle.make_settings(smooth_iterations=it, smooth_window=ws)
    o = oracle.deconvolute(x, y, sb, st)
    status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st)
    assert status[0] == o.status
    if o.status == 0:
        assert np.array_equal(out[0, : counts[0]], o.params)
        assert np.array_equal(ctx.last_peaks(0).astype(np.int64), o.selected)


def test_device_synth_matches_host_and_oracle(ctx):
    torch = pytest.importorskip("torch")
    b, n = 3, 131072
    x = torch.empty(n, dtype=torch.float64, device="cuda")
    y = torch.empty((b, n), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    rc = nat.lib().mdg_synth_batch_device(ctx.handle, b, n, 14.8, 20.0, 0, 2048, -1.8, 11.4,
                                          1.0e3, x.data_ptr(), y.data_ptr())
    assert rc == 0
    ctx.synchronize()
    for s in range(b):
        hx, hy, _ = synth_spectrum(s)
        assert np.array_equal(x.cpu().numpy(), hx)
        assert np.array_equal(y[s].cpu().numpy(), hy)
    # device-resident deconvolution of the same batch vs oracle (configs[1] shape)
    sb = torch.tensor([[11.8, -2.2]] * b, dtype=torch.float64, device="cuda")
    cap = 4096
    out = torch.zeros((b, cap, 3), dtype=torch.float64, device="cuda")
    cnt = torch.zeros(b, dtype=torch.int32, device="cuda")
    mse = torch.zeros(b, dtype=torch.float64, device="cuda")
    status = torch.zeros(b, dtype=torch.int32, device="cuda")
    s = nat.default_settings()
    rc = nat.lib().mdg_deconvolute_batch_device(
        ctx.handle, b, n, x.data_ptr(), 0, y.data_ptr(), n, sb.data_ptr(), ctypes.byref(s), None,
        0, out.data_ptr(), cap, cnt.data_ptr(), mse.data_ptr(), status.data_ptr())
    assert rc == 0
    ctx.synchronize()
    for k in range(b):
        g = np.load(os.path.join(GOLDEN, "expected", f"synth_128k_2k_s{k}.npz")) if k < 2 else None
        hx, hy, _ = synth_spectrum(k)
        o = oracle.deconvolute(hx, hy, (11.8, -2.2), threads=16) if g is None else None
        ref_p = g["params"] if g is not None else o.params
        ref_m = float(g["mse"]) if g is not None else o.mse
        check_against(ref_p, ref_m, int(status[k]), int(cnt[k]), out[k].cpu().numpy(),
                      float(mse[k]))


def test_deterministic_bits(ctx):
    x, y, sb, st, _ = load_case("blood_07")
    a = gpu_batch(ctx, x, y[None, :], [sb], st)
    b = gpu_batch(ctx, x, y[None, :], [sb], st)
    assert np.array_equal(a[2], b[2]) and a[3][0] == b[3][0]


def test_rows_past_counts_untouched(ctx):
    """mdg_deconvolute_batch writes only rows below counts[i] (mdgpu.h): the result rows
    come back with a guessed row count (the context's last one), so a call after one
    with more peaks must leave the caller's rows past its own counts alone."""
    big = load_case("synth_128k_2k_s1")
    small = load_case("blood_07")
    gpu_batch(ctx, big[0], big[1][None, :], [big[2]], big[3])  # a large guess
    for rows_x, rows_y, sbs, st in (
            (small[0], small[1][None, :], [small[2]], small[3]),
            (small[0], np.stack([small[1], small[1] * 1.5, small[1]]), [small[2]] * 3, small[3])):
        ys = np.ascontiguousarray(rows_y)
        b, n = ys.shape
        s = nat.Settings()
        for f, _ in nat.Settings._fields_:
            setattr(s, f, getattr(st, f))
        cap = n // 2 + 2
        out = np.full((b, cap, 3), 7.25)
        counts = np.zeros(b, dtype=np.uintp)
        mse = np.zeros(b)
        status = np.zeros(b, dtype=np.intc)
        sbv = np.ascontiguousarray(np.broadcast_to(np.asarray(sbs, dtype=np.float64), (b, 2)))
        rc = nat.lib().mdg_deconvolute_batch(
            ctx.handle, b, n, nat.ptr(np.ascontiguousarray(rows_x)), 0, nat.ptr(ys), n, nat.ptr(sbv),
            ctypes.byref(s), None, 0, nat.ptr(out), cap, nat.ptr(counts, nat._szp), nat.ptr(mse),
            status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        assert rc < 100, nat.strerror(rc)
        for i in range(b):
            k = int(counts[i])
            assert 0 < k < 4000
            assert not np.any(out[i, :k] == 7.25)
            assert np.all(out[i, k:] == 7.25), i


def test_stage_profiling(ctx):
    ctx.reset_stage_times()
    ctx.set_profiling(True)
    x, y, sb, st, _ = load_case("blood_01")
    gpu_batch(ctx, x, y[None, :], [sb], st)
    t = ctx.stage_times()
    ctx.set_profiling(False)
    assert t["fit_superposition"][1] == 10 and t["mse_superposition"][0] > 0


def _smooth_rows(ctx, ys, it, ws):
    """Run the batch (any final status) and read back every smoothed row."""
    xs = np.linspace(14.8, -5.2, ys.shape[1])
    st = oracle.make_settings(smooth_iterations=it, smooth_window=ws)
    gpu_batch(ctx, xs, ys, [(11.8, -2.2)], st)
    return [ctx.last_smoothed(s, ys.shape[1]) for s in range(ys.shape[0])]


@pytest.mark.parametrize("path", ["chain", "pipe", "generic"])
def test_smoothed_rows_bit_exact(ctx, path, monkeypatch, engine_env):
    """Smoothed intensities of every kernel equal the oracle's moving average bit for
    bit (moving_average.rs:53-83), on real spectra and a synthetic 128k one."""
    engine_env.setenv("MDG_SMOOTH", path)
    ys = np.stack([load_case(f"blood_{i:02d}")[1] for i in (1, 7, 16)] + [synth_spectrum(0)[1]])
    for s, row in enumerate(_smooth_rows(ctx, ys, 3, 3)):
        assert np.array_equal(row, oracle.moving_average(ys[s], 3, 3)), s


@pytest.mark.parametrize("ws", [2, 3, 4, 5, 6, 7, 8])
def test_chain_smoother_shapes(ctx, ws, monkeypatch, engine_env):
    """k_smooth_chain at the edges of its range: short spectra (generic head/tail
    blocks only), lengths off the block and group grids, up to 16 passes, batches
    that do not fill the 8-spectrum placement groups."""
    engine_env.setenv("MDG_SMOOTH", "chain")
    rng = np.random.default_rng(ws)
    for n, b, it in [(400, 1, 1), (401, 3, 2), (487, 2, 3), (577, 9, 5), (1000, 1, 16),
                     (4101, 13, 3), (20000, 2, 4)]:
        t = np.linspace(0, 1, n)
        ys = rng.normal(0, 1, (b, n)) * 10.0 ** rng.integers(0, 6, (b, 1)) + 1e4 * np.sin(
            40 * t)[None, :]
        for s, row in enumerate(_smooth_rows(ctx, ys, it, ws)):
            assert np.array_equal(row, oracle.moving_average(ys[s], it, ws)), (n, b, it, s)


def test_chain_smoother_repeated_launches(ctx, monkeypatch, engine_env):
    """Back-to-back launches rewrite the chain's hand-off buffers: a stale line in
    any cache would show as a mismatch in the second and third runs."""
    engine_env.setenv("MDG_SMOOTH", "chain")
    rng = np.random.default_rng(7)
    for rep in range(3):
        ys = rng.normal(0, 1, (5, 131072)) * 1e3 + rep
        for s, row in enumerate(_smooth_rows(ctx, ys, 3, 3)):
            assert np.array_equal(row, oracle.moving_average(ys[s], 3, 3)), (rep, s)


# the library's fit kernels (fit_choice, mdg_kernels.hip); "twf*" are the batch-wide
# tile lists, "tw3s"/"twf3s" single-buffered; ":G" = G workgroups (many tiles each);
# "small" = every iteration in one workgroup per spectrum (k_fit_small, the default for
# N <= 4096; forced on the 131072-point cases it takes its global-row form, P > 512)
FIT_KERNELS = ["tf", "tf12", "tw7", "tw3s", "twf", "twf1", "twf3s", "twf:5", "twf3s:7", "plain", "small"]


@pytest.mark.parametrize("mode", ["fine", "coarse"])
def test_peak_chunkings(ctx, mode, monkeypatch, engine_env):
    """k_peaks over 64-word chunks (small batches) and 256-word chunks (large ones),
    forced by MDG_PEAKS, on a single spectrum and a batch of three: the oracle's
    results either way (peak lists, scores and the selection behind them)."""
    engine_env.setenv("MDG_PEAKS", mode)
    for name in ("blood_03", "sim_03"):
        x, y, sb, st, ign = load_case(name)
        o = oracle.deconvolute(x, y, sb, st, ignore=ign)
        status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st, ignore=ign)
        assert status[0] == o.status, name
        assert np.array_equal(out[0, : counts[0]], o.params), name
    rows, ref = [], []
    for seed in (6, 7, 8):
        x, y = synth_spectrum(seed, n=65536, n_peaks=500 + 200 * seed)[:2]
        rows.append(y)
        ref.append(oracle.deconvolute(x, y, (11.8, -2.2)))
    status, counts, out, mse = gpu_batch(ctx, x, np.stack(rows), [(11.8, -2.2)], oracle.default_settings())
    for s, o in enumerate(ref):
        assert status[s] == o.status == 0
        assert np.array_equal(out[s, : counts[s]], o.params), s


def test_selection_many_signal_peaks(ctx):
    """k_select compacts up to 16 candidates per thread from registers (16384 signal-
    region peaks); a pure-noise spectrum with a wide signal region has ~27k, so its
    workgroup takes the general loop. One batch with a blood spectrum (the register
    path) beside it: both against the oracle, bit for bit."""
    n = 131072
    rng = np.random.default_rng(11)
    x = np.linspace(14.8, -5.2, n)
    noise = rng.normal(size=n) * 100 + 1000
    st = oracle.default_settings()
    bx, by, bsb, bst, _ = load_case("blood_05")
    assert bx.size == n
    for rows, sbs in (([noise], [(14.5, -4.9)]), ([noise, by], [(14.5, -4.9), bsb])):
        ys = np.stack(rows)
        status, counts, out, mse = gpu_batch(ctx, x if len(rows) == 1 else np.stack([x, bx]), ys, sbs, st)
        for k, (yy, sb) in enumerate(zip(rows, sbs)):
            xx = x if k == 0 else bx
            o = oracle.deconvolute(xx, yy, sb, st)
            assert status[k] == o.status == 0
            assert np.array_equal(out[k, : counts[k]], o.params), k
            assert abs(mse[k] - o.mse) <= MSE_RTOL * abs(o.mse), k


def _force_fit(engine_env, path):
    kernel, _, g = path.partition(":")
    engine_env.setenv("MDG_FITSUP", kernel)
    if g:
        engine_env.setenv("MDG_TW_G", g)


@pytest.mark.parametrize("path", FIT_KERNELS)
def test_fit_superposition_kernels(ctx, path, monkeypatch, engine_env):
    """Every fit-superposition kernel the library ships (24- and 63-point term folds,
    one thread per point; forced by MDG_FITSUP) gives the oracle's Lorentzians bit for
    bit, including peak counts that are not multiples of the tiles and chunks."""
    _force_fit(engine_env, path)
    names = ["sim_03", "blood_03", "synth_128k_2k_s1"]
    for name in names:
        x, y, sb, st, ign = load_case(name)
        o = oracle.deconvolute(x, y, sb, st, ignore=ign)
        status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st, ignore=ign)
        assert status[0] == o.status, name
        assert np.array_equal(out[0, : counts[0]], o.params), name
        assert abs(mse[0] - o.mse) <= MSE_RTOL * abs(o.mse), name


@pytest.mark.parametrize("path", FIT_KERNELS)
def test_fit_superposition_kernels_batch(ctx, path, monkeypatch, engine_env):
    """The fit kernels on a batch whose spectra have different peak counts (tail
    tiles, grid-stride loops, per-spectrum range flags) against the oracle."""
    _force_fit(engine_env, path)
    rows, ref = [], []
    for seed in (3, 4, 5):
        x, y = synth_spectrum(seed, n=65536, n_peaks=700 + 300 * seed)[:2]
        rows.append(y)
        ref.append(oracle.deconvolute(x, y, (11.8, -2.2)))
    st = oracle.default_settings()
    status, counts, out, mse = gpu_batch(ctx, x, np.stack(rows), [(11.8, -2.2)], st)
    for s, o in enumerate(ref):
        assert status[s] == o.status == 0
        assert np.array_equal(out[s, : counts[s]], o.params), s
        assert abs(mse[s] - o.mse) <= MSE_RTOL * abs(o.mse), s


@pytest.mark.parametrize("pk", ["20", "30"])
@pytest.mark.parametrize("npt", ["2", "4"])
@pytest.mark.parametrize("near_cap", [None, "8", "0"])
def test_mse_cases(ctx, near_cap, npt, pk, monkeypatch, engine_env):
    """The MSE (k_mse_local, 2 and 4 points per thread, 20 powers at radius 5 and 30
    at radius 3) against the oracle: ignore regions (two in one spectrum), a short
    signal region (sim) and a batch whose spectra differ in peak count; also with a
    tiny near-list capacity (crowded tiles take the kernel's direct sum) and none at
    all (every tile direct)."""
    engine_env.setenv("MDG_MSE_NPT", npt)
    engine_env.setenv("MDG_MSE_PK", pk)
    if near_cap is not None:
        engine_env.setenv("MDG_MSE_NEARCAP", near_cap)
    for name in ["blood_01_water", "blood_02_two_regions_increasing", "sim_05", "synth_128k_2k_s0"]:
        x, y, sb, st, ign = load_case(name)
        o = oracle.deconvolute(x, y, sb, st, ignore=ign)
        status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st, ignore=ign)
        assert status[0] == o.status == 0, name
        assert np.array_equal(out[0, : counts[0]], o.params), name
        assert abs(mse[0] - o.mse) <= MSE_RTOL * abs(o.mse), (name, mse[0], o.mse)
    rows, ref = [], []
    for seed in (6, 7, 8):
        x, y = synth_spectrum(seed, n=65536, n_peaks=500 + 400 * (seed - 6))[:2]
        rows.append(y)
        ref.append(oracle.deconvolute(x, y, (11.8, -2.2)))
    status, counts, out, mse = gpu_batch(ctx, x, np.stack(rows), [(11.8, -2.2)], oracle.default_settings())
    for s, o in enumerate(ref):
        assert status[s] == o.status == 0
        assert np.array_equal(out[s, : counts[s]], o.params), s
        assert abs(mse[s] - o.mse) <= MSE_RTOL * abs(o.mse), s


def _left_fold(acc, terms):
    for t in terms:
        acc = acc + float(t)
    return acc


def test_ordered_sum_window_fold(ctx):
    """The windowed parallel fold behind k_select's SFR mean/variance equals the
    sequential left fold bit for bit, including inputs that defeat its candidate
    windows (a huge first term, then a long tail of terms below half an ulp; wide
    dynamic range; zeros; subnormals; exact ties) and so run its fallback path."""
    rng = np.random.default_rng(11)
    cases = [
        rng.uniform(0, 1e3, 8418),
        rng.exponential(300.0, 5116) ** 2,
        np.concatenate([[1e16], rng.uniform(0, 0.9, 4000)]),
        10.0 ** rng.uniform(-300, 300, 3000),
        np.zeros(500),
        np.concatenate([np.full(100, 5e-324), rng.uniform(0, 1e-310, 900)]),
        np.full(4096, 0.5) * np.arange(4096) % 7,
        rng.uniform(0, 1, 129),
        rng.uniform(0, 1e6, 16384),
        rng.uniform(0, 1e6, 40000),
    ]
    for k, t in enumerate(cases):
        t = np.ascontiguousarray(t, dtype=np.float64)
        out = ctypes.c_double()
        rc = nat.lib().mdg_ordered_sum(ctx.handle, nat.ptr(t), t.size, -0.0, ctypes.byref(out))
        assert rc == 0, nat.strerror(rc)
        ref = _left_fold(-0.0, t)
        assert np.float64(out.value).tobytes() == np.float64(ref).tobytes(), (k, out.value, ref)
    bad = np.array([1.0, -1.0])
    assert nat.lib().mdg_ordered_sum(ctx.handle, nat.ptr(bad), 2, -0.0, ctypes.byref(out)) != 0


def _division_check(ctx, variant, cases, seed, n):
    bad, tested = ctypes.c_uint64(1), ctypes.c_uint64(0)
    rc = nat.lib().mdg_check_division(ctx.handle, variant, cases, seed, n, ctypes.byref(bad),
                                      ctypes.byref(tested))
    assert rc == 0, nat.strerror(rc)
    return bad.value, tested.value


@pytest.mark.parametrize("seed", [0x9E3779B97F4A7C15, 20261016])
def test_fast_division_matches_ieee(ctx, seed):
    """div_rn (reciprocal + two Newton steps + residual correction: the compiler's
    own '/' expansion minus its no-op scaling wrappers) is the divider of every
    FAST-path evaluation in the fit and superposition_vec. On operands in
    [2^-200, 2^200] (the range the fast flags gate) it must round exactly like
    IEEE '/': 2^32 seeded random pairs per seed (a quarter with trailing-ones /
    single-bit mantissas), and 2^31 candidates of the constructed near-midpoint
    family (quotients 2^-53 ulp from a tie -- the only inputs on which a
    not-quite-correct reciprocal can misround)."""
    bad, tested = _division_check(ctx, 0, 0, seed, 1 << 32)
    assert tested == 1 << 32 and bad == 0
    bad, tested = _division_check(ctx, 0, 1, seed, 1 << 31)
    assert tested > (1 << 31) // 3 and bad == 0, (bad, tested)


def test_one_newton_division_is_not_exact_on_hard_cases(ctx):
    """Power check of the hard-case family: the one-Newton-step quotient (kept for
    the MSE only, which the tests compare at 1e-12 relative) does misround on
    constructed near-midpoint pairs, while it almost never does on random pairs
    -- the reason it was retired from the bit-exact paths."""
    bad_hard, tested = _division_check(ctx, 1, 1, 5, 1 << 28)
    assert tested > 0 and bad_hard > 0, (bad_hard, tested)


def test_device_graph_replay(ctx, monkeypatch, engine_env):
    """With MDG_GRAPHS=1 mdg_deconvolute_batch_device replays a cached hipGraph for
    repeated argument sets: refilling the same device buffers with other spectra
    must still give the oracle's results on the replayed launch, and the same bits
    as the uncaptured pipeline (MDG_GRAPHS=0, the default)."""
    torch = pytest.importorskip("torch")
    engine_env.setenv("MDG_GRAPHS", "1")
    names = [["blood_02", "blood_04"], ["blood_09", "blood_11"], ["blood_02", "blood_04"]]
    n = load_case("blood_02")[1].size
    b = 2
    dev = "cuda"
    x = torch.empty((b, n), dtype=torch.float64, device=dev)
    y = torch.empty((b, n), dtype=torch.float64, device=dev)
    sb = torch.empty((b, 2), dtype=torch.float64, device=dev)
    cap = n // 2 + 2
    out = torch.zeros((b, cap, 3), dtype=torch.float64, device=dev)
    cnt = torch.zeros(b, dtype=torch.int32, device=dev)
    mse = torch.zeros(b, dtype=torch.float64, device=dev)
    status = torch.zeros(b, dtype=torch.int32, device=dev)
    s = nat.default_settings()

    def run():
        rc = nat.lib().mdg_deconvolute_batch_device(
            ctx.handle, b, n, x.data_ptr(), n, y.data_ptr(), n, sb.data_ptr(), ctypes.byref(s),
            None, 0, out.data_ptr(), cap, cnt.data_ptr(), mse.data_ptr(), status.data_ptr())
        assert rc == 0
        ctx.synchronize()
        return [(int(status[k]), out[k, : int(cnt[k])].cpu().numpy().copy(), float(mse[k]))
                for k in range(b)]

    results = []
    for batch in names:
        cases = [load_case(nm) for nm in batch]
        for k, (cx, cy, csb, _, _) in enumerate(cases):
            x[k] = torch.from_numpy(cx)
            y[k] = torch.from_numpy(cy)
            sb[k] = torch.tensor(csb, dtype=torch.float64)
        torch.cuda.synchronize()
        got = run()
        for (cx, cy, csb, cst, _), (st_, p, m) in zip(cases, got):
            o = oracle.deconvolute(cx, cy, csb, cst)
            assert st_ == o.status and np.array_equal(p, o.params)
            assert abs(m - o.mse) <= MSE_RTOL * abs(o.mse)
        results.append(got)
    engine_env.setenv("MDG_GRAPHS", "0")
    plain = run()  # last batch again, uncaptured
    for (s1, p1, m1), (s2, p2, m2) in zip(results[-1], plain):
        assert s1 == s2 and np.array_equal(p1, p2) and m1 == m2


def test_graph_key_follows_kernel_overrides(monkeypatch, engine_env):
    """A cached pipeline graph is keyed by the kernel-choice overrides too: the
    same device buffers with MDG_SMOOTH / MDG_FITSUP switched between calls launch
    the newly chosen kernels (reported by the engine), each call equal to the
    oracle."""
    torch = pytest.importorskip("torch")
    engine_env.setenv("MDG_GRAPHS", "1")
    cx, cy, csb, cst, _ = load_case("blood_03")
    n = cy.size
    c = nat.Context(0)
    x = torch.from_numpy(cx).cuda()
    y = torch.from_numpy(cy).cuda()
    sb = torch.tensor([csb], dtype=torch.float64, device="cuda")
    cap = n // 2 + 2
    out = torch.zeros((1, cap, 3), dtype=torch.float64, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    mse = torch.zeros(1, dtype=torch.float64, device="cuda")
    status = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = nat.default_settings()
    o = oracle.deconvolute(cx, cy, csb, cst)
    seen = []
    for sm_k, fit_k in [("chain", "tw7"), ("pipe", "tw7"), ("chain", "plain"), ("chain", "tw7")]:
        engine_env.setenv("MDG_SMOOTH", sm_k)
        engine_env.setenv("MDG_FITSUP", fit_k)
        rc = nat.lib().mdg_deconvolute_batch_device(
            c.handle, 1, n, x.data_ptr(), 0, y.data_ptr(), n, sb.data_ptr(), ctypes.byref(s), None,
            0, out.data_ptr(), cap, cnt.data_ptr(), mse.data_ptr(), status.data_ptr())
        assert rc == 0
        c.synchronize()
        k = c.stage_kernels()
        seen.append((k["smooth"], k["fit_superposition"]))
        assert int(status[0]) == 0
        assert np.array_equal(out[0, : int(cnt[0])].cpu().numpy(), o.params)
        assert abs(float(mse[0]) - o.mse) <= MSE_RTOL * abs(o.mse)
    c.close()
    assert seen[0][0].startswith("k_smooth_chain") and seen[1][0].startswith("k_smooth_pipe")
    assert seen[2][1] == "k_fit_sup" and seen[3] == seen[0]


@pytest.mark.parametrize("name", ["sim_01", "sim_07"])
def test_optimize_settings_matches_exhaustive_oracle(name):
    """Deconvoluter.optimize_settings (GPU: 27 batched pipelines + exact tie
    check) picks the same setting as an exhaustive oracle search over the
    reference's 810 combinations (first minimum, deconvoluter.rs:762-825) and
    returns that setting's MSE bit for bit (summed in the reference's order)."""
    import metabodecon as md
    from metabodecon import exceptions as mexc
    x, y, sb, _, ign = load_case(name)
    best, first_err = None, None
    for it in range(2, 11):
        for ws in (3, 5, 7):
            for c in range(10):
                thr = 5.0 + (c * (8.0 - 5.0)) / 9.0
                for fit in (5, 10, 15):
                    st = oracle.make_settings(smooth_iterations=it, smooth_window=ws, threshold=thr,
                                              fit_iterations=fit)
                    r = oracle.deconvolute(x, y, sb, st, ignore=ign)
                    if r.status and first_err is None:
                        first_err = r.status
                    if r.status == 0 and (best is None or r.mse < best[0]):
                        best = (r.mse, it, ws, thr, fit)
    d = md.Deconvoluter()
    spec = md.Spectrum(x, y, sb)
    if first_err is not None:
        with pytest.raises(mexc.DeconvolutionError):
            d.optimize_settings(spec)
        return
    mse = d.optimize_settings(spec)
    assert mse == best[0]
    s = d.settings
    assert (s.smooth_iterations, s.smooth_window, s.fit_iterations) == (best[1], best[2], best[4])
    assert s.threshold == best[3]


def test_jcampdx_and_serde_inputs_through_the_device(tmp_path):
    """Rows f3/f4 feeding the hot path: a spectrum read from the reference's
    JCAMP-DX file, and the same spectrum after a MessagePack and a JSON round
    trip (axis rebuilt as start + i * step), deconvolute bit-identically to the
    oracle on the same arrays; the Deconvolution written as MessagePack reads
    back as Lorentzian::new(sf * hw, hw^2, maxp)."""
    import gzip
    import shutil
    import metabodecon as md
    src = os.path.join(GOLDEN, "jcampdx", "blood_01.dx.gz")
    p = str(tmp_path / "blood_01.dx")
    with gzip.open(src, "rb") as g, open(p, "wb") as f:
        shutil.copyfileobj(g, f)
    s = md.Spectrum.read_jcampdx(p, (-2.2, 11.8))
    s.write_bin(str(tmp_path / "s.bin"))
    s.write_json(str(tmp_path / "s.json"))
    dec = md.Deconvoluter()
    dec.add_ignore_region((4.7, 4.9))
    for sp in (s, md.Spectrum.read_bin(str(tmp_path / "s.bin")),
               md.Spectrum.read_json(str(tmp_path / "s.json"))):
        d = dec.deconvolute_spectrum(sp)
        o = oracle.deconvolute(sp.chemical_shifts, sp.intensities, sp.signal_boundaries,
                               ignore=[(4.7, 4.9)], threads=16)
        assert o.status == 0
        assert np.array_equal(d.params, o.params)
        assert abs(d.mse - o.mse) <= MSE_RTOL * abs(o.mse)
    d.write_bin(str(tmp_path / "d.bin"))
    r = md.Deconvolution.read_bin(str(tmp_path / "d.bin"))
    hw = np.sqrt(d.params[:, 1])
    sf = d.params[:, 0] / hw
    assert np.array_equal(r.params, np.stack([sf * hw, hw * hw, d.params[:, 2]], axis=1))
    assert r.mse == d.mse


def test_graph_cache_survives_workspace_growth(ctx, monkeypatch, engine_env):
    """A cached pipeline graph bakes the workspace layout. Growing the workspace
    (a larger batch, then a longer spectrum on a fresh context) must drop the cached
    graphs, so B=1 -> B=2 -> B=1 -> longer N -> B=1 on the same tensors keeps
    giving the oracle's results (stale graph after reallocation)."""
    torch = pytest.importorskip("torch")
    engine_env.setenv("MDG_GRAPHS", "1")
    c = nat.Context(0)
    try:
        names = ["sim_04", "sim_09"]
        cases = [load_case(nm) for nm in names]
        n = cases[0][1].size
        dev = "cuda"
        x = torch.from_numpy(np.stack([cc[0] for cc in cases])).to(dev)
        y = torch.from_numpy(np.stack([cc[1] for cc in cases])).to(dev)
        sb = torch.tensor([cc[2] for cc in cases], dtype=torch.float64, device=dev)
        cap = n // 2 + 2
        out = torch.zeros((2, cap, 3), dtype=torch.float64, device=dev)
        cnt = torch.zeros(2, dtype=torch.int32, device=dev)
        mse = torch.zeros(2, dtype=torch.float64, device=dev)
        status = torch.zeros(2, dtype=torch.int32, device=dev)
        s = nat.default_settings()
        refs = [oracle.deconvolute(cc[0], cc[1], cc[2], cc[3]) for cc in cases]

        def run(b):
            out.zero_(); mse.zero_()
            torch.cuda.synchronize()
            rc = nat.lib().mdg_deconvolute_batch_device(
                c.handle, b, n, x.data_ptr(), n, y.data_ptr(), n, sb.data_ptr(), ctypes.byref(s),
                None, 0, out.data_ptr(), cap, cnt.data_ptr(), mse.data_ptr(), status.data_ptr())
            assert rc == 0, nat.strerror(rc)
            c.synchronize()
            for k in range(b):
                o = refs[k]
                assert int(status[k]) == o.status == 0
                assert np.array_equal(out[k, : int(cnt[k])].cpu().numpy(), o.params)
                assert abs(float(mse[k]) - o.mse) <= MSE_RTOL * abs(o.mse), (b, k)

        for b in (1, 2, 1, 2, 1):
            run(b)
        # a longer spectrum through the host API grows the arena under the cached graphs
        bx, by, bsb, bst, _ = load_case("blood_03")
        gpu_batch(c, bx, by[None, :], [bsb], bst)
        run(1)
        run(2)
    finally:
        c.close()


def test_par_deconvolute_spectra_rccl_world1():
    """The multi-GPU product path itself (metabodecon.distributed) on the box's GPU:
    nccl (RCCL) process group of world size 1, the shard run through the
    single-process host path (Deconvoluter._run), the packed results gathered over
    RCCL (distributed.gather_host); results equal the goldens, and an injected
    failure raises the first error in order."""
    import socket
    import torch
    import torch.distributed as dist
    import metabodecon as md
    from metabodecon import exceptions as mexc
    from metabodecon.distributed import par_deconvolute_spectra
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        spectra = md.Spectrum.read_bruker_set(os.path.join(GOLDEN, "bruker", "blood"), 10, 10,
                                              (-2.2, 11.8))[:6]
        decs = par_deconvolute_spectra(md.Deconvoluter(), spectra)
        for k, d in enumerate(decs):
            g = np.load(os.path.join(GOLDEN, "expected", f"blood_{k + 1:02d}.npz"))
            assert np.array_equal(d.params, g["params"])
            assert abs(d.mse - float(g["mse"])) <= MSE_RTOL * abs(float(g["mse"]))
        flat = md.Spectrum(spectra[0].chemical_shifts, np.full(len(spectra[0]), 5.0),
                           (-2.2, 11.8))
        with pytest.raises(mexc.NoPeaksDetected):
            par_deconvolute_spectra(md.Deconvoluter(), [spectra[1], flat, spectra[2]])
        # ragged lengths through the same path: one device batch per length
        ragged, expect = _ragged_set()
        decs = par_deconvolute_spectra(md.Deconvoluter(), ragged)
        for d, (params, mse) in zip(decs, expect):
            assert np.array_equal(d.params, params)
            assert abs(d.mse - mse) <= MSE_RTOL * abs(mse)
    finally:
        dist.destroy_process_group()


def _ragged_set():
    """Spectra of four lengths interleaved: blood (131072 points), sim (2048-point
    simulated), blood_05 cut to its first 100 001 points, blood_06 cut to 70 001;
    expected (params, mse) from the goldens or the oracle."""
    import metabodecon as md
    spectra, expect = [], []
    for k in range(1, 5):
        for name in (f"blood_{k:02d}", f"sim_{k:02d}"):
            x, y, sb, _, _ = load_case(name)
            g = np.load(os.path.join(GOLDEN, "expected", f"{name}.npz"))
            spectra.append(md.Spectrum(x, y, sb))
            expect.append((g["params"], float(g["mse"])))
        if k <= 2:
            x, y, _, _, _ = load_case(f"blood_{k + 4:02d}")
            m = 100001 if k == 1 else 70001
            x, y = x[:m].copy(), y[:m].copy()
            sb = (11.8, float(x[-1]) + 1.0)
            o = oracle.deconvolute(x, y, sb, threads=16)
            assert o.status == 0
            spectra.append(md.Spectrum(x, y, sb))
            expect.append((o.params, o.mse))
    return spectra, expect


def test_ragged_lengths_through_the_python_surface():
    """Deconvoluter.par_deconvolute_spectra on a set of four interleaved lengths
    (one batched pipeline per length, each cut over the lanes): every result in
    input order, bit for bit."""
    import metabodecon as md
    spectra, expect = _ragged_set()
    decs = md.Deconvoluter().par_deconvolute_spectra(spectra)
    assert len(decs) == len(spectra)
    for d, (params, mse) in zip(decs, expect):
        assert np.array_equal(d.params, params)
        assert abs(d.mse - mse) <= MSE_RTOL * abs(mse)


def test_graph_repoint_in_flight_bit_exact(monkeypatch, engine_env):
    """One cached pipeline graph serves calls on distinct device arrays
    (mdg_capi.hip repoint_graph): every call here passes its own x/y/sb rows and
    writes straight into its own result rows, and all calls are enqueued on two
    contexts before any synchronisation, so a graph's node arguments are
    rewritten while earlier launches of it are still queued or running (the
    CUDA/HIP contract: launches already enqueued are not affected). Every call
    must equal the oracle bit for bit, and the MSE within 1e-12."""
    torch = pytest.importorskip("torch")
    engine_env.setenv("MDG_GRAPHS", "1")
    names = ["blood_02", "blood_05", "blood_07", "blood_11", "blood_13", "blood_16"]
    cases = [load_case(nm) for nm in names]
    refs = [oracle.deconvolute(c[0], c[1], c[2], c[3]) for c in cases]
    dev = torch.device("cuda", 0)
    n = cases[0][1].size
    assert all(c[1].size == n for c in cases)
    cap = n // 2 + 2
    X = torch.from_numpy(np.stack([c[0] for c in cases])).to(dev)
    Y = torch.from_numpy(np.stack([c[1] for c in cases])).to(dev)
    SB = torch.tensor([c[2] for c in cases], dtype=torch.float64, device=dev)
    ctxs = [nat.Context(0) for _ in range(2)]
    try:
        s = nat.default_settings()
        steps = 5 * len(cases)
        res_out = torch.zeros((steps, cap, 3), dtype=torch.float64, device=dev)
        res_cnt = torch.zeros(steps, dtype=torch.int32, device=dev)
        res_mse = torch.zeros(steps, dtype=torch.float64, device=dev)
        res_st = torch.full((steps,), -1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        for k in range(steps):
            c = ctxs[k % 2]
            j = (k * 5) % len(cases)
            rc = nat.lib().mdg_deconvolute_batch_device(
                c.handle, 1, n, X[j].data_ptr(), 0, Y[j].data_ptr(), n, SB[j].data_ptr(),
                ctypes.byref(s), None, 0, res_out[k].data_ptr(), cap, res_cnt[k].data_ptr(),
                res_mse[k].data_ptr(), res_st[k].data_ptr())
            assert rc == 0, nat.strerror(rc)
        for c in ctxs:
            c.synchronize()
        for k in range(steps):
            o = refs[(k * 5) % len(cases)]
            assert int(res_st[k]) == o.status == 0, k
            cnt = int(res_cnt[k])
            assert np.array_equal(res_out[k, :cnt].cpu().numpy(), o.params), k
            assert abs(float(res_mse[k]) - o.mse) <= 1e-12 * abs(o.mse), k
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("graphs", ["0", "1"])
def test_concurrent_contexts_stream_bit_exact(graphs, monkeypatch, engine_env):
    """The bench's stream mode: 6 contexts, each on its own stream,
    run their pipelines (launched directly, or replayed as captured graphs with
    MDG_GRAPHS=1) on a stream of distinct spectra (input row
    refilled on the context stream before each replay, results copied out after
    it), all enqueued before any synchronisation so the pipelines overlap on the
    GPU. Every spectrum's Lorentzians must equal the oracle's bit for bit: no
    workspace or counter is shared between concurrent contexts, and the
    whole-CU chain smoother and the term-fold fit stay exact when other
    pipelines run beside them."""
    torch = pytest.importorskip("torch")
    engine_env.setenv("MDG_GRAPHS", graphs)
    names = ["blood_02", "blood_05", "blood_07", "blood_11", "blood_13", "blood_16",
             "sim_02", "sim_05", "sim_08", "sim_11", "sim_14", "sim_16"]
    cases = [load_case(nm) for nm in names]
    refs = [oracle.deconvolute(c[0], c[1], c[2], c[3]) for c in cases]
    dev = torch.device("cuda", 0)
    by_n: dict = {}
    for k, c in enumerate(cases):
        by_n.setdefault(c[1].size, []).append(k)
    ctxs = [nat.Context(0) for _ in range(6)]
    try:
        s = nat.default_settings()
        for n, idx in by_n.items():
            cap = n // 2 + 2
            X = torch.from_numpy(np.stack([cases[k][0] for k in idx])).to(dev)
            Y = torch.from_numpy(np.stack([cases[k][1] for k in idx])).to(dev)
            SB = torch.tensor([cases[k][2] for k in idx], dtype=torch.float64, device=dev)
            slots = []
            for c in ctxs:
                st = torch.cuda.ExternalStream(c.stream(), device=dev)
                slots.append(dict(c=c, st=st, x=torch.empty(n, dtype=torch.float64, device=dev),
                                  y=torch.empty(n, dtype=torch.float64, device=dev),
                                  sb=torch.empty(2, dtype=torch.float64, device=dev),
                                  out=torch.zeros((1, cap, 3), dtype=torch.float64, device=dev),
                                  cnt=torch.zeros(1, dtype=torch.int32, device=dev),
                                  mse=torch.zeros(1, dtype=torch.float64, device=dev),
                                  status=torch.zeros(1, dtype=torch.int32, device=dev)))
            steps = 4 * len(idx)
            res_out = torch.zeros((steps, cap, 3), dtype=torch.float64, device=dev)
            res_cnt = torch.zeros(steps, dtype=torch.int32, device=dev)
            res_st = torch.full((steps,), -1, dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            for k in range(steps):  # round-robin over contexts, nothing synchronised
                sl = slots[k % len(slots)]
                j = k % len(idx)
                with torch.cuda.stream(sl["st"]):
                    sl["x"].copy_(X[j]); sl["y"].copy_(Y[j]); sl["sb"].copy_(SB[j])
                    rc = nat.lib().mdg_deconvolute_batch_device(
                        sl["c"].handle, 1, n, sl["x"].data_ptr(), 0, sl["y"].data_ptr(), n,
                        sl["sb"].data_ptr(), ctypes.byref(s), None, 0, sl["out"].data_ptr(), cap,
                        sl["cnt"].data_ptr(), sl["mse"].data_ptr(), sl["status"].data_ptr())
                    assert rc == 0, nat.strerror(rc)
                    res_out[k].copy_(sl["out"][0]); res_cnt[k].copy_(sl["cnt"][0])
                    res_st[k].copy_(sl["status"][0])
            torch.cuda.synchronize()
            for k in range(steps):
                o = refs[idx[k % len(idx)]]
                assert int(res_st[k]) == o.status == 0, (n, k)
                c = int(res_cnt[k])
                assert np.array_equal(res_out[k, :c].cpu().numpy(), o.params), (n, k)
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("selector,forced", [("noise_score", None), ("detector_only", None),
                                             ("detector_only", "small")])
def test_small_spectra_take_the_one_launch_fit(ctx, selector, forced, monkeypatch, engine_env):
    """N <= 4096 with the noise-score selector (the sim spectra, 2048 points, ~26 peaks;
    the reference's benchmark case at sb (3.34, 3.56)): the whole fit runs in one
    k_fit_small launch per call -- its term-parallel form (3 P^2 <= 6144) -- single and
    batched, bit-identical to the oracle, MSE within 1e-12. Detector-only keeps ~250
    peaks: the engine takes the tile fits; forced onto k_fit_small it runs the
    per-point LDS form (P <= 512)."""
    if forced:
        engine_env.setenv("MDG_FITSUP", forced)
    want = "k_fit_small" if (selector == "noise_score" or forced) else None
    st = oracle.make_settings(selector=selector)
    names = [f"sim_{i:02d}_harness" for i in (1, 2, 11)]
    data = [load_case(n) for n in names]
    for x, y, sb, _, _ in data[:1]:
        o = oracle.deconvolute(x, y, sb, st)
        status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st)
        k = ctx.stage_kernels()["fit_superposition"]
        assert k == want if want else k != "k_fit_small", k
        check_against(o.params, o.mse, status[0], counts[0], out[0], mse[0])
    xs = np.stack([d[0] for d in data])
    ys = np.stack([d[1] for d in data])
    status, counts, out, mse = gpu_batch(ctx, xs, ys, [d[2] for d in data], st)
    k = ctx.stage_kernels()["fit_superposition"]
    assert k == want if want else k != "k_fit_small", k
    for k, (x, y, sb, _, _) in enumerate(data):
        o = oracle.deconvolute(x, y, sb, st)
        check_against(o.params, o.mse, status[k], counts[k], out[k], mse[k])


@pytest.mark.parametrize("n,b,it,ws", [(192, 1, 1, 2), (193, 3, 2, 2), (500, 2, 3, 3), (2048, 4, 3, 3),
                                       (2048, 1, 10, 7), (3001, 5, 15, 31), (4096, 2, 4, 32),
                                       (4096, 1, 3, 5), (1000, 2, 9, 4)])
def test_small_smoother_shapes(ctx, n, b, it, ws, monkeypatch, engine_env):
    """k_smooth_small (N <= 4096: one workgroup per spectrum, one wave per pass, the
    passes handing 16-tick blocks over through LDS rings): smoothed rows equal the
    oracle's moving average bit for bit at the edges of its range -- the shortest rows
    it takes, lengths off the 16-tick grid, 1 to 15 passes, windows 2 to 32. Selected
    with MDG_SMOOTH=small: measured slower than k_smooth_chain, not the default."""
    rng = np.random.default_rng(n + ws)
    t = np.linspace(0, 1, n)
    ys = rng.normal(0, 1, (b, n)) * 10.0 ** rng.integers(0, 6, (b, 1)) + 1e4 * np.sin(40 * t)[None, :]
    engine_env.setenv("MDG_SMOOTH", "small")
    rows = _smooth_rows(ctx, ys, it, ws)
    assert ctx.stage_kernels()["smooth"] == "k_smooth_small"
    for s, row in enumerate(rows):
        assert np.array_equal(row, oracle.moving_average(ys[s], it, ws)), (n, b, it, ws, s)


@pytest.mark.parametrize("detect", ["fused", "separate"])
def test_small_spectra_detection_inside_select(ctx, detect, engine_env):
    """Spectra of <= 4096 points run the detection inside k_select's workgroup
    (k_flags' predicates and k_peaks' word scans and scores over the row staged in LDS;
    MDG_DETECT=separate keeps the two launches): the 16 sim spectra at the harness's
    boundaries as one batch equal their goldens and the detected triples the oracle's;
    an ignore region inside the signal region, 4096 noisy points whose ~1500 peaks send
    the selection's folds down the windowed path, and the statuses the detection and
    selection raise (no peaks, no signal-free peaks, no signal peaks), equal the
    oracle's."""
    engine_env.setenv("MDG_DETECT", detect)
    data = [load_case(f"sim_{k:02d}_harness") for k in range(1, 17)]
    x, st = data[0][0], data[0][3]
    ys = np.stack([d[1] for d in data])
    status, counts, out, mse = gpu_batch(ctx, x, ys, [d[2] for d in data], st)
    want = "k_select<1024, det>" if detect == "fused" else "k_flags+k_peaks<64>"
    assert ctx.stage_kernels()["detect"] == want
    for k in range(16):
        g = np.load(os.path.join(GOLDEN, "expected", f"sim_{k + 1:02d}_harness.npz"))
        check_against(g["params"], float(g["mse"]), status[k], counts[k], out[k], mse[k])
    det = ctx.last_peaks(15, "detected").astype(np.int64)
    l, c, r = oracle.detect_peaks(oracle.second_derivative(oracle.moving_average(ys[15], 3, 3)))
    assert np.array_equal(det, np.stack([l, c, r], axis=1))
    # an ignore region over part of the signal region
    sb = data[0][2]
    ign = ((3.40, 3.45),)
    o = oracle.deconvolute(x, ys[0], sb, st, ignore=ign)
    status, counts, out, mse = gpu_batch(ctx, x, ys[:1], [sb], st, ignore=ign)
    check_against(o.params, o.mse, status[0], counts[0], out[0], mse[0], o.status)
    # 4096 points of noise around a few peaks, a narrow signal region: > 1024
    # signal-free-region scores, so the selection's folds take the windowed path
    rng = np.random.default_rng(11)
    n4 = 4096
    x4 = np.linspace(10.0, 0.0, n4)
    t4 = np.arange(n4, dtype=np.float64)
    y4 = rng.normal(0, 1, n4) + sum(3e3 / (1.0 + ((t4 - c0) / 4.0) ** 2) for c0 in (2000, 2050, 2110))
    st4 = oracle.make_settings(smoother="identity")  # the noise peaks unsmoothed: ~1500
    o = oracle.deconvolute(x4, y4, (5.3, 4.6), st4)
    assert o.status == 0 and o.n_detected > 1400
    status, counts, out, mse = gpu_batch(ctx, x4, y4[None, :], [(5.3, 4.6)], st4)
    check_against(o.params, o.mse, status[0], counts[0], out[0], mse[0])
    # statuses: a flat row, peaks only inside the signal region, peaks only outside it
    n = x.size
    t = np.arange(n, dtype=np.float64)
    lor = lambda c0: 1e4 / (1.0 + ((t - c0) / 3.0) ** 2)
    inside = float(np.searchsorted(-x, -0.5 * (sb[0] + sb[1])))
    rows = np.stack([np.full(n, 5.0), lor(inside), lor(200.0) + lor(1800.0)])
    status, counts, out, mse = gpu_batch(ctx, x, rows, [sb], st)
    for k in range(rows.shape[0]):
        o = oracle.deconvolute(x, rows[k], sb, st)
        assert status[k] == o.status, (k, status[k], o.status)
        assert o.status != 0, k


def _random_small_case(seed, n_range=(48, 4097)):
    """A small spectrum of random shape (N 48..4096, a few Lorentzians over noise, a
    random signal region, sometimes an ignore region, random smoothing, threshold and
    iteration count) for the small-spectrum kernels (fused detection, k_fit_small)."""
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(*n_range))
    lo, hi = sorted(rng.uniform(-1.0, 12.0, 2))
    hi = lo + max(hi - lo, 0.5)
    desc = rng.random() < 0.7
    x = np.linspace(hi, lo, n) if desc else np.linspace(lo, hi, n)
    t = np.arange(n, dtype=np.float64)
    y = rng.normal(0.0, 10.0 ** rng.uniform(-1, 1), n)
    a0, b0 = np.sort(rng.uniform(0.15, 0.85, 2))
    for _ in range(int(rng.integers(1, 12))):  # most of them inside the signal region
        f = rng.uniform(a0, max(b0, a0 + 0.05)) if rng.random() < 0.7 else rng.uniform(0, 1)
        c0, wd = ((1.0 - f) if desc else f) * (n - 1), rng.uniform(1.0, max(1.5, n / 60))
        y += 10.0 ** rng.uniform(1, 4) / (1.0 + ((t - c0) / wd) ** 2)
    sb = (lo + a0 * (hi - lo), lo + max(b0, a0 + 0.05) * (hi - lo))
    if desc:
        sb = sb[::-1]
    ign = ()
    if rng.random() < 0.3:
        m = 0.5 * (sb[0] + sb[1])
        ign = ((m, m + 0.02 * (hi - lo)),)
    st = oracle.make_settings(smooth_iterations=int(rng.integers(1, 5)),
                              smooth_window=int(rng.integers(2, 8)),
                              threshold=float(rng.uniform(0.5, 4.0)),
                              fit_iterations=int(rng.integers(1, 16)))
    return x, y, sb, st, ign


@pytest.mark.parametrize("seed", range(40))
def test_small_spectra_random_shapes(ctx, seed):
    """Random small spectra through the default small-spectrum path (the detection
    inside k_select, k_fit_small, k_mse_local) against the oracle: status, selected
    parameters bit for bit, MSE within MSE_RTOL -- whatever the length, axis
    direction, signal region, ignore region and settings draw."""
    x, y, sb, st, ign = _random_small_case(seed)
    o = oracle.deconvolute(x, y, sb, st, ignore=ign)
    status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st, ignore=ign)
    check_against(o.params, o.mse, status[0], counts[0], out[0], mse[0], o.status)


@pytest.mark.parametrize("seed", range(12))
def test_random_shapes_beyond_the_small_path(ctx, seed):
    """The same random shapes at 4097..60000 points (the general path: k_flags,
    k_peaks, k_select, the batch-size fit kernels) against the oracle."""
    x, y, sb, st, ign = _random_small_case(500 + seed, (4097, 60001))
    o = oracle.deconvolute(x, y, sb, st, ignore=ign)
    status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st, ignore=ign)
    check_against(o.params, o.mse, status[0], counts[0], out[0], mse[0], o.status)


@pytest.mark.parametrize("peaks", ["fine", "coarse"])
@pytest.mark.parametrize("detect", ["fused", "separate"])
def test_detection_with_borders_beyond_the_chunk(ctx, peaks, detect, engine_env):
    """k_peaks with the predicates inside (the default) holds the masks of its chunk
    and one word either side; a border farther away is found on the smoothed row. Broad
    noise-free Lorentzians (half-widths of thousands of points) over narrow ones put
    borders several chunks away: the detected triples equal the oracle's, and so does
    the whole deconvolution, on both chunk sizes, against the separate k_flags."""
    engine_env.setenv("MDG_PEAKS", peaks)
    engine_env.setenv("MDG_DETECT", detect)
    n = 131072
    t = np.arange(n, dtype=np.float64)
    x = np.linspace(14.8, -5.2, n)
    rng = np.random.default_rng(5)
    y = np.zeros(n)
    for c0, wd, amp in [(15000, 9000.0, 1e6), (75000, 12000.0, 8e5), (110000, 7000.0, 6e5)]:
        y += amp / (1.0 + ((t - c0) / wd) ** 2)
    for c0 in rng.uniform(40000, 56000, 12):
        y += rng.uniform(1e3, 1e5) / (1.0 + ((t - c0) / rng.uniform(3, 40)) ** 2)
    st = oracle.default_settings()
    sb = (11.8, -2.2)
    o = oracle.deconvolute(x, y, sb, st)
    status, counts, out, mse = gpu_batch(ctx, x, y[None, :], [sb], st)
    want = {("fused", "fine"): "k_peaks<64, flags>", ("fused", "coarse"): "k_peaks<256, flags>",
            ("separate", "fine"): "k_flags+k_peaks<64>", ("separate", "coarse"): "k_flags+k_peaks<256>"}
    assert ctx.stage_kernels()["detect"] == want[(detect, peaks)]
    det = ctx.last_peaks(0, "detected").astype(np.int64)
    l, c, r = oracle.detect_peaks(oracle.second_derivative(oracle.moving_average(y, 3, 3)))
    assert np.array_equal(det, np.stack([l, c, r], axis=1))
    far = (np.abs(r - c) > 4200) | (np.abs(c - l) > 4200)
    assert far.any()  # some border lies beyond a fine chunk's window
    check_against(o.params, o.mse, status[0], counts[0], out[0], mse[0], o.status)


def _same_bits_or_nan(a, b):
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint64), b[~nb].view(np.uint64))


@pytest.mark.parametrize("path", ["chain", "small", "pipe"])
def test_smoothers_on_non_finite_rows(ctx, path, engine_env):
    """Intensities are not checked for finiteness (neither here nor in the reference),
    so infinities and NaNs reach the moving average: every smoother keeps the IEEE
    results of the reference's adds -- NaN where the oracle has NaN, the same bits
    elsewhere. For k_smooth_small this is its redo path: a 16-tick DPP block whose sum
    went non-finite is recomputed tick by tick (its 0/1 capture would turn inf * 0 into
    NaN)."""
    engine_env.setenv("MDG_SMOOTH", path)
    n = 2048
    rng = np.random.default_rng(7)
    ys = rng.normal(0, 1, (4, n)) + 1e3 * np.sin(np.linspace(0, 30, n))[None, :]
    ys[0, n - 40] = np.nan
    ys[1, n - 100] = np.inf
    ys[1, n - 60] = -np.inf
    ys[2, 700:703] = 1.5e308  # the running sum overflows mid-row and stays infinite
    ys[3, 1000] = -np.inf
    rows = _smooth_rows(ctx, ys, 3, 5)
    if path == "small":
        assert ctx.stage_kernels()["smooth"] == "k_smooth_small"
    for s, row in enumerate(rows):
        assert _same_bits_or_nan(row, oracle.moving_average(ys[s], 3, 5)), (path, s)


@pytest.mark.parametrize("smooth", [None, "small"])
def test_small_spectra_compact_rows_through_the_python_surface(smooth, engine_env):
    """The sim spectra as the Bruker reader keeps them (int32 samples decoded by the
    smoother launch itself from page-locked memory) through Deconvoluter: one at a
    time and the 16 as one set, against the sim_XX_harness goldens -- with the
    default smoother and with k_smooth_small."""
    import metabodecon as md
    if smooth:
        engine_env.setenv("MDG_SMOOTH", smooth)
    sims = md.Spectrum.read_bruker_set(os.path.join(GOLDEN, "bruker", "sim"), 10, 10, (3.34, 3.56))
    dec = md.Deconvoluter()
    res = dec.par_deconvolute_spectra(sims)
    one = [dec.deconvolute_spectrum(sims[k]) for k in (0, 9)]
    for k, d in list(enumerate(res)) + [(0, one[0]), (9, one[1])]:
        g = np.load(os.path.join(GOLDEN, "expected", f"sim_{k + 1:02d}_harness.npz"))
        assert np.array_equal(d.params, g["params"]), k
        assert abs(d.mse - float(g["mse"])) <= MSE_RTOL * abs(float(g["mse"])), k
