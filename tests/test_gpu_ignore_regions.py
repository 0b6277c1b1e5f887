"""GPU parity of ignore regions (deconvoluter.rs:438-472, 865-904) beyond the
round-2 engine's 64-region limit, and across calls that change the regions on
the same device buffers (cached graphs and direct launches).

Bars as in test_gpu_parity.py: Lorentzian parameters bit-identical to the oracle,
MSE within 1e-12 relative (its residual sum is a fixed-order tree on the GPU).
"""
import ctypes

import numpy as np
import pytest

import oracle
from tests.golden.cases import load_case

pytestmark = pytest.mark.gpu

MSE_RTOL = 1e-12

nat = pytest.importorskip("metabodecon._native")


def many_regions(count, lo=0.6, hi=8.9, width=0.004):
    """`count` disjoint regions of `width` ppm spread over [lo, hi] (merged form)."""
    regs = []
    for k in range(count):
        a = lo + (hi - lo) * k / count
        regs = oracle.add_ignore_region(regs, (a + width, a))  # reversed ends on purpose
    assert len(regs) == count
    return regs


def engine_settings(st):
    """The oracle's settings as the engine's ctypes struct (same fields)."""
    s = nat.Settings()
    for f, _ in nat.Settings._fields_:
        setattr(s, f, getattr(st, f))
    return s


def host_run(ctx, x, y, sb, st, regs):
    st = engine_settings(st)
    ign = np.asarray(regs, dtype=np.float64).reshape(-1)
    n = y.size
    cap = n // 2 + 2
    out = np.zeros((1, cap, 3))
    counts = np.zeros(1, dtype=np.uintp)
    mse = np.zeros(1)
    status = np.zeros(1, dtype=np.intc)
    rc = nat.lib().mdg_deconvolute_batch(
        ctx.handle, 1, n, nat.ptr(np.ascontiguousarray(x)), 0, nat.ptr(np.ascontiguousarray(y)),
        n, nat.ptr(np.asarray(sb, dtype=np.float64)), ctypes.byref(st),
        nat.ptr(ign) if ign.size else None, ign.size // 2, nat.ptr(out), cap,
        nat.ptr(counts, nat._szp), nat.ptr(mse),
        status.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    assert rc < 100, nat.strerror(rc)
    return int(status[0]), out[0, : int(counts[0])].copy(), float(mse[0])


def check(o, got):
    status, params, mse = got
    assert status == o.status
    if o.status:
        return
    assert np.array_equal(params, o.params), \
        np.max(np.abs(params - o.params) / np.abs(o.params))
    assert abs(mse - o.mse) <= MSE_RTOL * abs(o.mse)


def increasing(case):
    """The case on an increasing axis (arrays and boundaries reversed): with two or
    more ignore regions on a decreasing axis the reference's MSE regions run
    backwards and it panics (Rust slice start > end, deconvoluter.rs:846-853)."""
    x, y, sb, st, ign = load_case(case)
    return x[::-1].copy(), y[::-1].copy(), (sb[1], sb[0]), st


def filtered_detection(x, y, sb, regs):
    """The oracle's detected peaks after the ignore filter (noise_score_filter.rs:41-48)."""
    l, c, r = oracle.detect_peaks(oracle.second_derivative(oracle.moving_average(y, 3, 3)))
    pairs = oracle.ignore_region_indices(x, sb, regs)
    inside = lambda v: any(a <= v < b for a, b in pairs)  # noqa: E731
    keep = [k for k in range(len(c)) if not (inside(l[k]) or inside(r[k]))]
    return np.stack([np.asarray(l)[keep], np.asarray(c)[keep], np.asarray(r)[keep]], axis=1)


@pytest.mark.parametrize("count", [9, 65, 300])
def test_many_ignore_regions_match_oracle(count):
    """More than 64 disjoint regions (the reference has no limit): the detector's
    ignore filter and the MSE regions switch to binary searches over the sorted
    index pairs above 8 regions. Full parity on an increasing axis."""
    ctx = nat.context(0)
    x, y, sb, st = increasing("blood_01")
    regs = many_regions(count)
    assert len(oracle.ignore_region_indices(x, sb, regs)) > 8
    o = oracle.deconvolute(x, y, sb, st, ignore=regs)
    assert o.status == 0
    check(o, host_run(ctx, x, y, sb, st, regs))
    assert np.array_equal(ctx.last_peaks(0, "detected").astype(np.int64),
                          filtered_detection(x, y, sb, regs))


@pytest.mark.parametrize("count", [9, 300])
def test_many_ignore_regions_decreasing_axis(count):
    """On the decreasing (Bruker) axis the index pairs descend: the reference panics
    in compute_mse (status 30 here, like the oracle), and the detector's ignore
    filter -- the descending branch of the binary search -- keeps exactly the
    oracle's peaks."""
    ctx = nat.context(0)
    x, y, sb, st, _ = load_case("blood_01")
    regs = many_regions(count)
    o = oracle.deconvolute(x, y, sb, st, ignore=regs)
    assert o.status == 30
    got = host_run(ctx, x, y, sb, st, regs)
    assert got[0] == 30
    assert np.array_equal(ctx.last_peaks(0, "detected").astype(np.int64),
                          filtered_detection(x, y, sb, regs))


def test_python_surface_accepts_many_regions():
    import metabodecon as md
    x, y, sb, st = increasing("blood_02")
    sp = md.Spectrum(x, y, sb)
    dec = md.Deconvoluter()
    regs = many_regions(120)
    for r in regs:
        dec.add_ignore_region(r)
    assert len(dec.ignore_regions) == 120
    d = dec.deconvolute_spectrum(sp)
    o = oracle.deconvolute(x, y, sb, st, ignore=regs)
    assert np.array_equal(d.params, o.params)
    assert abs(d.mse - o.mse) <= MSE_RTOL * abs(o.mse)


@pytest.mark.parametrize("graphs", ["0", "1"])
def test_device_path_alternating_ignore_sets(graphs, monkeypatch, engine_env):
    """the same device buffers, calls alternating between ignore-region
    sets (none, two, 70, two again, a different two), direct launches and cached
    graph replays: every call equals the oracle with that call's regions."""
    torch = pytest.importorskip("torch")
    engine_env.setenv("MDG_GRAPHS", graphs)
    ctx = nat.Context(0)
    try:
        cx, cy, csb, cst = increasing("blood_05")
        n = cy.size
        dev = "cuda"
        x = torch.from_numpy(cx).to(dev)
        y = torch.from_numpy(cy).to(dev)[None, :].contiguous()
        sb = torch.tensor([csb], dtype=torch.float64, device=dev)
        cap = n // 2 + 2
        out = torch.zeros((1, cap, 3), dtype=torch.float64, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        mse = torch.zeros(1, dtype=torch.float64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        s = nat.default_settings()
        sets = [[], [(1.2, 1.3), (4.7, 4.9)], many_regions(70), [(1.2, 1.3), (4.7, 4.9)],
                [(3.0, 3.1), (6.0, 6.2)], []]
        for rnd, regs in enumerate(sets + sets):
            ign = np.asarray(regs, dtype=np.float64).reshape(-1)
            rc = nat.lib().mdg_deconvolute_batch_device(
                ctx.handle, 1, n, x.data_ptr(), 0, y.data_ptr(), n, sb.data_ptr(),
                ctypes.byref(s), nat.ptr(ign) if ign.size else None, ign.size // 2,
                out.data_ptr(), cap, cnt.data_ptr(), mse.data_ptr(), status.data_ptr())
            assert rc == 0, nat.strerror(rc)
            ign[:] = -1.0  # the engine must have taken its own copy at call time
            ctx.synchronize()
            o = oracle.deconvolute(cx, cy, csb, cst, ignore=regs)
            assert o.status == 0
            got = (int(status[0]), out[0, : int(cnt[0])].cpu().numpy(), float(mse[0]))
            check(o, got)
    finally:
        ctx.close()


def exhaustive_optimize(x, y, sb, ign):
    """The reference's 810-setting grid through the oracle, first minimum
    (deconvoluter.rs:762-825); returns (mse, iterations, window, threshold, fit)."""
    best = None
    for it in range(2, 11):
        for ws in (3, 5, 7):
            for c in range(10):
                thr = 5.0 + (c * (8.0 - 5.0)) / 9.0
                for fit in (5, 10, 15):
                    st = oracle.make_settings(smooth_iterations=it, smooth_window=ws,
                                              threshold=thr, fit_iterations=fit)
                    r = oracle.deconvolute(x, y, sb, st, ignore=ign)
                    assert r.status == 0
                    if best is None or r.mse < best[0]:
                        best = (r.mse, it, ws, thr, fit)
    return best


def test_optimize_settings_exact_mse_with_many_regions():
    """optimize_settings reads the exact-order MSE regions from the workspace rows on
    the device (no fixed-size host copy): on sim_07 (increasing axis) with 12 ignore regions (binary
    searches above 8) its argmin and MSE equal an exhaustive oracle sweep."""
    import metabodecon as md
    x, y, sb, _ = increasing("sim_07")
    merged = []
    for k in range(12):
        a = 3.36 + 0.015 * k
        merged = oracle.add_ignore_region(merged, (a, a + 0.002))
    dec = md.Deconvoluter()
    for r in merged:
        dec.add_ignore_region(r)
    got = dec.optimize_settings(md.Spectrum(x, y, sb))
    best = exhaustive_optimize(x, y, sb, merged)
    assert got == best[0]
    s = dec.settings
    assert (s.smooth_iterations, s.smooth_window, s.threshold, s.fit_iterations) == best[1:]
