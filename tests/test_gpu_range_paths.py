"""GPU: the plain-IEEE-division paths and both range-flag protocols.

Inside the fast ranges the fit and superposition_vec divide with div_rn, the IEEE
division's own sequence minus its no-op wrappers (bit-identical by construction,
DESIGN.md §2); a spectrum whose parameters or axis leave the ranges must take `/`,
decided per iteration from range flags that rotate in two protocols:
- ping-pong slots `it & 1` (k_fit_sup reads, k_fit_update counts), and
- three slots `it % 3` (the term folds read it % 3, count (it + 1) % 3, clear (it + 2) % 3),
with slot 0 seeded by the fit initialisation at the end of k_select.
The cases of tests/golden/range_cases.py scale golden spectra so that the flag flips
in the middle of the fit, both ways, or stays raised throughout, or the axis leaves
the range. Every fit kernel the library ships runs them, alone and in one batch, and
so do the queue, the exact-order MSE and superposition_vec; results must equal the
oracle bit for bit (MSE within 1e-12 relative, exactly for the exact-order MSE), and
the engine's own record of its slow launches (mdg_ctx_last_range_flags) must equal
the oracle's range trace: the slow path ran exactly where the ranges say it must.
Reference: lorentzian.rs:546-548, fitter_analytical.rs:147-172, deconvoluter.rs:828-862.
"""
import numpy as np
import pytest

import oracle
from tests.golden.range_cases import (RANGE_CASES, mask_bits, mixed_superposition_inputs,
                                      range_case)
from tests.test_gpu_parity import FIT_KERNELS, MSE_RTOL, _force_fit, gpu_batch

pytestmark = pytest.mark.gpu

nat = pytest.importorskip("metabodecon._native")

SLOW_MSE, SLOW_MSE_EXACT = 1 << 30, 1 << 31
_REF = {}


@pytest.fixture(scope="module")
def ctx():
    return nat.context(0)


def _case(case):
    if case[0] not in _REF:
        x, y, sb, st, ign = range_case(case)
        _REF[case[0]] = ((x, y, sb, st, ign), oracle.deconvolute(x, y, sb, st, ignore=ign, threads=8))
    return _REF[case[0]]


def expected_mask(o, iters):
    """The launches that must take `/`: fit iteration it when version it has a value
    outside the ranges or the axis does; the MSE when a retained Lorentzian or the axis
    is outside them."""
    fit = (1 << iters) - 1
    m = fit if not o.x_ok else o.range_mask & fit
    if not o.x_ok or o.unsafe_kept > 0:
        m |= SLOW_MSE
    return m


def check(ctx, k, o, status, counts, out, mse, iters, tag, exact_mse=False, small=False):
    assert status[k] == o.status == 0, tag
    assert counts[k] == o.params.shape[0], tag
    assert np.array_equal(out[k, : counts[k]], o.params), tag
    if exact_mse:
        assert mse[k] == o.mse, (tag, mse[k], o.mse)
    else:
        assert abs(mse[k] - o.mse) <= MSE_RTOL * abs(o.mse), (tag, mse[k], o.mse)
    x_ok, slow, unsafe_kept = ctx.last_range_flags(k)
    want = expected_mask(o, iters)
    if exact_mse and want & SLOW_MSE:
        want |= SLOW_MSE_EXACT
    assert x_ok == o.x_ok, tag
    assert unsafe_kept == o.unsafe_kept, tag
    assert slow == want, (tag, format(slow, "032b"), format(want, "032b"))


def test_oracle_cases_flip_mid_fit():
    """The cases do flip: fast then slow, slow then fast, one slow iteration alone."""
    masks = {c[0]: _case(c)[1].range_mask for c in RANGE_CASES}
    assert masks["flip_blood01"] & 0b111 == 0b101
    assert masks["dip_blood05"] & (1 << 5) == 0 and masks["dip_blood05"] & (1 << 6)
    assert masks["low_blood01"] & 1 == 0 and masks["low_blood01"] & (1 << 9)


@pytest.mark.parametrize("path", FIT_KERNELS + ["default"])
def test_range_cases_single_spectrum(ctx, path, monkeypatch, engine_env):
    """Each case alone (B = 1) through every fit kernel, and the engine's own choice."""
    if path != "default":
        _force_fit(engine_env, path)
    for case in RANGE_CASES:
        (x, y, sb, st, ign), o = _case(case)
        res = gpu_batch(ctx, x, y[None, :], [sb], st, ign)
        small = path == "small" or (path == "default" and y.size <= 4096)
        check(ctx, 0, o, *res, st.fit_iterations, (path, case[0]), small=small)


BATCH = [c for c in RANGE_CASES if c[1].startswith("blood")]


@pytest.mark.parametrize("path", FIT_KERNELS + ["default"])
def test_range_cases_batch(ctx, path, monkeypatch, engine_env):
    """The blood cases in one batch beside the unscaled spectrum (fast throughout):
    the flags are per spectrum, so one launch runs both forms side by side."""
    if path != "default":
        _force_fit(engine_env, path)
    from tests.golden.cases import load_case
    x0, y0, sb0, st, _ = load_case("blood_01")
    o0 = oracle.deconvolute(x0, y0, sb0, st)
    rows = [(x0, y0, sb0, o0)] + [(*_case(c)[0][:3], _case(c)[1]) for c in BATCH]
    xs = np.stack([r[0] for r in rows])
    ys = np.stack([r[1] for r in rows])
    res = gpu_batch(ctx, xs, ys, [r[2] for r in rows], st)
    for k, r in enumerate(rows):
        check(ctx, k, r[3], *res, st.fit_iterations, (path, k), small=path == "small")
    assert ctx.last_range_flags(0) == (1, 0, 0)


def test_range_cases_batch_over_24(ctx):
    """Above 24 spectra the engine's own choice is k_fit_sup + k_fit_update (the
    ping-pong protocol) and the 1024-point MSE tiles: 28 spectra, the cases four times."""
    st = oracle.default_settings()
    rows = [(*_case(c)[0][:3], _case(c)[1]) for c in BATCH] * 4
    rows = rows[:28]
    res = gpu_batch(ctx, np.stack([r[0] for r in rows]), np.stack([r[1] for r in rows]),
                    [r[2] for r in rows], st)
    for k, r in enumerate(rows):
        check(ctx, k, r[3], *res, st.fit_iterations, k)


def test_range_cases_exact_mse(ctx):
    """MDG_OPTION_EXACT_MSE: the reference's operation order, so the MSE equals the
    oracle's bit for bit; its residual kernel takes `/` where a retained Lorentzian or
    the axis is out of range (bit 31)."""
    for case in RANGE_CASES:
        (x, y, sb, st, ign), o = _case(case)
        s = nat.Settings()
        for f, _ in nat.Settings._fields_:
            setattr(s, f, getattr(st, f))
        s.options = nat.OPTION_EXACT_MSE
        res = gpu_batch(ctx, x, y[None, :], [sb], s, ign)
        check(ctx, 0, o, *res, st.fit_iterations, case[0], exact_mse=True, small=y.size <= 4096)


def test_range_cases_through_the_queue():
    """The spectrum queue (single-spectrum submissions gathered into batches on two
    lanes) on the blood cases and the unscaled spectrum, against the oracle."""
    torch = pytest.importorskip("torch")
    from tests.golden.cases import load_case
    x0, y0, sb0, st, _ = load_case("blood_01")
    rows = [(x0, y0, sb0, oracle.deconvolute(x0, y0, sb0, st))] + \
        [(*_case(c)[0][:3], _case(c)[1]) for c in BATCH]
    n, k = y0.size, len(rows)
    cap = n // 2 + 2
    X = torch.from_numpy(np.stack([r[0] for r in rows])).cuda()
    Y = torch.from_numpy(np.stack([r[1] for r in rows])).cuda()
    out = torch.zeros((k, cap, 3), dtype=torch.float64, device="cuda")
    cnt = torch.zeros(k, dtype=torch.int32, device="cuda")
    mse = torch.zeros(k, dtype=torch.float64, device="cuda")
    stt = torch.full((k,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    q = nat.SpectrumQueue(0, n, 3, 2, nat.default_settings())
    try:
        for i in range(k):
            q.submit(X[i].data_ptr(), Y[i].data_ptr(), rows[i][2], out[i].data_ptr(), cap,
                     cnt[i:].data_ptr(), mse[i:].data_ptr(), stt[i:].data_ptr())
        q.synchronize()
    finally:
        q.close()
    for i, r in enumerate(rows):
        o = r[3]
        assert int(stt[i]) == 0 and int(cnt[i]) == o.params.shape[0], i
        assert np.array_equal(out[i, : int(cnt[i])].cpu().numpy(), o.params), i
        assert abs(float(mse[i]) - o.mse) <= MSE_RTOL * abs(o.mse), i


def test_superposition_vec_mixed_ranges(ctx):
    """superposition_vec with five parameters outside the ranges among 300 in-range
    ones (every point takes `/`), and in-range parameters on an axis with three points
    beyond 2^100 (those lanes take `/`, the others div_rn): the oracle's in-order
    sums, bit for bit."""
    import metabodecon as md
    x, x_far, params = mixed_superposition_inputs()
    assert np.array_equal(md.superposition_vec(x, params), oracle.superposition_vec(x, params, threads=8))
    ok = np.delete(params, [7, 100, 150, 151, 299], axis=0)
    got = md.superposition_vec(x_far, ok)
    assert np.array_equal(got, oracle.superposition_vec(x_far, ok, threads=8))
    assert np.array_equal(md.superposition_vec(x_far, params),
                          oracle.superposition_vec(x_far, params, threads=8))
