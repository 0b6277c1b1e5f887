"""Full-size GPU parity for the batch configurations of BASELINE.json.

configs[2]: 256 synthetic 131072-point spectra (seeds 0..255, 2048 injected
Lorentzians, SURVEY 8d recipe) in ONE batched device call
(mdg_deconvolute_batch_device: the B > 8 grid layouts -- spectrum-interleaved
fit grid, CU-interleaved MSE grid, k_smooth_chain at B*passes = 768 -- that no
smaller test reaches). configs[3]: 4096 synthetic 65536-point spectra (1024
Lorentzians, half widths x2) in one call on one GPU: the lane-pipelined
k_smooth_pipe path (B*passes > 2048, beyond the chain) at its largest size.

Every spectrum is compared with the oracle (the C restatement, run on the box's
cores as the checker; the spectra come from the device generator, which is
bit-identical to the host one -- test_synth_device_matches_host): status and
kept count equal, Lorentzian parameters bit-identical, MSE within MSE_RTOL.
This mirrors par_deconvolute_spectra (deconvoluter.rs:700-710): a map over
independent spectra.
"""
import ctypes

import numpy as np
import pytest

import oracle
from tests.golden.cases import host_threads, synth_spectrum

pytestmark = pytest.mark.gpu

MSE_RTOL = 1e-12
nat = pytest.importorskip("metabodecon._native")
torch = pytest.importorskip("torch")
SB = (11.8, -2.2)


def _device_batch(B, n, peaks, hw_scale, cap, seed0=0, sigma=1.0e3):
    ctx = nat.Context(0)
    dev = torch.device("cuda", 0)
    x = torch.empty(n, dtype=torch.float64, device=dev)
    y = torch.empty((B, n), dtype=torch.float64, device=dev)
    rc = nat.lib().mdg_synth_batch_device_hw(ctx.handle, B, n, 14.8, 20.0, seed0, peaks, -1.8,
                                             11.4, hw_scale, sigma, x.data_ptr(), y.data_ptr())
    assert rc == 0, nat.strerror(rc)
    sb = torch.tensor([SB] * B, dtype=torch.float64, device=dev)
    out = torch.zeros((B, cap, 3), dtype=torch.float64, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    mse = torch.zeros(B, dtype=torch.float64, device=dev)
    status = torch.full((B,), -1, dtype=torch.int32, device=dev)
    settings = nat.default_settings()
    ctx.synchronize()
    rc = nat.lib().mdg_deconvolute_batch_device(
        ctx.handle, B, n, x.data_ptr(), 0, y.data_ptr(), n, sb.data_ptr(), ctypes.byref(settings),
        None, 0, out.data_ptr(), cap, cnt.data_ptr(), mse.data_ptr(), status.data_ptr())
    assert rc == 0, nat.strerror(rc)
    ctx.synchronize()
    res = dict(x=x.cpu().numpy(), y=y.cpu().numpy(), out=out.cpu().numpy(),
               cnt=cnt.cpu().numpy(), mse=mse.cpu().numpy(), status=status.cpu().numpy(),
               kernels=ctx.stage_kernels(), ctx=ctx)
    return res


def _compare(res, cap, inner_threads=1):
    B, n = res["y"].shape
    st, counts, params, mse = oracle.deconvolute_batch(res["x"], res["y"], np.array([SB] * B),
                                                       threads=host_threads(), cap=cap,
                                                       inner_threads=inner_threads)
    assert np.array_equal(res["status"], st), np.nonzero(res["status"] != st)
    assert np.array_equal(res["cnt"].astype(np.int64), counts)
    bad = [s for s in range(B)
           if not np.array_equal(res["out"][s, : counts[s]], params[s, : counts[s]])]
    assert not bad, f"{len(bad)} spectra differ, first {bad[:8]}"
    rel = np.abs(res["mse"] - mse) / np.abs(mse)
    assert rel.max() <= MSE_RTOL, (rel.max(), int(rel.argmax()))
    return counts


def test_synth_device_matches_host():
    """mdg_synth_batch_device_hw == the host generator (synth_spectrum), bit for bit."""
    for hw_scale, n, peaks in ((1.0, 131072, 2048), (2.0, 65536, 1024)):
        res = _device_batch(2, n, peaks, hw_scale, 8, seed0=7)
        for s in range(2):
            x, y, _ = synth_spectrum(7 + s, n=n, n_peaks=peaks, hw_scale=hw_scale)
            assert np.array_equal(res["x"], x)
            assert np.array_equal(res["y"][s], y)
        res["ctx"].close()


def test_configs2_256x131072_bit_exact():
    cap = 4096
    res = _device_batch(256, 131072, 2048, 1.0, cap)
    k = res["kernels"]
    assert k["smooth"].startswith("k_smooth_chain<3, false>") and k["fit_superposition"].startswith("k_fit_sup")
    counts = _compare(res, cap)
    assert counts.min() > 1900  # ~2k injected peaks survive selection and the fit
    res["ctx"].close()


def test_long_spectra_bit_exact():
    """Two 4 000 037-point spectra (odd length, 30x configs[1]; 2048 injected
    Lorentzians): row lengths far past every other test -- 62 501 mask words, 245
    peak chunks, ~760k detected peaks, ~19k selected and fitted (P^2 = 3.6e8 terms
    per fit point set), a 2 000 020-peak capacity -- against the oracle, bit for bit."""
    n = 4000037
    cap = n // 2 + 2
    res = _device_batch(2, n, 2048, 1.0, cap, seed0=11)
    counts = _compare(res, cap, inner_threads=max(1, host_threads() // 2))
    assert counts.min() > 10000  # the noise peaks of 4M points pass the noise-score filter
    res["ctx"].close()


def test_configs3_4096x65536_bit_exact():
    cap = 2048
    res = _device_batch(4096, 65536, 1024, 2.0, cap)
    assert res["kernels"]["smooth"].startswith("k_smooth_pipe<3>")
    counts = _compare(res, cap)
    assert counts.min() > 900
    res["ctx"].close()


def test_optimize_settings_blood_01_full_size():
    """Deconvoluter.optimize_settings on a real 131072-point
    spectrum (blood_01, Bruker 10/10, sb (-2.2, 11.8)) against the exhaustive
    810-setting oracle sweep (deconvoluter.rs:762-825; first minimum in the grid's
    order) on the box's cores: the argmin and its MSE bit for bit."""
    import os
    import metabodecon as md
    from tests.conftest import GOLDEN
    sp = md.Spectrum.read_bruker(os.path.join(GOLDEN, "bruker", "blood", "blood_01"), 10, 10,
                                 (-2.2, 11.8))
    dec = md.Deconvoluter()
    got = dec.optimize_settings(sp)
    st, best, mse = oracle.optimize_settings(sp.chemical_shifts, sp.intensities,
                                             sp.signal_boundaries, threads=host_threads())
    assert st == 0
    s = dec.settings
    assert (s.smooth_iterations, s.smooth_window, s.threshold, s.fit_iterations) == best
    assert got == mse


@pytest.mark.parametrize("hw_scale,sigma", [(0.5, 1.0), (0.3, 1.0e-3), (0.5, 0.0)])
def test_mse_narrow_peaks_close_fit(hw_scale, sigma):
    """k_mse_local sums the far Lorentzians of a tile as a 20-term series of
    Im[a/(x - z)], whose terms exceed the Lorentzian by ~distance/half-width, so its
    roundoff is amplified most by narrow peaks; and a close fit (near-zero noise)
    makes the residual, hence the MSE, small against the superposition. Narrow
    half-widths (x0.3, x0.5) with sigma 1, 1e-3 and 0: every MSE within MSE_RTOL of
    the oracle's left fold (and the parameters bit-identical, as everywhere)."""
    cap = 4096
    res = _device_batch(4, 131072, 2048, hw_scale, cap, seed0=40, sigma=sigma)
    assert res["kernels"].get("mse_superposition", "").startswith("k_mse_local")
    counts = _compare(res, cap)
    assert counts.min() > 100
    res["ctx"].close()
