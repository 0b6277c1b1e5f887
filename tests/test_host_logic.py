"""Host-side logic of the product (no GPU): settings, ignore regions, Spectrum
validation, Bruker reader, serialisation, synthetic generator determinism."""
import math
import os

import numpy as np
import pytest

import oracle
from tests.conftest import GOLDEN
from metabodecon import Deconvoluter, Deconvolution, Lorentzian, Spectrum, exceptions
from metabodecon import _native as nat


def test_default_settings_match_reference():
    s = nat.default_settings()
    o = oracle.default_settings()
    for f, _ in nat.Settings._fields_:
        assert getattr(s, f) == getattr(o, f)


@pytest.mark.parametrize("kw", [
    dict(smooth_iterations=0), dict(smooth_window=1), dict(smooth_window=0),
    dict(threshold=0.0), dict(threshold=-1.0), dict(threshold=float("nan")),
    dict(threshold=float("inf")), dict(fit_iterations=0), dict(),
    dict(smoother="identity", smooth_iterations=0), dict(selector="detector_only", threshold=0.0),
])
def test_validate_matches_oracle(kw):
    o = oracle.make_settings(**kw)
    s = nat.Settings()
    for f, _ in nat.Settings._fields_:
        setattr(s, f, getattr(o, f))
    assert nat.validate(s) == oracle.lib().mdo_validate_settings(o)


def test_engine_options_validation():
    """mdg_settings.options: MDG_OPTION_EXACT_MSE is the one defined bit (0 and 1 are
    valid), every other bit is MDG_INVALID_ARGUMENT; Deconvoluter.exact_mse sets and
    clears it without touching the reference settings."""
    s = nat.default_settings()
    assert s.options == 0 and nat.validate(s) == 0
    s.options = nat.OPTION_EXACT_MSE
    assert nat.validate(s) == 0
    for bad in (2, 3, 1 << 30, -1):
        s.options = bad
        assert nat.validate(s) == nat.INVALID_ARGUMENT, bad
    d = Deconvoluter()
    before = d.settings
    d.exact_mse = True
    assert d.exact_mse and d.settings.options == nat.OPTION_EXACT_MSE
    d.set_noise_score_selector(6.0)
    assert d.exact_mse  # other setters keep the option
    d.exact_mse = False
    after = d.settings
    assert after.options == 0 and after.threshold == 6.0
    for f, _ in nat.Settings._fields_:
        if f != "threshold":
            assert getattr(after, f) == getattr(before, f), f


def test_deconvoluter_setters_raise_reference_exceptions():
    d = Deconvoluter()
    with pytest.raises(exceptions.InvalidSmoothingSettings):
        d.set_moving_average_smoother(0, 3)
    with pytest.raises(exceptions.InvalidSmoothingSettings):
        d.set_moving_average_smoother(2, 1)
    with pytest.raises(exceptions.InvalidSelectionSettings):
        d.set_noise_score_selector(0.0)
    with pytest.raises(exceptions.InvalidSelectionSettings):
        d.set_noise_score_selector(float("nan"))
    with pytest.raises(exceptions.InvalidFittingSettings):
        d.set_analytical_fitter(0)
    with pytest.raises(ValueError):
        d.set_threads(1)
    d.set_identity_smoother()
    d.set_detector_only()
    d.set_analytical_fitter(20)
    assert d.settings.fit_iterations == 20 and d.settings.smoother == 0


def test_ignore_regions_match_oracle():
    rng = np.random.default_rng(7)
    for _ in range(50):
        d = Deconvoluter()
        ref = []
        for _ in range(rng.integers(1, 6)):
            a, b = rng.uniform(-2, 12, 2)
            d.add_ignore_region((a, b))
            ref = oracle.add_ignore_region(ref, (a, b))
        assert d.ignore_regions == ref
    d = Deconvoluter()
    for bad in [(float("nan"), 1.0), (1.0, float("inf")), (1.0, 1.0)]:
        with pytest.raises(exceptions.InvalidIgnoreRegion):
            d.add_ignore_region(bad)
    d.add_ignore_region((1.0, 2.0))
    d.clear_ignore_regions()
    assert d.ignore_regions is None


def test_spectrum_validation():
    x = np.linspace(10, 0, 11)
    y = np.ones(11)
    s = Spectrum(x, y, (2, 8))
    assert s.signal_boundaries == (8.0, 2.0)  # decreasing axis: (max, min)
    s = Spectrum(x[::-1], y, (8, 2))
    assert s.signal_boundaries == (2.0, 8.0)
    with pytest.raises(exceptions.EmptyData):
        Spectrum([], [], (0, 1))
    with pytest.raises(exceptions.DataLengthMismatch):
        Spectrum(x, y[:-1], (2, 8))
    with pytest.raises(exceptions.NonUniformSpacing):
        Spectrum(np.r_[x[:-1], -3.0], y, (2, 8))
    with pytest.raises(exceptions.InvalidIntensities):
        Spectrum(x, np.r_[y[:-1], np.nan], (2, 8))
    with pytest.raises(exceptions.InvalidSignalBoundaries):
        Spectrum(x, y, (2, 2))
    with pytest.raises(exceptions.InvalidSignalBoundaries):
        Spectrum(x, y, (2, 11))
    # spectrum.rs:731-738 doc test
    s = Spectrum([1.0, 2.0, 3.0, 4.0, 5.0], [1.0, 2.0, 3.0, 4.0, 5.0], (2.25, 3.75))
    assert s.signal_boundaries_indices() == (1, 3)


def test_bruker_reader_matches_reference_tests():
    # bruker.rs:517-548 (read_acquisition/processing_parameters) and check macros
    s = Spectrum.read_bruker(os.path.join(GOLDEN, "bruker", "blood", "blood_01"), 10, 10,
                             (-2.2, 11.8))
    assert len(s) == 131072
    assert s.nucleus == "1H"
    assert math.isclose(s.frequency, 600.252821089118, rel_tol=0, abs_tol=1e-12)
    assert s.chemical_shifts[0] == 14.81146
    assert s.chemical_shifts[1] == 14.81146 - (1.0 * 20.0236139622347) / 131071.0
    sims = Spectrum.read_bruker_set(os.path.join(GOLDEN, "bruker", "sim"), 10, 10, (3.34, 3.56))
    assert len(sims) == 16 and all(len(t) == 2048 for t in sims)
    assert math.isclose(sims[0].frequency, 600.2528069499997, rel_tol=0, abs_tol=1e-9)
    with pytest.raises(OSError):  # Error::IoError -> PyIOError (src/error.rs:93)
        Spectrum.read_bruker(os.path.join(GOLDEN, "bruker", "sim"), 10, 10, (3.34, 3.56))


def test_lorentzian_host_api():
    # lorentzian.rs:678-706 accessors / mutators
    lz = Lorentzian.from_transformed(1.0, 0.25, 0.0)
    assert (lz.sfhw, lz.hw2, lz.maxp, lz.sf, lz.hw) == (1.0, 0.25, 0.0, 2.0, 0.5)
    lz = Lorentzian.from_transformed(1.5, 2.25, 1.0)
    assert lz.sf == 1.0 and lz.hw == 1.5
    lz = Lorentzian(0.3, 0.15, 5.0)  # bindings/lorentzian.rs:26-31
    assert lz.sfhw == 0.3 * 0.15 and lz.hw2 == 0.15 * 0.15
    assert abs(lz.evaluate(5.0) - 2.0) < 1e-12
    assert math.isclose(lz.integral(), math.pi * lz.sf)
    trip = [Lorentzian.from_transformed(0.03, 0.0009, 4.8),
            Lorentzian.from_transformed(0.02, 0.0004, 5.0),
            Lorentzian.from_transformed(0.03, 0.0009, 5.2)]
    assert abs(Lorentzian.superposition(5.0, trip) - 51.466992) <= 1e-6
    assert np.array_equal(trip[0].evaluate_vec(np.array([4.8, 5.0])),
                          oracle.superposition_vec([4.8, 5.0], [[0.03, 0.0009, 4.8]]))


def test_deconvolution_json_round_trip(tmp_path):
    # deconvolution.rs:133-183 serialization_round_trip
    p = np.array([[5.5, 0.25, 3.0], [7.0, 0.16, 5.0], [5.5, 0.25, 7.0]])
    d = Deconvolution(p, 0.5, nat.default_settings())
    f = str(tmp_path / "d.json")
    d.write_json(f)
    e = Deconvolution.read_json(f)
    assert e.mse == 0.5
    assert np.allclose(e.params, p, rtol=4 * 2.2e-16, atol=2.2e-16)
    js = d.to_json_dict()
    assert js["smoothingSettings"] == {"method": "MovingAverage", "iterations": 3, "windowSize": 3}
    assert js["selectionSettings"]["method"] == "NoiseScoreFilter"
    assert js["fittingSettings"] == {"method": "Analytical", "iterations": 10}
    with pytest.raises(exceptions.SerializationError):
        bad = tmp_path / "bad.json"
        bad.write_text("{}")
        Deconvolution.read_json(str(bad))


def test_synth_generator_is_deterministic_and_exact():
    a = np.empty((64, 3))
    b = np.empty((64, 3))
    nat.lib().mdg_synth_lorentzians(3, 64, -1.8, 11.4, nat.ptr(a))
    nat.lib().mdg_synth_lorentzians(3, 64, -1.8, 11.4, nat.ptr(b))
    assert np.array_equal(a, b)
    assert np.all(np.diff(a[:, 2]) > 0)  # jitter < half a grid cell keeps order
    hw = np.sqrt(a[:, 1])
    assert hw.min() >= 3e-4 - 1e-12 and hw.max() <= 8e-4 + 1e-12
    n = np.empty(100000)
    nat.lib().mdg_synth_noise(5, n.size, 1.0e3, nat.ptr(n))
    assert abs(n.mean()) < 20 and 950 < n.std() < 1050
    assert np.all(np.abs(n) <= 6e3)


def test_no_cpu_fallback_without_device():
    """With no GPU the product must fail loudly, not compute on the CPU."""
    cnt = __import__("ctypes").c_int(-1)
    nat.lib().mdg_device_count(__import__("ctypes").byref(cnt))
    if cnt.value > 0:
        pytest.skip("GPU present")
    x = np.linspace(14, -5, 4096)
    s = Spectrum(x, np.ones(4096), (-2.2, 11.8))
    with pytest.raises(nat.DeviceUnavailableError):
        Deconvoluter().deconvolute_spectrum(s)


def test_division_hard_cases_lie_next_to_rounding_midpoints():
    """mdg_division_hard_case (the generator mdg_check_division runs on the
    device) yields operand pairs whose exact quotient is within 2^-53 ulp of a
    rounding midpoint (checked in exact rational arithmetic), inside the
    fast-division range [2^-200, 2^200]."""
    import ctypes
    from fractions import Fraction
    n, d = ctypes.c_double(), ctypes.c_double()
    valid = 0
    for i in range(3000):
        if nat.lib().mdg_division_hard_case(11, i, ctypes.byref(n), ctypes.byref(d)):
            continue
        valid += 1
        for v in (n.value, d.value):
            assert 2.0 ** -200 <= abs(v) <= 2.0 ** 200
        q = Fraction(n.value) / Fraction(d.value)
        ulp = Fraction(2) ** (math.frexp(float(q))[1] - 53)
        t = q / ulp  # significand scaled to [2^52, 2^53)
        dist = abs(t - math.floor(t) - Fraction(1, 2))
        assert 0 < dist <= Fraction(1, 2 ** 53), (i, float(dist))
    assert valid > 1000


def test_ignore_regions_have_no_engine_limit():
    """The reference's add_ignore_region accepts any number of disjoint regions
    (deconvoluter.rs:438-472); so does this one (the engine sizes its per-spectrum
    region rows per call), merging exactly like the oracle."""
    d = Deconvoluter()
    for k in range(300):
        d.add_ignore_region((0.01 * k, 0.01 * k + 0.005))
    assert len(d.ignore_regions) == 300
    d.add_ignore_region((0.0, 0.012))  # merges the first two
    assert len(d.ignore_regions) == 299
    assert d.ignore_regions[0] == (0.0, 0.015)


@pytest.mark.parametrize("visible,local_rank,want", [(1, "1", 0), (1, "3", 0), (8, "3", 3),
                                                      (2, "5", 1), (0, "2", 0)])
def test_default_device_wraps_local_rank_to_visible_devices(monkeypatch, visible, local_rank,
                                                            want):
    """A launcher that exposes one GPU per rank (HIP_VISIBLE_DEVICES) with LOCAL_RANK>0
    must still land on a device that exists (LOCAL_RANK used unchecked)."""
    monkeypatch.delenv("MDGPU_DEVICE", raising=False)
    monkeypatch.setenv("LOCAL_RANK", local_rank)
    monkeypatch.setattr(nat, "device_count", lambda: visible)
    assert nat.default_device() == want
    monkeypatch.setenv("MDGPU_DEVICE", "1")
    assert nat.default_device() == 1
    monkeypatch.delenv("MDGPU_DEVICE")
    monkeypatch.delenv("LOCAL_RANK")
    assert nat.default_device() == 0
