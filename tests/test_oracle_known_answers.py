"""Pin the C oracle to every known answer the reference's own tests hold for the hot path.

Each test restates one ``#[test]`` / doc test of SombkeMaximilian/metabodecon-rust
(file:line cited, relative to metabodecon/src/). ``approx_eq`` reproduces
float_cmp's ``assert_approx_eq!(f64, a, b)`` default margin (epsilon = f64::EPSILON,
ulps = 4).
"""
import math
import struct

import numpy as np
import pytest

import oracle


def _ulps(a: float, b: float) -> int:
    ia = struct.unpack("<q", struct.pack("<d", a))[0]
    ib = struct.unpack("<q", struct.pack("<d", b))[0]
    return abs(ia - ib)


def approx_eq(a, b, epsilon=2.220446049250313e-16, ulps=4):
    a, b = float(a), float(b)
    return abs(a - b) <= epsilon or _ulps(a, b) <= ulps


# ---------------------------------------------------------------- peak_selection/common.rs
def test_second_derivative():  # common.rs:49-58
    sd = oracle.second_derivative([1.0, 2.0, 3.0, 2.0, 1.0])
    assert all(approx_eq(a, b) for a, b in zip(sd, [0.0, -2.0, 0.0]))
    assert len(sd) == 3


def test_peak_region_boundaries():  # common.rs:60-68
    assert oracle.peak_region_boundaries([2, 4, 5, 8], (3, 7)) == (1, 3)


# ---------------------------------------------------------------- peak_selection/detector.rs
def test_find_peak_centers():  # detector.rs:240-246
    assert oracle.find_peak_centers([0.0, -2.0, 0.0]) == [2]


def _borders(sd, center):
    """Detector::find_peak_borders for one center (detector.rs:202-212)."""
    sd = np.asarray(sd, dtype=np.float64)
    left = center - oracle.find_left_border(sd[:center])
    right = center + oracle.find_right_border(sd[center - 1:])
    return left, right


@pytest.mark.parametrize(
    "sd,center,expected",
    [  # detector.rs:248-277
        ([0.5, -0.5, -1.0, 0.0, 0.5, 0.0], 3, (2, 5)),
        ([0.0, 0.5, 0.0, -1.0, -0.5, 0.5], 4, (2, 5)),
        ([1.0, 1.0, 1.0, 1.5, 1.0], 3, (0, 4)),
        ([1.0, 1.5, 1.0, 1.0, 1.0], 3, (2, 6)),
        ([1.0, 1.0, 1.0, 1.0, 1.0], 3, (0, 6)),
    ],
)
def test_find_peak_borders(sd, center, expected):
    assert _borders(sd, center) == expected


@pytest.mark.parametrize(
    "sd,sl,expected",
    [  # detector.rs:279-287
        ([0.0, -2.0, -1.0, -0.5, 0.5], slice(2, None), 1),
        ([0.0, -2.0, -1.0, 0.0, 0.5, 0.0], slice(2, None), 2),
        ([1.0, 1.0, 1.0, 1.0, 1.0], slice(2, None), 3),
    ],
)
def test_find_right_border(sd, sl, expected):
    assert oracle.find_right_border(np.asarray(sd)[sl]) == expected


@pytest.mark.parametrize(
    "sd,sl,expected",
    [  # detector.rs:289-297
        ([0.5, -0.5, -1.0, -2.0, 0.0], slice(0, 3), 1),
        ([0.0, 0.5, 0.0, -1.0, -2.0, 0.0], slice(0, 4), 2),
        ([1.0, 1.0, 1.0, 1.0, 1.0], slice(0, 3), 3),
    ],
)
def test_find_left_border(sd, sl, expected):
    assert oracle.find_left_border(np.asarray(sd)[sl]) == expected


# ---------------------------------------------------------------- scorer / noise filter
def test_minimum_sum_scores():  # scorer.rs:264-278
    abs_sd = [1.0, 2.0, 4.0, 2.0, 2.0, 5.0, 4.0, 3.0, 2.0]
    scores = [oracle.score_minimum_sum(abs_sd, *p) for p in [(1, 3, 4), (5, 6, 9)]]
    assert approx_eq(scores[0], 6.0) and approx_eq(scores[1], 7.0)


def test_mean_sd_scores():  # noise_score_filter.rs:153-170
    peaks = [(i - 1, i, i + 1) for i in [2, 4, 5, 8]]
    abs_sd = [1.0, 2.0, 4.0, 2.0, 2.0, 5.0, 4.0, 3.0, 2.0]
    b = (1, 3)
    sfr = peaks[: b[0]] + peaks[b[1]:]
    mean, sd = oracle.mean_sd([oracle.score_minimum_sum(abs_sd, *p) for p in sfr])
    assert approx_eq(mean, 4.0) and approx_eq(sd, 1.0)


# ---------------------------------------------------------------- fitting
def test_mirror_shoulder():  # peak_stencil.rs:372-405
    st = oracle.mirror_shoulder([1.0, 2.0, 3.0, 1.0, 2.0, 3.0])
    assert all(approx_eq(a, b) for a, b in zip(st, [1.0, 2.0, 3.0, 1.0, 2.0, 1.0]))
    st = oracle.mirror_shoulder([1.0, 2.0, 4.0, 3.0, 2.0, 1.0])
    assert all(approx_eq(a, b) for a, b in zip(st, [0.0, 2.0, 4.0, 1.0, 2.0, 1.0]))


def test_fitter_approximations():  # fitter_analytical.rs:187-196
    sfhw, hw2, maxp = oracle.solve_stencil([4.0, 8.0, 12.0, 5.0, 10.0, 5.0])
    assert approx_eq(maxp, 8.0)
    assert approx_eq(math.sqrt(hw2), 4.0)
    assert approx_eq(sfhw / math.sqrt(hw2), 40.0)


# ---------------------------------------------------------------- lorentzian.rs
def test_lorentzian_evaluate():  # lorentzian.rs:708-739
    x = np.array([-5.0 + i for i in range(11)])
    exp = [1 / 26, 1 / 17, 1 / 10, 1 / 5, 1 / 2, 1.0, 1 / 2, 1 / 5, 1 / 10, 1 / 17, 1 / 26]
    y = oracle.superposition_vec(x, [[1.0, 1.0, 0.0]])
    assert all(approx_eq(a, b) for a, b in zip(y, exp))


def test_lorentzian_superposition():  # lorentzian.rs:741-788
    L = [[1.0, 0.5, -2.0], [2.0, 0.75, 0.0], [1.0, 0.5, 2.0]]
    x = np.array([-5.0 + i for i in range(11)])
    exp = [
        1.0 / 9.5 + 2.0 / 25.75 + 1.0 / 49.5,
        1.0 / 4.5 + 2.0 / 16.75 + 1.0 / 36.5,
        1.0 / 1.5 + 2.0 / 9.75 + 1.0 / 25.5,
        1.0 / 0.5 + 2.0 / 4.75 + 1.0 / 16.5,
        1.0 / 1.5 + 2.0 / 1.75 + 1.0 / 9.5,
        1.0 / 4.5 + 2.0 / 0.75 + 1.0 / 4.5,
        1.0 / 9.5 + 2.0 / 1.75 + 1.0 / 1.5,
        1.0 / 16.5 + 2.0 / 4.75 + 1.0 / 0.5,
        1.0 / 25.5 + 2.0 / 9.75 + 1.0 / 1.5,
        1.0 / 36.5 + 2.0 / 16.75 + 1.0 / 4.5,
        1.0 / 49.5 + 2.0 / 25.75 + 1.0 / 9.5,
    ]
    for threads in (1, 4):
        y = oracle.superposition_vec(x, L, threads=threads)
        assert all(approx_eq(a, b) for a, b in zip(y, exp))


def test_lorentzian_doc_examples():  # lorentzian.rs:88-131 (doc tests)
    assert approx_eq(oracle.superposition_vec([5.0], [[0.045, 0.0225, 5.0]])[0], 2.0)
    triplet = [[0.03, 0.0009, 4.8], [0.02, 0.0004, 5.0], [0.03, 0.0009, 5.2]]
    assert abs(oracle.superposition_vec([5.0], triplet)[0] - 51.466992) <= 1e-6


# ---------------------------------------------------------------- spectrum / deconvoluter
def test_signal_boundaries_indices():  # spectrum.rs:731-738 (doc test)
    x = np.array([1.0, 2.0, 3.0, 4.0, 5.0])
    # exercise via ignore_region_indices' internal sbi: an ignore region spanning
    # everything is clamped to exactly (sbi.0, sbi.1)
    assert oracle.ignore_region_indices(x, (2.25, 3.75), [(0.0, 10.0)]) == [(1, 3)]
    r = oracle.deconvolute(x, x, (2.25, 3.75))
    assert r.sbi == (1, 3)


def test_default_settings():  # deconvoluter.rs:218-275 (doc), smoother/selector/fitter defaults
    s = oracle.default_settings()
    assert (s.smoother, s.smooth_iterations, s.smooth_window) == (1, 3, 3)
    assert (s.selector, s.scoring, s.threshold) == (1, 0, 5.0)
    assert (s.fitter, s.fit_iterations) == (0, 10)


@pytest.mark.parametrize(
    "kw,code",
    [  # deconvoluter.rs:922-1010
        (dict(smooth_iterations=0, smooth_window=3), 10),
        (dict(smooth_iterations=2, smooth_window=0), 10),
        (dict(smooth_iterations=0, smooth_window=0), 10),
        (dict(smooth_window=1), 10),
        (dict(threshold=0.0), 11),
        (dict(threshold=float("nan")), 11),
        (dict(threshold=float("inf")), 11),
        (dict(threshold=float("-inf")), 11),
        (dict(fit_iterations=0), 12),
    ],
)
def test_invalid_settings(kw, code):
    s = oracle.make_settings(**kw)
    assert oracle.lib().mdo_validate_settings(s) == code


def test_add_ignore_region_merge():  # deconvoluter.rs:1012-1026 and doc :421-437
    r = oracle.add_ignore_region([], (1.0, 2.0))
    r = oracle.add_ignore_region(r, (3.0, 4.0))
    assert len(r) == 2
    r = oracle.add_ignore_region(r, (2.0, 3.0))
    assert len(r) == 1 and approx_eq(r[0][0], 1.0) and approx_eq(r[0][1], 4.0)
    r = oracle.add_ignore_region([], (4.7, 4.9))
    r = oracle.add_ignore_region(r, (5.2, 5.6))
    assert len(r) == 2
    r = oracle.add_ignore_region(r, (4.8, 5.4))
    assert len(r) == 1


@pytest.mark.parametrize(
    "region",
    [  # deconvoluter.rs:1028-1074
        (float("nan"), 1.0), (1.0, float("nan")), (float("inf"), 1.0), (1.0, float("inf")),
        (float("-inf"), 1.0), (1.0, float("-inf")), (1.0, 1.0),
    ],
)
def test_invalid_ignore_region(region):
    with pytest.raises(ValueError):
        oracle.add_ignore_region([], region)


# ---------------------------------------------------------------- moving average semantics
def test_moving_average_running_sum_semantics():
    """moving_average.rs:53-83 has no numeric test in the reference; pin the edge
    handling its doc table describes (window grows 2->3 at the left edge, shrinks at
    the right edge) on exactly representable data."""
    v = np.array([3.0, 6.0, 9.0, 12.0, 15.0])
    out = oracle.moving_average(v, 1, 3)
    exp = [(3 + 6) / 2, (3 + 6 + 9) * (1 / 3), (6 + 9 + 12) * (1 / 3), (9 + 12 + 15) * (1 / 3),
           (12 + 15) / 2]
    assert np.array_equal(out, np.array(exp))
    # window 5: right = 2; left edge windows 3, 4, 5 elements
    v = np.arange(1.0, 9.0)
    out = oracle.moving_average(v, 1, 5)
    assert out[0] == (1 + 2 + 3) * (1 / 3)
    assert out[1] == (1 + 2 + 3 + 4) * (1 / 4)
    assert out[2] == (1 + 2 + 3 + 4 + 5) * (1 / 5)
    assert out[-1] == (6 + 7 + 8) * (1 / 3)
