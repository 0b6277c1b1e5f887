"""The committed golden fixtures equal the live oracle (neither side drifted)."""
import os

import numpy as np
import pytest

import oracle
from tests.conftest import GOLDEN
from tests.golden.cases import CASES, load_case

FAST = [c for c in CASES if not c.startswith("synth_")]


@pytest.mark.parametrize("name", FAST)
def test_golden_matches_oracle(name):
    g = np.load(os.path.join(GOLDEN, "expected", f"{name}.npz"))
    x, y, sb, st, ign = load_case(name)
    r = oracle.deconvolute(x, y, sb, st, ignore=ign)
    assert r.status == int(g["status"])
    assert np.array_equal(r.params, g["params"])
    assert r.mse == float(g["mse"])
    assert np.array_equal(r.selected, g["selected"])


def test_par_equals_seq_oracle():
    """par_deconvolute_spectrum == deconvolute_spectrum bitwise."""
    x, y, sb, st, ign = load_case("blood_03")
    a = oracle.deconvolute(x, y, sb, st, threads=1)
    b = oracle.deconvolute(x, y, sb, st, threads=8)
    assert np.array_equal(a.params, b.params) and a.mse == b.mse


def test_sim_recovers_ground_truth_roughly():
    """Physical sanity only (NOT parity): sim_01's fitted peaks sit on the
    generating Lorentzians of data/bruker/sim/sim_01/lorentzians.csv."""
    truth = np.loadtxt(os.path.join(GOLDEN, "bruker", "sim", "sim_01", "lorentzians.csv"),
                       delimiter=",", skiprows=1)
    g = np.load(os.path.join(GOLDEN, "expected", "sim_01.npz"))
    fitted = g["params"][:, 2]
    d = np.abs(fitted[:, None] - truth[None, :, 2]).min(axis=1)
    assert np.median(d) < 2e-3
