"""CPU: the out-of-range cases of tests/golden/range_cases.py do what they claim.

The oracle's range_mask (bit v: parameter version v has a value outside the engine's
fast-division ranges) is pinned for each scaled spectrum, so the GPU test's
comparison of the engine's slow launches against it exercises mid-fit flips of
both kinds. The oracle is test infrastructure (md_oracle.c)."""
import oracle
from tests.golden.range_cases import RANGE_CASES, mask_bits, range_case

import pytest


@pytest.mark.parametrize("case", RANGE_CASES, ids=[c[0] for c in RANGE_CASES])
def test_range_case_masks(case):
    x, y, sb, st, ign = range_case(case)
    r = oracle.deconvolute(x, y, sb, st, ignore=ign)
    assert r.status == 0
    assert r.range_mask == mask_bits(case[4]), format(r.range_mask, "011b")[::-1]
    assert (r.unsafe_kept > 0) == case[5]
    assert r.x_ok == (case[3] == 1.0)
