"""Fast-math drift at the headline run lengths.

The timed passes use the fast-math fp64 arithmetic (one folded per-cell
factor, FMAs), bitwise equal to its CPU twin but not to the canonical update
(scripts/diffusion_2D_perf.jl:8-10). Diffusion is contractive, so the
rounding differences do not accumulate: after 1000 and 20000 steps (the
reference's nt = 1e3 and the sustained bench length) on a 2050^2 random field
the max |fast - canonical| stays at a few ulps of the field's O(1) values.
The bound is bench.DRIFT_BOUND, the one the bench record carries."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


@pytest.mark.parametrize("steps", [1000, 20000])
def test_fast_math_drift_bounded_at_headline_length(steps):
    import bench

    info = bench.drift_check(2050, 24, steps, "cuda", 1, 60.0)
    assert info["steps"] == steps
    assert 0 <= info["fast_math_drift_max"] <= bench.DRIFT_BOUND == 1e-14
