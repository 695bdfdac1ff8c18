"""Randomised decomposition-invariance on the CPU (Python pass loop with the
C++ CPU twins, loopback ranks): the same random configurations as
test_fuzz_gpu.py (fuzz_cases.py)."""
import pytest

from fuzz_cases import check


@pytest.mark.parametrize("seed", range(128))
def test_random_decompositions_match_one_rank_cpu(seed):
    check(seed, "cpu")
