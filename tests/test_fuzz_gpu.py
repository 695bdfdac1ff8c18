"""Randomised decomposition-invariance of the native GPU path.

P loopback ranks run the native executor on the GPU (planned passes, width-K
exchanges, frame/interior streams) for random configurations (fuzz_cases.py);
every tile must equal the same region of a 1-rank CPU run of the global grid
bitwise (the CPU twins of the same arithmetic). Complements the hand-picked
cases of test_multirank_gpu.py with sizes and depths nobody chose."""
import pytest

from fuzz_cases import check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(128))
def test_random_decompositions_match_one_cpu_rank(seed):
    check(seed, "cuda")
