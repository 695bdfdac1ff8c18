"""Cartesian topology: MPI Dims_create / Cart semantics (native vs Python twin)."""
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from rocm_mpi_amd._native import native
from rocm_mpi_amd.parallel.topology import (PROC_NULL, CartTopology, PyCartTopology,
                                            dims_create, py_dims_create)


@pytest.mark.parametrize("n,dims,want", [
    (1, [0, 0, 1], [1, 1, 1]), (2, [0, 0, 1], [2, 1, 1]), (4, [0, 0, 1], [2, 2, 1]),
    (8, [0, 0, 1], [4, 2, 1]), (6, [0, 0, 1], [3, 2, 1]), (12, [0, 0, 1], [4, 3, 1]),
    (8, [0, 0, 0], [2, 2, 2]), (16, [0, 0, 0], [4, 2, 2]), (8, [1, 0, 1], [1, 8, 1]),
    (12, [0, 2, 0], [3, 2, 2]), (7, [0, 0, 1], [7, 1, 1]), (36, [0, 0, 1], [6, 6, 1]),
])
def test_dims_create_known(n, dims, want):
    assert dims_create(n, dims) == want
    assert py_dims_create(n, dims) == want


def test_dims_create_errors():
    with pytest.raises(ValueError):
        dims_create(6, [4, 0, 1])
    with pytest.raises(ValueError):
        dims_create(4, [2, 1, 1])


@settings(max_examples=200, deadline=None)
@given(st.integers(1, 512), st.lists(st.integers(0, 4), min_size=3, max_size=3))
def test_dims_create_property(n, dims):
    try:
        a = py_dims_create(n, dims)
    except ValueError:
        with pytest.raises(ValueError):
            dims_create(n, dims)
        return
    b = dims_create(n, dims)
    assert a == b
    assert b[0] * b[1] * b[2] == n
    for i in range(3):
        if dims[i] > 0:
            assert b[i] == dims[i]
    free = [b[i] for i in range(3) if dims[i] == 0]
    assert free == sorted(free, reverse=True)


@settings(max_examples=100, deadline=None)
@given(st.integers(1, 6), st.integers(1, 6), st.integers(1, 3), st.lists(st.integers(0, 1),
                                                                           min_size=3, max_size=3))
def test_cart_bijection_and_neighbour_symmetry(d0, d1, d2, periods):
    n = d0 * d1 * d2
    nat = CartTopology(n, [d0, d1, d2], periods)
    py = PyCartTopology(n, [d0, d1, d2], periods)
    seen = set()
    for r in range(n):
        c = list(nat.coords(r))
        assert c == py.coords(r)
        assert nat.rank_of(c) == r
        seen.add(tuple(c))
        nb = [list(x) for x in nat.neighbors(r)]
        assert nb == py.neighbors(r)
        for d in range(3):
            lo, hi = nb[d]
            if hi != PROC_NULL:
                assert list(nat.neighbors(hi))[d][0] == r
            if lo != PROC_NULL:
                assert list(nat.neighbors(lo))[d][1] == r
            if not periods[d]:
                assert (lo == PROC_NULL) == (c[d] == 0)
                assert (hi == PROC_NULL) == (c[d] == [d0, d1, d2][d] - 1)
    assert len(seen) == n


def test_mpi_row_major_order():
    t = native().CartTopology(4, [2, 2, 1], [0, 0, 0])
    assert [list(t.coords(r)) for r in range(4)] == [[0, 0, 0], [0, 1, 0], [1, 0, 0], [1, 1, 0]]
