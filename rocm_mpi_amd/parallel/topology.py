"""Cartesian topology (MPI Dims_create / Cart_create / Cart_coords / Cart_shift).

The native implementation (``csrc/runtime/topology.cpp``) is authoritative;
``py_dims_create`` / ``PyCartTopology`` are independent pure-Python twins used
as a test oracle and when the extension is unavailable.
"""
from __future__ import annotations

from typing import Sequence

from .._native import has_native, native

PROC_NULL = -1


def py_dims_create(nprocs: int, dims: Sequence[int]) -> list[int]:
    dims = list(dims) + [0] * (3 - len(dims))
    if nprocs < 1 or any(d < 0 for d in dims):
        raise ValueError("invalid nprocs/dims")
    fixed = 1
    free = []
    for i, d in enumerate(dims):
        if d > 0:
            fixed *= d
        else:
            free.append(i)
    if nprocs % fixed:
        raise ValueError(f"nprocs={nprocs} not divisible by fixed dims product {fixed}")
    rest = nprocs // fixed
    if not free:
        if rest != 1:
            raise ValueError("prod(dims) != nprocs")
        return dims
    primes = []
    p = 2
    while p * p <= rest:
        while rest % p == 0:
            primes.append(p)
            rest //= p
        p += 1
    if rest > 1:
        primes.append(rest)
    slots = [1] * len(free)
    for q in sorted(primes, reverse=True):
        i = slots.index(min(slots))
        slots[i] *= q
    slots.sort(reverse=True)
    for i, d in zip(free, slots):
        dims[i] = d
    return dims


def dims_create(nprocs: int, dims: Sequence[int]) -> list[int]:
    dims = list(dims) + [0] * (3 - len(dims))
    if has_native():
        try:
            return list(native().dims_create(int(nprocs), dims))
        except RuntimeError as e:
            raise ValueError(str(e)) from None
    return py_dims_create(nprocs, dims)


class PyCartTopology:
    def __init__(self, nprocs: int, dims: Sequence[int], periods: Sequence[int]):
        self.nprocs = nprocs
        self.dims = list(dims)
        self.periods = list(periods)
        if self.dims[0] * self.dims[1] * self.dims[2] != nprocs:
            raise ValueError("prod(dims) != nprocs")

    def coords(self, rank: int) -> list[int]:
        d = self.dims
        return [rank // (d[2] * d[1]), (rank // d[2]) % d[1], rank % d[2]]

    def rank_of(self, c: Sequence[int]) -> int:
        c = list(c)
        for i in range(3):
            if not 0 <= c[i] < self.dims[i]:
                if not self.periods[i]:
                    return PROC_NULL
                c[i] %= self.dims[i]
        return (c[0] * self.dims[1] + c[1]) * self.dims[2] + c[2]

    def shift(self, rank: int, dim: int) -> list[int]:
        lo, hi = self.coords(rank), self.coords(rank)
        lo[dim] -= 1
        hi[dim] += 1
        return [self.rank_of(lo), self.rank_of(hi)]

    def neighbors(self, rank: int) -> list[list[int]]:
        return [self.shift(rank, d) for d in range(3)]

    def diagonals(self, rank: int) -> list[int]:
        """Ranks at (x-1,y-1), (x+1,y-1), (x-1,y+1), (x+1,y+1) (-1 outside)."""
        c = self.coords(rank)
        out = []
        for k in range(4):
            d = list(c)
            d[0] += 1 if k & 1 else -1
            d[1] += 1 if k & 2 else -1
            out.append(self.rank_of(d))
        return out


def CartTopology(nprocs: int, dims: Sequence[int], periods: Sequence[int]):
    if has_native():
        return native().CartTopology(int(nprocs), list(dims), [int(p) for p in periods])
    return PyCartTopology(nprocs, dims, periods)
