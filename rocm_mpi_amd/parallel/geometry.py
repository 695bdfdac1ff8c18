"""Implicit-global-grid geometry (ImplicitGlobalGrid nx_g / x_g semantics).

Pure functions of the grid description; no communication. Reference call
sites: ``dx = lx/nx_g()`` (scripts/diffusion_2D_ap.jl:19) and the initial
condition ``x_g(ix,dx,T)`` (ap.jl:28). SURVEY.md C17:

* ``nx_g = dims*(nx-overlap) + overlap`` for an open (non-periodic) dimension,
  ``dims*(nx-overlap)`` for a periodic one;
* ``x_g(ix) = (coords*(nx-overlap) + ix)*dx + x0`` with 0-based ``ix`` (IGG's
  1-based ``ix-1``) and ``x0 = 0.5*(nx - size(A,1))*dx`` for staggered arrays;
  periodic dimensions shift by one cell (the first cell is a ghost) and wrap.
"""
from __future__ import annotations

import torch


def n_global(n_local: int, dims: int, overlap: int, periodic: int) -> int:
    return dims * (n_local - overlap) + (0 if periodic else overlap)


def coord(ix, d: float, coords: int, n_local: int, n_A: int, overlap: int, n_g: int,
          periodic: int):
    """Global coordinate of 0-based local index ``ix`` (scalar or tensor)."""
    x0 = 0.5 * (n_local - n_A) * d
    x = (coords * (n_local - overlap) + ix) * d + x0
    if periodic:
        x = x - d
        if isinstance(x, torch.Tensor):
            x = torch.where(x > (n_g - 1) * d, x - n_g * d, x)
            x = torch.where(x < 0, x + n_g * d, x)
        else:
            if x > (n_g - 1) * d:
                x = x - n_g * d
            if x < 0:
                x = x + n_g * d
    return x


def coords_1d(g0: int, n: int, d: float, off: float, n_g: int, periodic: int) -> torch.Tensor:
    """Vector of global coordinates of a tile row/column (matches the kernel)."""
    g = torch.arange(g0, g0 + n, dtype=torch.float64)
    x = g * d + off
    if periodic:
        x = x - d
        x = torch.where(x > (n_g - 1) * d, x - n_g * d, x)
        x = torch.where(x < 0, x + n_g * d, x)
    return x
