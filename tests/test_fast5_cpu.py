"""The fast-math (fast5) arithmetic pinned on the CPU: the C++ twin
(stencilk5_rects_cpu, std::fma) against an independent exact-rational golden
model (tests/golden.py run5), bitwise; the torch fallback twin; and the
fast-math multi-rank path (loopback ranks on the CPU twins) against the
1-rank run of the global grid, bitwise, across decompositions and planned pass
depths. The GPU kernels are pinned to the same twin in tests/test_pipe_gpu.py,
so the bench's headline arithmetic is checked bitwise end to end."""
import numpy as np
import pytest
import torch

import golden
from helpers import run_loopback
from rocm_mpi_amd import ops
from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
from rocm_mpi_amd.parallel import implicit_grid as gg


def coef():
    return ops.StencilCoef(-1.3, 1 / 0.037, 1 / 0.041, 0.00031)


def rand(shape, seed, lo=0.0, hi=1.0):
    g = torch.Generator().manual_seed(seed)
    return lo + (hi - lo) * torch.rand(shape, generator=g, dtype=torch.float64)


@pytest.mark.parametrize("K", [1, 2, 5])
def test_fast5_cpu_twin_equals_exact_golden(K):
    ny, nx = 11, 13
    T, iCp = rand((ny, nx), 1), rand((ny, nx), 2, 0.5, 1.0)
    out = torch.full_like(T, -5.0)
    ops.stencilk_step(K, out, T, iCp, coef(), None, ops.StencilTuning(kernel="pipe"))
    ref = golden.run5(T.numpy(), iCp.numpy(), K, *coef())
    inner = np.full_like(ref, -5.0)
    inner[1:-1, 1:-1] = ref[1:-1, 1:-1]
    assert np.array_equal(out.numpy(), inner)


def test_fast5_differs_from_canonical_but_rounding_close():
    ny, nx = 20, 24
    T, iCp = rand((ny, nx), 3), rand((ny, nx), 4, 0.5, 1.0)
    a, b = torch.zeros_like(T), torch.zeros_like(T)
    ops.stencilk_step(6, a, T, iCp, coef(), None, ops.StencilTuning(kernel="pipe"))
    ops.stencilk_step(6, b, T, iCp, coef(), None, ops.StencilTuning(kernel="pipec"))
    assert not torch.equal(a, b)
    assert float((a - b).abs().max()) < 1e-14


def test_torch_fma_fallback_matches_twin():
    ny, nx = 40, 52
    T, iCp = rand((ny, nx), 5), rand((ny, nx), 6, 0.5, 1.0)
    a, b = torch.zeros_like(T), torch.zeros_like(T)
    ops.stencilk_step(1, a, T, iCp, coef(), None, ops.StencilTuning(kernel="pipe"))
    ops.stencil5_torch(b, T, iCp, coef(), [ops.interior_rect(nx, ny)])
    # the double-double fma rounds like std::fma except in rare tie cases
    assert int((a != b).sum()) <= 2
    assert float((a - b).abs().max()) < 1e-15


def spmd_fast(rank, hub, nx, ny, nt, dims, K):
    gg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1], overlaps=(2 * K, 2 * K, 2),
                        halowidths=(K, K, 1), quiet=True, loopback=(hub, rank), device="cpu")
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny, nt=nt, init="random",
                                    quiet=True, dims=(*dims, 0), temporal=K, fast_math=True,
                                    device="cpu"))
    plan = m.plan(nt)
    m.step(nt)
    out = (m.g.coords, m.field.numpy().copy(), m.g.nxyz_g, plan)
    m.close()
    return out


@pytest.mark.parametrize("P,dims,K,nt", [(2, (2, 1), 4, 11), (4, (2, 2), 7, 23),
                                         (4, (1, 4), 16, 37), (8, (4, 2), 24, 29)])
def test_fast_math_decomposition_invariant_on_cpu(P, dims, K, nt):
    nx = ny = 6 * K + 4
    res = run_loopback(P, spmd_fast, nx, ny, nt, dims, K, timeout=240)
    nxg, nyg, _ = res[0][2]
    assert sum(res[0][3]) == nt and max(res[0][3]) <= K
    one = run_loopback(1, spmd_fast, nxg, nyg, nt, (1, 1), K, timeout=240)[0][1]
    for coords, T, _, _ in res:
        gx0, gy0 = coords[0] * (nx - 2 * K), coords[1] * (ny - 2 * K)
        assert np.array_equal(T, one[gy0:gy0 + ny, gx0:gx0 + nx])


def test_fma_exact_against_correct_rounding():
    """fma_exact (the no-extension fallback's fma emulation) vs the
    correctly rounded fma computed in exact rationals (float(Fraction) rounds
    to nearest even): equal on random operands of mixed magnitude and under
    near-total cancellation; on constructed near-ties (exact result within a
    tiny distance of a rounding boundary) at most one ulp away, as its
    docstring states."""
    import fractions
    import random

    import torch

    from rocm_mpi_amd.ops import fma_exact

    F = fractions.Fraction
    rng = random.Random(7)
    n = 3000

    def exact(a, b, c):
        return torch.tensor([float(F(x) * F(y) + F(z)) for x, y, z in
                             zip(a.tolist(), b.tolist(), c.tolist())], dtype=torch.float64)

    a = torch.tensor([rng.uniform(-1, 1) for _ in range(n)], dtype=torch.float64)
    b = torch.tensor([rng.uniform(-1, 1) * 10 ** rng.randint(-3, 3) for _ in range(n)],
                     dtype=torch.float64)
    c = torch.tensor([rng.uniform(-1, 1) * 10 ** rng.randint(-3, 3) for _ in range(n)],
                     dtype=torch.float64)
    assert torch.equal(fma_exact(a, b, c), exact(a, b, c))
    c2 = -(a * b) * (1 + torch.tensor([rng.uniform(-1e-15, 1e-15) for _ in range(n)],
                                      dtype=torch.float64))
    assert torch.equal(fma_exact(a, b, c2), exact(a, b, c2))
    # near-ties: c = -round(a*b) + half an ulp of the product (+- a hair)
    p = a * b
    half = torch.nextafter(p.abs(), torch.full_like(p, float("inf"))) - p.abs()
    c3 = half / 2 * torch.sign(p) + torch.tensor([rng.choice((-1, 1)) * 2.0 ** -80
                                                  for _ in range(n)], dtype=torch.float64)
    r3, e3 = fma_exact(a, b, c3), exact(a, b, c3)
    ulp = torch.nextafter(e3.abs(), torch.full_like(e3, float("inf"))) - e3.abs()
    assert bool(((r3 - e3).abs() <= ulp).all())
