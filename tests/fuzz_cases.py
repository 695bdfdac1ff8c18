"""Random multi-rank configurations shared by test_fuzz_cpu.py / test_fuzz_gpu.py:
a process grid, periodic dimensions, tile size, pass depth K (1..24), step count,
frame width, variant and arithmetic drawn from a fixed seed, run on P loopback
ranks."""
import random

import numpy as np

from helpers import run_loopback
from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
from rocm_mpi_amd.parallel import implicit_grid as gg

DIMS = [(1, 1), (2, 1), (1, 2), (2, 2), (3, 1), (1, 3), (3, 2), (4, 2)]


def case(seed):
    r = random.Random(seed)
    dims = r.choice(DIMS)
    K = r.randint(1, 24)
    nx = 4 * K + r.randint(6, 120)
    ny = 4 * K + r.randint(6, 90)
    return dict(dims=dims, K=K, nx=nx, ny=ny, nt=r.randint(1, 3 * K + 4),
                variant=r.choice(["perf", "perf_hide"]), fast=r.random() < 0.6,
                bw=(r.randint(1, 9), r.randint(1, 9)),
                periods=(int(r.random() < 0.3), int(r.random() < 0.3)))


def spmd(rank, hub, c, device):
    K, dims = c["K"], c["dims"]
    per = c["periods"]
    gg.init_global_grid(c["nx"], c["ny"], 1, dimx=dims[0], dimy=dims[1], periodx=per[0],
                        periody=per[1], overlaps=(2 * K, 2 * K, 2), halowidths=(K, K, 1),
                        quiet=True, loopback=(hub, rank), device=device)
    m = Diffusion2D(DiffusionConfig(variant=c["variant"], nx=c["nx"], ny=c["ny"], nt=c["nt"],
                                    init="random", quiet=True, dims=(*dims, 0), temporal=K,
                                    fast_math=c["fast"], b_width=c["bw"], device=device,
                                    periods=(*per, 0)))
    if device != "cpu":
        assert m.executor is not None
    m.step(c["nt"])
    out = (m.g.coords, m.field.cpu().numpy().copy(), m.g.nxyz_g)
    m.close()
    gg.finalize_global_grid()
    return out


def check(seed, device):
    """Every tile of the P-rank run on ``device`` == the same region of a 1-rank
    CPU run of the global grid, bitwise."""
    c = case(seed)
    P = c["dims"][0] * c["dims"][1]
    res = run_loopback(P, spmd, c, device, timeout=180)
    nxg, nyg, _ = res[0][2]
    # the 1-rank grid with the same global size: a periodic dimension keeps its
    # overlap on top (nx_g = dims * (nx - ol) there), so tile c's window starts
    # at c * (nx - ol) in both cases
    ol = 2 * c["K"]
    one = dict(c, nx=nxg + ol * c["periods"][0], ny=nyg + ol * c["periods"][1], dims=(1, 1))
    ref = run_loopback(1, spmd, one, "cpu", timeout=180)[0][1]
    K = c["K"]
    for coords, T, _ in res:
        gx0, gy0 = coords[0] * (c["nx"] - 2 * K), coords[1] * (c["ny"] - 2 * K)
        assert np.array_equal(T, ref[gy0:gy0 + c["ny"], gx0:gx0 + c["nx"]]), (c, coords)
