#!/usr/bin/env python
"""A 2D heat-diffusion solver written the way the reference's scripts use
ImplicitGlobalGrid (``/root/reference/scripts/diffusion_2D_perf.jl:15-60`` and
``diffusion_2D_perf_hide.jl:30-112``): the user owns the arrays and the time
loop, the package supplies the implicit global grid, the halo update and the
HIP stencil kernel.

    python examples/diffusion_2D_user.py --nx 4096 --ny 4096 --nt 200
    python -m rocm_mpi_amd.launch -n 4 -- examples/diffusion_2D_user.py --hide
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        examples/diffusion_2D_user.py --device cpu           # gloo, CPU twins

This is the composable API, one kernel launch and one ``update_halo_`` per
step. ``rocm_mpi_amd.models.Diffusion2D`` (and ``bench.py``) run the same
physics through the native executor instead: up to 24 steps per kernel pass,
width-K halos, hipGraph replay, which is what the performance numbers measure.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import rocm_mpi_amd as igg  # noqa: E402
from rocm_mpi_amd import ops  # noqa: E402


def diffusion2D(nx: int = 256, ny: int = 256, nt: int = 100, *, device: str | None = None,
                dims=(0, 0), hide: bool = False, b_width=(32, 4), warmup: int = 10,
                quiet: bool = False, finalize: bool = True, grid_kw: dict | None = None):
    """Run the reference problem; returns (T0_global, T_global, wtime) on rank 0
    (interiors gathered, halo excluded) and (None, None, wtime) elsewhere.
    ``grid_kw``: extra init_global_grid arguments (periods, transport, ...)."""
    # Physics (perf.jl:17-19)
    lx, ly = 10.0, 10.0
    lam, Cp0 = 1.0, 1.0
    me, dims, nprocs, coords, _ = igg.init_global_grid(nx, ny, 1, dimx=dims[0], dimy=dims[1],
                                                       device=device, quiet=quiet,
                                                       **(grid_kw or {}))
    dev = igg.global_grid().device
    dx, dy = lx / igg.nx_g(), ly / igg.ny_g()
    dt = min(dx * dx, dy * dy) * Cp0 / lam / 4.1
    coef = ops.StencilCoef.from_physics(lam, dx, dy, dt)
    # Arrays: (ny, nx) row-major == Julia's T[ix, iy]; the initial condition
    # from the global coordinates, as the reference's array comprehension
    f64 = dict(dtype=torch.float64)
    x = torch.tensor([igg.x_g(ix, dx, nx) for ix in range(nx)], **f64)
    y = torch.tensor([igg.y_g(iy, dy, ny) for iy in range(ny)], **f64)
    a = (x + dx / 2) - lx / 2
    b = (y + dy / 2) - ly / 2
    T = torch.exp(-(a * a)[None, :] - (b * b)[:, None]).to(dev)
    iCp = torch.full((ny, nx), 1.0 / Cp0, device=dev, **f64)
    T2 = T.clone()
    T0 = T[1:-1, 1:-1].contiguous().cpu()

    frame, inner = ops.hide_rects(nx, ny, *b_width)
    streams = None
    if hide and T.is_cuda:  # perf_hide.jl:63-68: high-priority frame, low-priority interior
        streams = (torch.cuda.Stream(dev, priority=-1), torch.cuda.Stream(dev, priority=0))

    for it in range(nt):
        if it == warmup:
            igg.tic()
        if streams is None:
            ops.stencil_step(T2, T, iCp, coef)          # perf.jl:46-48
            T, T2 = T2, T
            igg.update_halo_(T)                          # perf.jl:51
        else:
            hi, lo = streams
            cur = torch.cuda.current_stream(dev)
            hi.wait_stream(cur)
            lo.wait_stream(cur)
            with torch.cuda.stream(hi):                 # the send planes first ...
                ops.stencil_step(T2, T, iCp, coef, rects=frame)
                igg.update_halo_(T2)                     # ... exchanged while
            if inner is not None:
                with torch.cuda.stream(lo):             # ... the interior runs
                    ops.stencil_step(T2, T, iCp, coef, rects=[inner])
            cur.wait_stream(hi)
            cur.wait_stream(lo)
            T, T2 = T2, T
    wtime = igg.toc() if nt > warmup else float("nan")

    # perf.jl:55-58
    A_eff = (2 + 1) / 1e9 * nx * ny * 8
    if nt > warmup and me == 0 and not quiet:
        T_eff = A_eff / (wtime / (nt - warmup))
        print(f"Executed {nt} steps in = {wtime:1.3e} sec (@ T_eff = {T_eff:1.2f} GB/s)")
    T0_g = igg.gather_(T0)
    T_g = igg.gather_(T[1:-1, 1:-1].contiguous().cpu())
    if me == 0 and not quiet:
        print(f"max(T_v) = {float(T_g.max()):.6f} on {nprocs} rank(s), dims {tuple(dims[:2])}")
    if finalize:
        igg.finalize_global_grid()
    return T0_g, T_g, wtime


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--nx", type=int, default=4096)
    ap.add_argument("--ny", type=int, default=4096)
    ap.add_argument("--nt", type=int, default=100)
    ap.add_argument("--device", default=None, help="cpu / cuda (default: cuda when present)")
    ap.add_argument("--hide", action="store_true", help="perf_hide's frame/interior split")
    ap.add_argument("--b-width", type=lambda s: tuple(int(v) for v in s.split(",")),
                    default=(32, 4))
    a = ap.parse_args(argv)
    diffusion2D(a.nx, a.ny, a.nt, device=a.device, hide=a.hide, b_width=a.b_width)
    return 0


if __name__ == "__main__":
    sys.exit(main())
