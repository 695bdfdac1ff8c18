"""Shared command line of the diffusion entry points.

The reference hard-codes its parameters per script (e.g.
``scripts/diffusion_2D_perf.jl:17-25``) and selects the variant by
(un)commenting ``scripts/runme.sh:5-9``. Every entry point here keeps the
reference's defaults and exposes them as flags, plus the BASELINE.json
configurations as named presets (``--preset``).

The reference's global problem is kept by default: one step per kernel pass,
the canonical flux-form arithmetic, IGG's overlap 2, so ``--dims 2,1 --nx
12288`` solves ``nx_g = 2*(12288-2)+2 = 24574`` (``diffusion_2D_perf.jl:22,
26,28``). The measured bench path (up to 24 steps per pass, fast-math,
``bench.py``) is opt-in: ``--bench-plan``, an explicit ``--temporal K``, or a
BASELINE preset. K-step passes need width-K halos, i.e. grid overlap 2K, which
changes ``nx_g``, ``dx`` and ``dt`` on a multi-rank grid: the run then prints
both grids (``[grid]`` line) and records them (result ``extra``, checkpoint).
"""
from __future__ import annotations

import argparse
import math
import os
import sys

# Reference defaults per script.
DEFAULTS = {
    "ap": dict(nx=128, ny=128, nt=1000, do_vis=True),                      # ap.jl:15-16
    "kp": dict(nx=128, ny=128, nt=1000, do_vis=True),                      # kp.jl:62-65
    "perf": dict(nx=12 * 1024, ny=12 * 1024, nt=1000, do_vis=False),       # perf.jl:21-25
    "perf_hide": dict(nx=12 * 1024, ny=12 * 1024, nt=100,                   # perf_hide.jl:37-43
                      do_vis=False),
    "perf_hide_prof": dict(nx=8 * 1024, ny=8 * 1024, nt=300,               # _prof.jl:71-77
                           do_vis=False, profile=True, threads=(32, 4)),
}

# What bench.py runs (its --temporal default, fast-math on). With
# --bench-plan (or a BASELINE preset) the perf / perf_hide entry points run
# the same planner and kernels on tiles big enough to fill the GPU with K-step
# tasks (below ~1.5M cells one step per pass is faster, see Diffusion2D's
# warning). Without it they keep the reference's one-step canonical update
# and its overlap-2 global grid.
BENCH_TEMPORAL = 24
AUTO_TEMPORAL_MIN_CELLS = 1_500_000


def auto_temporal(variant: str, nx: int, ny: int, temporal=None, fast_math=None,
                  bench_plan: bool = False) -> tuple:
    """(temporal, fast_math) of a run: explicit values win; otherwise one
    canonical step per pass (the reference), or with ``bench_plan`` the
    bench.py defaults for perf / perf_hide on tiles of >= 1.5M cells."""
    base = "perf_hide" if variant == "perf_hide_prof" else variant
    if base not in ("perf", "perf_hide"):
        return 1, False
    if temporal is None:
        temporal = (BENCH_TEMPORAL if bench_plan and nx * ny >= AUTO_TEMPORAL_MIN_CELLS
                    else 1)
    if fast_math is None:
        fast_math = temporal > 1
    return int(temporal), bool(fast_math)


# BASELINE.json "configs", in order (the perf ones as bench.py measures them).
PRESETS = {
    "ap256_cpu": dict(variant="ap", nx=256, ny=256, nt=1000, device="cpu"),
    "kp16k": dict(variant="kp", nx=16384, ny=16384, nt=1000),
    "perf_2x1": dict(variant="perf", nx=16384, ny=16384, nt=1000, dims=(2, 1, 0),
                     bench_plan=True),
    "hide_2x2": dict(variant="perf_hide", nx=16384, ny=16384, nt=1000, dims=(2, 2, 0),
                     bench_plan=True),
    "hide_4x2_288GB": dict(variant="perf_hide", auto_size=True, nt=1000, dims=(4, 2, 0),
                           bench_plan=True),
}


def global_sizes(nx: int, ny: int, dims, periods, nprocs: int, temporal: int) -> tuple:
    """((nx_g, ny_g) of the run, (nx_g, ny_g) with IGG's overlap 2): K-step
    passes (temporal K > 1) need overlap 2K (models/diffusion.py)."""
    from ..parallel import geometry as geo
    from ..parallel.topology import dims_create

    d = dims_create(nprocs, [int(dims[0]), int(dims[1]), 1])
    ol = 2 * temporal if temporal > 1 else 2
    run = tuple(geo.n_global(n, d[i], ol, int(periods[i])) for i, n in enumerate((nx, ny)))
    ref = tuple(geo.n_global(n, d[i], 2, int(periods[i])) for i, n in enumerate((nx, ny)))
    return run, ref


def grid_line(model) -> str | None:
    """The loud note when the solved global grid is not the reference's
    (overlap 2K of K-step passes on a multi-rank grid); None when equal."""
    g, cfg = model.g, model.cfg
    run = tuple(g.nxyz_g[:2])
    _, ref = global_sizes(cfg.nx, cfg.ny, g.dims, g.periods, g.nprocs, 1)
    if run == ref:
        return None
    dx_ref, dy_ref = cfg.lx / ref[0], cfg.ly / ref[1]
    dt_ref = min(dx_ref * dx_ref, dy_ref * dy_ref) * cfg.Cp0 / cfg.lam / 4.1
    return (f"[grid] global grid {run[0]}x{run[1]} (overlap {g.overlaps[0]} for "
            f"{cfg.temporal}-step passes), dx = {model.dx:.6e}, dt = {model.dt:.6e}; the "
            f"reference's overlap 2 gives {ref[0]}x{ref[1]}, dx = {dx_ref:.6e}, dt = "
            f"{dt_ref:.6e} (run with --temporal 1 to solve the reference's problem)")


def _pair(s: str) -> tuple:
    return tuple(int(v) for v in s.split(","))


def build_parser(variant: str) -> argparse.ArgumentParser:
    d = DEFAULTS[variant]
    ap = argparse.ArgumentParser(
        prog=f"diffusion_2D_{variant}",
        description=f"2D heat diffusion, {variant} variant (reference "
                    f"scripts/diffusion_2D_{variant}.jl) on MI355X")
    ap.add_argument("--preset", choices=sorted(PRESETS), help="a BASELINE.json configuration")
    ap.add_argument("--nx", type=int, default=d["nx"], help="local grid points in x (halo incl.)")
    ap.add_argument("--ny", type=int, default=d["ny"])
    ap.add_argument("--nt", type=int, default=d["nt"], help="time steps (first 10 untimed)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--threads", type=_pair, default=d.get("threads", (32, 8)),
                    help="accepted for compatibility with the reference's work-group shape "
                         "(perf.jl:23); the gfx950 kernels use 4 waves of 64 lanes marching "
                         "row chunks (tune with --chunk-rows / --vec) and record it only")
    ap.add_argument("--b-width", type=_pair, default=d.get("b_width", (1, 1)),
                    help="perf_hide frame width in cells (reference default 32,4)")
    ap.add_argument("--dims", type=_pair, default=(0, 0), help="process grid dimx,dimy")
    ap.add_argument("--periods", type=_pair, default=(0, 0))
    ap.add_argument("--init", choices=["gaussian", "random"], default="gaussian")
    ap.add_argument("--init-on", choices=["auto", "device", "host"], default="auto")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--transport", default=os.environ.get("RMA_TRANSPORT", "auto"),
                    choices=["auto", "rccl", "ipc", "staged", "gloo", "self"])
    ap.add_argument("--device", default=None, help="cpu, cuda, cuda:N (default: one GPU per rank)")
    ap.add_argument("--vis", dest="do_vis", action="store_true", default=d["do_vis"])
    ap.add_argument("--no-vis", dest="do_vis", action="store_false")
    ap.add_argument("--outdir", default="output")
    ap.add_argument("--profile", action="store_true", default=d.get("profile", False))
    ap.add_argument("--auto-size", action="store_true",
                    help="size the local tile to fill --hbm-frac of free HBM (288 GB MI355X)")
    ap.add_argument("--no-auto-size", dest="auto_size", action="store_false")
    ap.add_argument("--hbm-frac", type=float, default=0.80)
    ap.add_argument("--chunk-rows", type=int, default=4)
    ap.add_argument("--unroll", type=int, default=4)
    ap.add_argument("--kernel", choices=["march", "lds"], default="march")
    ap.add_argument("--nontemporal", type=int, default=3,
                    help="bitmask: 1 = NT T2 stores, 2 = NT 1/Cp loads, 4 = NT T loads")
    ap.add_argument("--vec", type=int, default=2, choices=[2, 4], help="cells per lane")
    ap.add_argument("--graph", action="store_true", help="replay steps from a hipGraph")
    ap.add_argument("--temporal", type=int, default=None, choices=list(range(1, 25)),
                    metavar="K",
                    help="perf/perf_hide: at most K (1..24) steps per kernel pass + width-K "
                         "halos (grid overlap 2K: a multi-rank nx_g differs from the "
                         "reference's); the executor plans the passes; bitwise identical to "
                         "one-step updates without --fast-math. Default: 1 (the reference), "
                         f"{BENCH_TEMPORAL} with --bench-plan on tiles of >= "
                         f"{AUTO_TEMPORAL_MIN_CELLS:,} cells")
    ap.add_argument("--bench-plan", dest="bench_plan", action="store_true", default=False,
                    help=f"perf/perf_hide: run what bench.py measures (up to {BENCH_TEMPORAL} "
                         "steps per pass, fast-math) on tiles of >= "
                         f"{AUTO_TEMPORAL_MIN_CELLS:,} cells; on a multi-rank grid the overlap "
                         "becomes 2K, which changes nx_g / dx / dt (printed)")
    ap.add_argument("--chunk2", type=int, default=0)
    ap.add_argument("--unroll2", type=int, default=2, choices=[2, 4])
    ap.add_argument("--fast-math", dest="fast_math", action="store_true", default=None,
                    help="passes with fast-math fp64 arithmetic (5-point sum, one folded "
                         "per-cell factor, FMAs): same scheme, not bitwise equal to the "
                         "canonical update, bitwise equal to its CPU twin (default with "
                         "K > 1 steps per pass, as in bench.py)")
    ap.add_argument("--canonical", dest="fast_math", action="store_false",
                    help="the bitwise-canonical arithmetic in every pass (the reference's "
                         "flux form; K-step passes stay bitwise equal to K one-step updates)")
    ap.add_argument("--halo-direct", dest="halo_direct", action="store_true",
                    help="direct-store halos: the K-step kernels store the neighbours' halo "
                         "cells into their fields (own periodic images, loopback ranks, IPC "
                         "processes of one node) instead of an exchange; fast-math perf / "
                         "perf_hide passes on a GPU (e.g. with --bench-plan)")
    ap.add_argument("--check-every", type=int, default=0, help="NaN/Inf guard period")
    ap.add_argument("--checkpoint", default="", help="save the final state to this directory")
    ap.add_argument("--resume", default="", help="start from a checkpoint directory")
    ap.add_argument("--json", action="store_true", help="print the run record as JSON (rank 0)")
    ap.add_argument("--quiet", action="store_true")
    return ap


def auto_tile(frac: float) -> int:
    import torch

    if not torch.cuda.is_available():
        raise RuntimeError("--auto-size needs a GPU")
    free, _ = torch.cuda.mem_get_info()
    return max(512, int(math.isqrt(int(frac * free / 24.0))) // 256 * 256)


def resolve(variant: str, argv=None):
    """Parse an entry point's command line into (DiffusionConfig, args); with
    --auto-size this selects the device and sizes the tile (collective)."""
    from ..models import DiffusionConfig
    from ..parallel import comm as C

    base = "perf_hide" if variant == "perf_hide_prof" else variant
    parser = build_parser(variant)
    pre, _ = parser.parse_known_args(argv)
    if pre.preset:  # a preset supplies defaults; explicit flags still win
        p = dict(PRESETS[pre.preset])
        pv = p.pop("variant")
        if pv != base:
            parser.error(f"preset {pre.preset} is a {pv} configuration, not {base}")
        if "dims" in p:
            p["dims"] = tuple(p["dims"][:2])
        parser.set_defaults(**p)
    a = parser.parse_args(argv)
    if a.temporal is not None and a.temporal > 1 and base not in ("perf", "perf_hide"):
        parser.error("--temporal > 1 applies to the perf and perf_hide variants")
    if a.fast_math and base not in ("perf", "perf_hide"):
        parser.error("--fast-math applies to the perf and perf_hide variants")
    if a.halo_direct and base not in ("perf", "perf_hide"):
        parser.error("--halo-direct applies to the perf and perf_hide variants")
    opts = dict(variant=base, nx=a.nx, ny=a.ny, nt=a.nt, warmup=a.warmup, b_width=a.b_width,
                init=a.init, init_on=a.init_on, seed=a.seed, dims=tuple(a.dims) + (0,),
                periods=tuple(a.periods) + (0,), transport=a.transport, device=a.device,
                chunk_rows=a.chunk_rows, unroll=a.unroll, vec=a.vec, kernel=a.kernel,
                nontemporal=a.nontemporal, use_graph=a.graph, do_vis=a.do_vis, outdir=a.outdir,
                profile=a.profile, check_every=a.check_every, quiet=a.quiet,
                chunk2=a.chunk2, unroll2=a.unroll2, halo_direct=a.halo_direct)
    if a.auto_size:
        rank, size, _ = C.env_world()
        if size > 1:
            C.init_distributed()
        local, _ = C.node_local_rank(rank, size)
        C.select_device(local)
        n = auto_tile(a.hbm_frac)
        if size > 1:
            import torch
            import torch.distributed as dist

            t = torch.tensor([n], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=C._gloo_group())
            n = int(t.item())
        opts["nx"] = opts["ny"] = n
    opts["temporal"], opts["fast_math"] = auto_temporal(base, opts["nx"], opts["ny"], a.temporal,
                                                        a.fast_math, a.bench_plan)
    return DiffusionConfig(**opts), a


def plan_line(model, steps: int) -> str:
    """What the timed loop runs: passes, kernel and arithmetic (printed next
    to the reference's T_eff line)."""
    import collections

    cfg = model.cfg
    plan = model.plan(steps)
    passes = ", ".join(f"{n} x {k}" for k, n in sorted(collections.Counter(plan).items(),
                                                         reverse=True))
    kern = ""
    if cfg.temporal > 1 or cfg.fast_math:
        try:
            from .. import ops
            from .._native import native

            K = max(plan) if plan else 1
            if cfg.fast_math and ops.fast5_ok(model.coef):
                kid = native().fast_kernel_k(K, cfg.ny, tuple(model.coef))[0]
            else:
                kid = native().canonical_kernel_k(K, cfg.ny)[0]
            kern = ", kernel " + ops.kernel_name(kid)
        except Exception:  # noqa: BLE001 - informational only
            pass
    arith = ("fast-math (5-point sum, folded factor; rounding-level vs canonical)"
             if cfg.fast_math else "canonical (bitwise = one-step updates)")
    return (f"[plan] {steps} timed steps in passes of {passes} step(s){kern}; "
            f"{arith}; max {cfg.temporal} steps per pass (--temporal, --canonical)")


def run_variant(variant: str, argv=None) -> int:
    from ..models import Diffusion2D
    from ..utils import checkpoint as ckpt

    cfg, a = resolve(variant, argv)
    model = Diffusion2D(cfg)
    if variant == "perf_hide_prof":  # warm-up call before the profiled run (_prof.jl:110)
        model.step(12)
        model.synchronize()
    if a.resume:
        ckpt.load_checkpoint(model, a.resume)
    gline = grid_line(model)
    if gline and model.g.me == 0:
        import warnings

        warnings.warn(gline, RuntimeWarning, stacklevel=2)
        if not cfg.quiet:
            print(gline, flush=True)
    res = model.run()
    if model.g.me == 0 and not cfg.quiet and cfg.variant in ("perf", "perf_hide"):
        print(plan_line(model, res.timed_steps), flush=True)
        if gline:
            print(gline, flush=True)
    if a.checkpoint:
        ckpt.save_checkpoint(model, a.checkpoint)
    res.extra["threads_requested"] = list(a.threads)
    res.extra["temporal"] = cfg.temporal
    res.extra["fast_math"] = bool(cfg.fast_math)
    res.extra["overlaps"] = list(model.g.overlaps[:2])
    res.extra["nxyz_g_reference"] = list(global_sizes(cfg.nx, cfg.ny, model.g.dims,
                                                      model.g.periods, model.g.nprocs, 1)[1])
    if a.json and model.g.me == 0:
        print(res.to_json(), flush=True)
    model.close()
    return 0


def main_for(variant: str):
    def _main(argv=None) -> int:
        return run_variant(variant, argv)

    return _main


if __name__ == "__main__":
    sys.exit(run_variant(sys.argv[1], sys.argv[2:]))
