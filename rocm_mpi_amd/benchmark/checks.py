"""Correctness checks of a bench.py run, all bounded and agreed by every rank:
the halo check (a small grid through the real halo path, bitwise against a
1-rank run), the fast-math drift bound, the headline window check (row windows
of the timed field, bitwise against the CPU twin) and the full-field check
(every cell of the timed field: finite and inside the initial field's bounds,
the explicit scheme's maximum principle)."""
from __future__ import annotations

import hashlib
import os
import time

from ..config import diag_flag, diag_value
from .common import CheckFailed, agree, bounded_gather_tiles, bounded_status

# fast-math drift bound (max |fast - canonical| after the run's steps on a
# random field in [0, 1)): diffusion is contractive, rounding differences do
# not accumulate (3.3e-16 after 24..5000 steps, CPU twins, 514^2)
DRIFT_BOUND = 1e-14


def _run_grid(nx, ny, dims_, K, steps_fast, steps_can, periodic, loopback=None, device=None,
              via=False):
    """A small grid through the production path: steps_fast fast-math steps,
    then steps_can canonical steps. Returns (field, coords, nxyz_g, transport, plan)."""
    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg

    ol = 2 * K
    per = 1 if periodic else 0
    kw = dict(dimx=dims_[0], dimy=dims_[1], overlaps=(ol, ol, 2), halowidths=(K, K, 1),
              quiet=True, periodx=per, periody=per)
    if loopback is not None:
        kw.update(loopback=loopback, device=device)
    elif via:
        kw.update(transport="rccl", self_via_transport=True)
    gg.init_global_grid(nx, ny, 1, **kw)
    try:
        m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=nx, ny=ny,
                                        nt=max(1, steps_fast + steps_can), init="random",
                                        quiet=True, dims=(*dims_, 0), temporal=K,
                                        periods=(per, per, 0), fast_math=True, device=device))
        plan = m.plan(steps_fast)
        m.step(steps_fast)
        if steps_can:
            m.set_temporal(K, fast_math=False)
            m.step(steps_can)
        m.synchronize()
        out = (m.field.clone(), m.g.coords, m.g.nxyz_g, m.g.transport, plan)
        m.close()
    finally:
        gg.finalize_global_grid(finalize_dist=False)
    return out


def _local_device(dev: str) -> str:
    import torch

    return dev if dev == "cpu" else f"cuda:{torch.cuda.current_device()}"


def _restore_stream(dev: str):
    """The loopback grid installs its own stream: put the caller's back."""
    import torch

    prev = torch.cuda.current_stream() if dev != "cpu" else None

    class _R:
        def __enter__(self):
            return self

        def __exit__(self, *exc):
            if prev is not None:
                torch.cuda.set_stream(prev)
            return False

    return _R()


def halo_check(n: int, dims, K: int, dev: str, world: int, rank: int, timeout_s: float,
               self_rccl: bool = False, inject: bool = True) -> dict:
    """Run a small grid with the bench's process grid through the real halo
    path (37 fast-math steps, then 23 canonical), gather every rank's tile on
    rank 0 and compare bitwise with a 1-rank run of the global grid on rank
    0's device. Raises CheckFailed on every rank on any error or mismatch.

    self_rccl (one rank): the check grid is periodic and its halos go through
    RCCL send/recv to itself; the reference is the same periodic tile with
    local self copies (exercises this path with real RCCL traffic on 1 GPU)."""
    import numpy as np

    from rocm_mpi_amd.parallel import comm as C

    n_fast, n_can = 37, 23
    ol = 2 * K
    t0 = time.perf_counter()
    err = ""
    field = coords = None
    info = {"local_tile": [n, n], "steps": [n_fast, n_can], "self_rccl": self_rccl}
    try:
        fault = diag_value("bench_check_raise") if inject and rank == world - 1 else ""
        if fault == "before":  # peers then block in the exchange: the watchdog path
            raise RuntimeError("injected halo-check failure before the run")
        field, coords, nxyz_g, transport, plan = _run_grid(n, n, dims, K, n_fast, n_can,
                                                           self_rccl, via=self_rccl)
        if fault == "after":
            raise RuntimeError("injected halo-check failure after the run")
        info.update(global_grid=list(nxyz_g[:2]), transport=transport, fast_math_plan=plan)
        if inject and diag_flag("bench_check_corrupt") and rank == world - 1:
            field[n // 2, n // 2] += 1e-12  # negative test (tests/test_multiprocess_cpu.py)
    except Exception as e:  # noqa: BLE001 - reported to every rank below
        err = f"{type(e).__name__}: {e}"
    agree(not err, err, world, timeout_s, "halo check run")
    import torch

    cxy = torch.tensor([coords[0], coords[1]], dtype=torch.float64)
    all_xy = bounded_gather_tiles(cxy, world, timeout_s)
    tiles = bounded_gather_tiles(field, world, timeout_s)
    bad, err = 0, ""
    if rank == 0:
        try:
            with _restore_stream(dev):
                rn = (n, n) if self_rccl else tuple(info["global_grid"])
                ref = _run_grid(*rn, (1, 1), K, n_fast, n_can, self_rccl,
                                loopback=(C.LoopbackHub(1), 0), device=_local_device(dev))[0]
            ref = ref.cpu().numpy()
            for xy, T in zip(all_xy, tiles):
                gx0, gy0 = int(xy[0]) * (n - ol), int(xy[1]) * (n - ol)
                if not np.array_equal(T.numpy(), ref[gy0:gy0 + n, gx0:gx0 + n]):
                    bad += 1
        except Exception as e:  # noqa: BLE001
            err = f"reference run: {type(e).__name__}: {e}"
    st = bounded_status(not err and bad == 0, err or f"{bad} tile(s) differ", world, timeout_s)
    info["tiles_mismatched"] = bad if rank == 0 else None
    info["seconds"] = round(time.perf_counter() - t0, 3)
    if not st[0][0]:
        info["tiles_mismatched"] = bad if rank == 0 else -1
        raise CheckFailed(f"halo check: {st[0][1]}", info)
    return info


def drift_check(n: int, K: int, steps: int, dev: str, world: int, timeout_s: float) -> dict:
    """max |fast - canonical| on an n x n random tile after `steps` steps
    (every rank on its own GPU, 1-rank grid); the fast fields must agree
    bitwise across ranks (same kernels, same data) and stay within DRIFT_BOUND."""
    from rocm_mpi_amd.parallel import comm as C

    t0 = time.perf_counter()
    err, drift, digest = "", None, ""
    try:
        with _restore_stream(dev):
            kw = dict(loopback=(C.LoopbackHub(1), 0), device=_local_device(dev))
            fast = _run_grid(n, n, (1, 1), K, steps, 0, False, **kw)
            can = _run_grid(n, n, (1, 1), K, 0, steps, False, **kw)
        drift = float((fast[0] - can[0]).abs().max())
        digest = hashlib.sha1(fast[0].cpu().numpy().tobytes()).hexdigest()[:16]
        if not drift <= DRIFT_BOUND:
            err = f"fast-math drift {drift:.3e} > bound {DRIFT_BOUND:.0e}"
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    st = bounded_status(not err, err or f"{digest} {drift!r}", world, timeout_s)
    bad = [f"{r}: {m}" for r, (o, m) in enumerate(st) if not o]
    if not bad and len({m.split()[0] for _, m in st}) != 1:
        bad = ["fast-math fields differ across GPUs: " + ", ".join(m for _, m in st)]
    info = {"tile": [n, n], "steps": steps, "fast_math_drift_max": drift, "bound": DRIFT_BOUND,
            "fast_field_sha1_16": digest, "seconds": round(time.perf_counter() - t0, 3)}
    if bad:
        raise CheckFailed("fast-math drift check: " + "; ".join(bad), info)
    return info


WINDOW_ROWS = 8
WINDOW_BUDGET = 3.0e9  # cell updates of the CPU twin for all windows of a rank


def snapshot_windows(model, h: int = WINDOW_ROWS) -> dict:
    """Three full-width row windows of this rank's field (top edge, middle,
    bottom edge), copied to the host right after the timed run, with what the
    CPU twin needs to recompute them from the initial condition."""
    import torch

    cfg, g = model.cfg, model.g
    ny, nx = model.field.shape
    h = min(h, ny)
    rows = sorted({0, max(0, ny // 2 - h // 2), ny - h})
    geo = model.geometry()
    tiles = [model.field[r:r + h].detach().cpu().clone() for r in rows]
    if diag_flag("bench_window_corrupt") and g.me == g.nprocs - 1:
        tiles[-1][h // 2, nx // 2] += 1e-12  # negative test (tests/test_multiprocess_cpu.py)
    return {"rows": rows, "h": h, "tiles": tiles,
            "nx": nx, "ny": ny, "geom": geo, "coef": model.coef, "seed": cfg.seed,
            "icp": 1.0 / cfg.Cp0, "fast": bool(cfg.fast_math), "steps": model.steps_done,
            "dtype": torch.float64}


def window_check(snap: dict, world: int, timeout_s: float, budget: float = WINDOW_BUDGET) -> dict:
    """the headline field itself, not a small proxy tile.
    Each window is recomputed on the CPU twin (the C++ fast5 / canonical
    arithmetic, bitwise equal to the GPU kernels) from the counter-based
    initial condition of the global grid (csrc/kernels/misc.hip init_random),
    over the window plus `steps` rows / columns of margin on every side that
    is not a global boundary (the dependency cone of `steps` updates), and
    compared bitwise. Full-width windows when the twin's cost fits `budget`
    cell updates, else three 64-column boxes per window (left edge, centre,
    right edge). Raises CheckFailed on every rank on any mismatch."""
    import torch

    from rocm_mpi_amd import ops

    t0 = time.perf_counter()
    S, h, nx, ny = snap["steps"], snap["h"], snap["nx"], snap["ny"]
    geo = snap["geom"]
    nxg, nyg = geo.nxg, geo.nyg
    per = geo.periodx or geo.periody
    full = (nx + 2 * S) * (h + 2 * S) * S * len(snap["rows"]) <= budget
    bw = nx if full else min(64, nx)
    cols = [0] if full else sorted({0, max(0, nx // 2 - bw // 2), nx - bw})
    tn = ops.StencilTuning(kernel="pipe" if snap["fast"] else "pipec")
    err, boxes, mism = "", 0, 0
    try:
        if per:
            raise CheckFailed("window check: periodic grids are not covered")
        for r0, tile in zip(snap["rows"], snap["tiles"]):
            for c0 in cols:
                # the box in global coordinates, with the margin, clipped to the grid
                gy_lo, gy_hi = geo.gy0 + r0, geo.gy0 + r0 + h
                gx_lo, gx_hi = geo.gx0 + c0, geo.gx0 + c0 + bw
                wy0, wy1 = max(0, gy_lo - S), min(nyg, gy_hi + S)
                wx0, wx1 = max(0, gx_lo - S), min(nxg, gx_hi + S)
                wg = ops.TileGeometry(gx0=wx0, gy0=wy0, nxg=nxg, nyg=nyg, dx=geo.dx, dy=geo.dy)
                a = torch.empty((wy1 - wy0, wx1 - wx0), dtype=snap["dtype"])
                ops.init_random_(a, wg, seed=snap["seed"])
                icp = torch.full_like(a, snap["icp"])
                b = a.clone()
                done = 0
                while done < S:
                    k = min(24, S - done)
                    if a.shape[0] >= 3 and a.shape[1] >= 3:
                        ops.stencilk_step(k, b, a, icp, snap["coef"], None, tn)
                    a, b = b, a
                    done += k
                want = a[gy_lo - wy0:gy_hi - wy0, gx_lo - wx0:gx_hi - wx0]
                got = tile[:, c0:c0 + bw]
                boxes += 1
                if not torch.equal(got, want):
                    mism += 1
                    d = (got - want).abs().max().item()
                    err = (f"window rows {r0}..{r0 + h} cols {c0}..{c0 + bw}: "
                           f"{int((got != want).sum())} cells differ (max |diff| {d:.3e})")
    except CheckFailed as e:
        err = str(e.args[0])
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {e}"
    info = {"windows": len(snap["rows"]), "rows_each": h, "row_starts": snap["rows"],
            "full_width": bool(full), "box_cols": None if full else bw, "boxes": boxes,
            "steps": S, "bitwise": not err and mism == 0,
            "arithmetic": "fast-math twin" if snap["fast"] else "canonical twin",
            "seconds": round(time.perf_counter() - t0, 3)}
    st = bounded_status(not err, err, world, timeout_s)
    bad = [f"{r}: {m}" for r, (o, m) in enumerate(st) if not o]
    if bad:
        info["bitwise"] = False
        raise CheckFailed("headline window check: " + "; ".join(bad), info)
    return info


# --- full-field check ----------------------------------
ULP1 = 2.0 ** -52  # one ulp of 1.0


def field_stats_global(field, comm) -> tuple[float, float, float]:
    """(non-finite cells, min, max of the finite cells) over every rank's whole
    local tile (halo and overlap included): one native device pass per rank
    (ops.field_stats, ~13 ms for an 82 GB tile), then three scalar all-reduces."""
    from rocm_mpi_amd import ops

    bad, lo, hi = ops.field_stats(field)
    return comm.allreduce(bad, "sum"), comm.allreduce(lo, "min"), comm.allreduce(hi, "max")


def full_field_check(field, init: tuple, steps: int, comm, world: int, rank: int,
                     timeout_s: float) -> dict:
    """Every cell of the timed field: finite, and within the initial field's
    [min, max] (the explicit scheme's maximum principle: with dt =
    min(dx^2, dy^2)/4.1 (scripts/diffusion_2D_perf.jl:30) and Cp = 1 each
    update is a convex combination of the cell and its 4 neighbours, weights
    1 - 2(gx + gy) >= 0.02 and gx, gy, so no value leaves the initial range;
    Dirichlet boundary cells keep their initial values and halo copies move
    values). The fp64 rounding of an update is below 8 ulps of the range's
    magnitude per step, hence the tolerance. RMA_DIAG bench_field_corrupt=nan |
    hot | cold injects one bad cell on the last rank first (negative test).
    Raises CheckFailed on every rank on a violation."""
    t0 = time.perf_counter()
    corrupt = diag_value("bench_field_corrupt")
    if corrupt and rank == world - 1:
        ny, nx = field.shape
        v = {"nan": float("nan"), "hot": init[2] + 0.5 * (abs(init[2]) + 1.0),
             "cold": init[1] - 0.5 * (abs(init[1]) + 1.0)}[corrupt]
        field[ny // 2, nx // 2] = v
    err = ""
    bad = lo = hi = None
    try:
        bad, lo, hi = field_stats_global(field, comm)
    except Exception as e:  # noqa: BLE001 - reported to every rank below
        err = f"{type(e).__name__}: {e}"
    lo0, hi0 = init[1], init[2]
    scale = max(abs(lo0), abs(hi0), 1e-300)
    tol = 8.0 * ULP1 * scale * (steps + 1)
    if not err:
        if bad:
            err = f"{int(bad)} non-finite cell(s) in the timed field"
        elif lo < lo0 - tol or hi > hi0 + tol:
            err = (f"maximum principle violated: field range [{lo!r}, {hi!r}] outside the "
                   f"initial [{lo0!r}, {hi0!r}] (tolerance {tol:.3e})")
    info = {"cells": int(field.numel()) * world,  # equal tiles on every rank
            "nonfinite": None if bad is None else int(bad), "min": lo, "max": hi,
            "init_min": lo0, "init_max": hi0, "init_nonfinite": int(init[0]),
            "tolerance": tol, "steps": steps, "ok": not err,
            "injected": corrupt or None, "seconds": round(time.perf_counter() - t0, 4)}
    st = bounded_status(not err, err, world, timeout_s)
    fails = [f"{r}: {m}" for r, (o, m) in enumerate(st) if not o]
    if fails:
        info["ok"] = False
        info["error"] = "; ".join(fails)
        raise CheckFailed("full-field check: " + "; ".join(fails), info)
    return info
