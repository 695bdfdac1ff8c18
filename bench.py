#!/usr/bin/env python
"""Headline benchmark: T_eff (GB/s) of 2D diffusion on 1..8 MI355X, weak scaling.

BASELINE.json metric: "T_eff (GB/s) + weak-scaling eff., 2D diffusion 1000 steps
at 1/2/4/8 MI355X"; flagship config "diffusion_2D_perf_hide ... per-GPU tile
sized to 288 GB HBM". One process per GPU (torch.distributed.run), halo
exchange GPU-direct over RCCL/xGMI overlapped with the interior kernel.

    python bench.py                                   # 1 GPU, 1000 steps, 10 warmup
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \\
        --master-addr 127.0.0.1 --master-port 29600 bench.py --gpus 8

T_eff per GPU follows the reference exactly (scripts/diffusion_2D_perf.jl:55-58):
A_eff = 3*nx*ny*8 B per step on the LOCAL tile (halo included), divided by the
time per step. W warmup steps run untimed (the reference skips 10); K steps
are timed between barrier+device-sync pairs; the step time is the MAX over
ranks; ``value`` is the whole-job aggregate = N x per-GPU T_eff (weak scaling:
the local tile is the same for every N). Data: synthetic random-init field.

The run validates itself and says which rank is slow (VERDICT r1 item 1, r2
items 1-3):
* preflight, before the HBM-sized tile is allocated: the GPU-direct ring
  send/recv of the reference's smoke test (scripts/rocmaware_test_selectdevice.jl:
  16-23) over the halo transport (RCCL; RCCL to self on one GPU) and a tiny
  halo check through the same path; a failure exits non-zero on every rank;
* RCCL is mandatory at N > 1 (no fallback to the host-staged transport) and
  every rank must drive a different physical GPU (PCI bus ids compared);
* ``config.ranks_detail``: per rank its coordinates, neighbours, PCI bus id,
  its OWN step time (taken before the closing barrier, so a slow GPU shows as
  the one slow entry), its solo re-time with the exchange disabled, and its
  per-pass HIP-event split (frame / halo / interior / exposed halo);
* after the timed run: the fast-math drift bound of this run's length
  (``fast_math_drift_max``: max |fast - canonical| on a small tile after
  warmup + steps steps, every rank, must agree bitwise across GPUs), and the
  halo check (a small grid with the bench's process grid through the real
  halo path, gathered and compared bitwise with a 1-rank run; on one GPU the
  grid is periodic and every halo goes through RCCL send/recv to itself).
  Any error or mismatch on any rank makes EVERY rank exit non-zero and rank 0
  still prints the record with the error; all check-phase collectives are
  bounded (``--check-timeout``) and a watchdog ends a rank stuck in the GPU
  runtime.
"""
from __future__ import annotations

import os

# dmabuf IPC (the host driver supports no legacy IPC); before torch / HIP load
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import argparse  # noqa: E402
import datetime  # noqa: E402
import hashlib  # noqa: E402
import json  # noqa: E402
import math  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402
import threading  # noqa: E402
import time  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "T_eff (GB/s) + weak-scaling eff., 2D diffusion 1000 steps at 1/2/4/8 MI355X"
# fast-math drift bound (max |fast - canonical| after the run's steps on a
# random field in [0, 1)): diffusion is contractive, rounding differences do
# not accumulate (3.3e-16 after 24..5000 steps, CPU twins, 514^2)
DRIFT_BOUND = 1e-14


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--variant", default="perf_hide", choices=["perf_hide", "perf", "kp"])
    ap.add_argument("--nx", type=int, default=0, help="local tile x size (0 = auto-size to HBM)")
    ap.add_argument("--ny", type=int, default=0, help="local tile y size (0 = --nx)")
    ap.add_argument("--hbm-frac", type=float, default=0.80,
                    help="fraction of free HBM for T, T2, 1/Cp when auto-sizing")
    ap.add_argument("--max-tile", type=int, default=0, help="cap auto-sized edge (0 = none)")
    ap.add_argument("--dims", default="0,0", help="process grid dimx,dimy (0 = auto)")
    ap.add_argument("--b-width", default="1,1")
    ap.add_argument("--chunk-rows", type=int, default=4)
    ap.add_argument("--kernel", default="march", choices=["march", "lds"])
    ap.add_argument("--unroll", type=int, default=4)
    ap.add_argument("--nontemporal", type=int, default=3,
                    help="bitmask: 1 = NT T2 stores, 2 = NT 1/Cp loads, 4 = NT T loads")
    ap.add_argument("--vec", type=int, default=2, choices=[2, 4], help="cells per lane")
    ap.add_argument("--graph", action="store_true", help="replay steps from a hipGraph")
    ap.add_argument("--temporal", type=int, default=24,
                    help="K: at most K time steps per kernel pass (1..24); the executor's "
                         "planner splits the steps into passes of <= K (e.g. 20 -> one "
                         "20-step pass, 1000 -> 24-step passes); halo width K, overlap 2K")
    ap.add_argument("--chunk2", type=int, default=0,
                    help="K-step kernel rows per task (0: per pass depth, executor default)")
    ap.add_argument("--unroll2", type=int, default=2, choices=[2, 4])
    ap.add_argument("--fast-math", dest="fast_math", action="store_true", default=True,
                    help="passes with the fast-math fp64 arithmetic (5-point sum, one folded "
                         "per-cell factor, FMAs): same scheme, not bitwise equal to the "
                         "canonical update but bitwise equal to its CPU twin (default; the "
                         "canonical K-step and one-step kernels are timed too)")
    ap.add_argument("--no-fast-math", dest="fast_math", action="store_false")
    ap.add_argument("--overlap", type=int, default=0,
                    help="grid overlap (0: 2 x steps-per-pass, the minimum)")
    ap.add_argument("--single-step-steps", type=int, default=100,
                    help="after the timed run, also time this many steps of the one-step "
                         "kernel on the same tile (reported in config; 0 = skip)")
    ap.add_argument("--canonical-steps", type=int, default=0,
                    help="steps of the canonical (bitwise) K-step passes timed on the same tile "
                         "(0: 2 x the canonical depth)")
    ap.add_argument("--solo-steps", type=int, default=-1,
                    help="steps re-timed with the exchange disabled for the same-run weak-scaling "
                         "efficiency (-1: = --steps; 0: skip)")
    ap.add_argument("--preflight", type=int, default=1,
                    help="ring send/recv + tiny halo check before the tile is allocated (1/0)")
    ap.add_argument("--check", type=int, default=-1,
                    help="halo bitwise check after the run (1 on, 0 off, -1: on with a GPU "
                         "or N > 1)")
    ap.add_argument("--check-nx", type=int, default=0,
                    help="local tile of the halo check (0: 2050 on GPU, 130 on CPU)")
    ap.add_argument("--check-self-rccl", type=int, nargs="?", const=1, default=-1,
                    help="one rank: run the halo check periodic with RCCL send/recv to self "
                         "(-1: on with a GPU)")
    ap.add_argument("--check-timeout", type=float, default=300.0,
                    help="seconds any check-phase collective (and the whole check phase, x3) "
                         "may take before the run fails")
    ap.add_argument("--window-check", type=int, default=1,
                    help="after the timed run, compare three full-width row windows of the "
                         "timed field bitwise with the CPU twin (1/0)")
    ap.add_argument("--drift-steps", type=int, default=-1,
                    help="steps of the fast-math drift measurement (-1: warmup + steps; 0: off)")
    ap.add_argument("--shared-gpu-test", action="store_true",
                    help="functional test of the multi-process path on ONE GPU: ranks share "
                         "the card over the host-staged transport; the record says so and is "
                         "never a scaling point")
    ap.add_argument("--shared-gpu-transport", default="staged", choices=["staged", "ipc", "rccl"],
                    help="halo transport of --shared-gpu-test: host-staged gloo, HIP IPC "
                         "device-to-device copies between the processes, or RCCL with one "
                         "fake host per rank (RMA_RCCL_SHARED_GPU: its socket transport)")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: the same driver on the C++ CPU twins over gloo (tests of the "
                         "multi-rank bench path; needs --nx; not a benchmark)")
    return ap.parse_args(argv)


def auto_tile(frac: float, cap: int) -> int:
    import torch

    free, _total = torch.cuda.mem_get_info()
    cells = frac * free / 24.0  # T, T2, 1/Cp in fp64
    n = int(math.isqrt(int(cells))) // 256 * 256
    if cap:
        n = min(n, cap)
    return max(n, 512)


def log(rank: int, msg: str) -> None:
    print(f"bench.py rank {rank}: {msg}", file=sys.stderr, flush=True)


class CheckFailed(RuntimeError):
    """A correctness check failed (on this or another rank)."""


# ---------------------------------------------------------------------------
# bounded collectives over the gloo group (metadata only)
# ---------------------------------------------------------------------------
def gather_obj(obj, world: int):
    """All-gather a small picklable object over the gloo group (main phase:
    every rank reaches it; torchrun ends the job if one rank dies)."""
    if world == 1:
        return [obj]
    import torch.distributed as dist

    from rocm_mpi_amd.parallel import comm as C

    out: list = [None] * world
    dist.all_gather_object(out, obj, group=C._gloo_group())
    return out


def _wait(work, timeout_s: float, what: str) -> None:
    try:
        work.wait(timeout=datetime.timedelta(seconds=timeout_s))
    except Exception as e:  # noqa: BLE001 - a peer is gone or stuck
        raise CheckFailed(f"{what}: no answer from every rank within {timeout_s:.0f} s ({e})") \
            from None


def bounded_status(ok: bool, msg: str, world: int, timeout_s: float) -> list:
    """All-gather (ok, message) from every rank, bounded: every rank learns
    whether any rank failed and why, and nobody blocks longer than timeout_s."""
    if world == 1:
        return [(ok, msg)]
    import torch
    import torch.distributed as dist

    from rocm_mpi_amd.parallel import comm as C

    raw = msg.encode("utf-8", "replace")[:480]
    buf = torch.zeros(512, dtype=torch.uint8)
    buf[0] = 1 if ok else 0
    buf[1] = len(raw) >> 8
    buf[2] = len(raw) & 0xFF
    if raw:
        buf[3:3 + len(raw)] = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    out = [torch.empty_like(buf) for _ in range(world)]
    _wait(dist.all_gather(out, buf, group=C._gloo_group(), async_op=True), timeout_s,
          "status exchange")
    res = []
    for b in out:
        n = (int(b[1]) << 8) | int(b[2])
        res.append((bool(b[0]), bytes(b[3:3 + n].tolist()).decode("utf-8", "replace")))
    return res


def agree(ok: bool, msg: str, world: int, timeout_s: float, what: str) -> None:
    """Raise CheckFailed on EVERY rank if any rank failed (bounded)."""
    st = bounded_status(ok, msg, world, timeout_s)
    bad = [(r, m) for r, (o, m) in enumerate(st) if not o]
    if bad:
        raise CheckFailed(f"{what} failed on rank(s) " +
                          "; ".join(f"{r}: {m}" for r, m in bad))


def bounded_gather_tiles(field, world: int, timeout_s: float):
    """The equal-shape tiles of every rank on rank 0 (host copies), bounded."""
    host = field.detach().cpu().contiguous()
    if world == 1:
        return [host]
    import torch
    import torch.distributed as dist

    from rocm_mpi_amd.parallel import comm as C

    lst = [torch.empty_like(host) for _ in range(world)] if dist.get_rank() == 0 else None
    _wait(dist.gather(host, lst, dst=0, group=C._gloo_group(), async_op=True), timeout_s,
          "tile gather")
    return lst


_DONE_KEY = "rma/bench/rank0_reported"


def signal_reported(world: int) -> None:
    """Rank 0 has printed its record (or is about to exit without one)."""
    if world > 1:
        try:
            import torch.distributed as dist

            dist.distributed_c10d._get_default_store().set(_DONE_KEY, "1")
        except Exception:  # noqa: BLE001 - best effort on an error path
            pass


def wait_reported(world: int, timeout_s: float) -> None:
    """A failing rank > 0 waits (bounded) for rank 0's record before it exits:
    torchrun ends the whole job as soon as one rank exits non-zero."""
    if world > 1:
        try:
            import torch.distributed as dist

            dist.distributed_c10d._get_default_store().wait(
                [_DONE_KEY], datetime.timedelta(seconds=timeout_s))
        except Exception:  # noqa: BLE001
            pass


class Watchdog:
    """Ends this rank if a phase outlives its deadline (a rank stuck inside
    the GPU runtime, RCCL or a gloo receive cannot be interrupted from
    Python): rank 0 first prints the record it has, with the failure, so the
    run still reports; the other ranks give it time to do so."""

    def __init__(self, rank: int, world: int, seconds: float, what: str, on_fire=None):
        self.rank, self.world, self.what, self.on_fire = rank, world, what, on_fire
        self._t = threading.Timer(seconds, self._fire)
        self._t.daemon = True
        self._t.start()

    def _fire(self) -> None:
        msg = f"watchdog: {self.what} did not finish in time"
        log(self.rank, msg + "; exiting")
        try:
            if self.rank == 0 and self.on_fire is not None:
                self.on_fire(msg)
        finally:
            finish_failed(self.rank, self.world, 6, 30.0)

    def cancel(self) -> None:
        self._t.cancel()


def finish_failed(rank: int, world: int, rc: int, wait_s: float) -> None:
    """Exit a failed run on this rank without touching the (possibly broken)
    process groups: rank 0 after its record, the others after rank 0's."""
    if rank == 0:
        signal_reported(world)
    else:
        wait_reported(world, wait_s)
    hard_exit(rank, rc)


def hard_exit(rank: int, rc: int) -> None:
    record_rc(rank, rc)
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(rc)


def record_rc(rank: int, rc: int) -> None:
    """RMA_BENCH_RC_DIR: every rank writes its exit status (tests)."""
    d = os.environ.get("RMA_BENCH_RC_DIR")
    if d:  # atomically: torchrun may end this rank right after (a half-written file)
        # one temp file per thread: the check-phase watchdog thread and the main
        # thread can both be exiting the rank at once; with one shared temp
        # name one thread renamed the other's still-empty file into place
        tmp = os.path.join(d, f".rc{rank}.{threading.get_ident()}.tmp")
        with open(tmp, "w") as f:
            f.write(str(rc))
            f.flush()
        os.replace(tmp, os.path.join(d, f"rc{rank}"))


# ---------------------------------------------------------------------------
# checks
# ---------------------------------------------------------------------------
def summarize_timings(ts: list, exchange: bool = True) -> dict:
    """Mean per-pass frame / halo / interior / exposed-halo ms of one rank.
    Without a neighbour (exchange=False) the halo events bracket an empty
    exchange: the halo keys are event-gap noise and the overlap fraction is
    not defined (None)."""
    if not ts:
        return {}
    n = len(ts)
    mean = {k: sum(t[k] for t in ts) / n for k in ("frame_ms", "halo_ms", "interior_ms",
                                                   "pass_ms", "exposed_halo_ms")}
    halo = sum(t["halo_ms"] for t in ts)
    exposed = sum(t["exposed_halo_ms"] for t in ts)
    mean["passes"] = n
    mean["depths"] = sorted({int(t["K"]) for t in ts}, reverse=True)
    mean["overlap_fraction"] = (1.0 - exposed / halo) if halo > 0 and exchange else None
    if not exchange:
        mean["note"] = "no neighbour: no halo exchange ran; halo_ms / exposed_halo_ms are event gaps"
    return mean


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
        fault = os.environ.get("RMA_BENCH_CHECK_RAISE", "") if inject and rank == world - 1 else ""
        if fault == "before":  # peers then block in the exchange: the watchdog path
            raise RuntimeError("injected halo-check failure before the run")
        field, coords, nxyz_g, transport, plan = _run_grid(n, n, dims, K, n_fast, n_can,
                                                           self_rccl, via=self_rccl)
        if fault == "after":
            raise RuntimeError("injected halo-check failure after the run")
        info.update(global_grid=list(nxyz_g[:2]), transport=transport, fast_math_plan=plan)
        if inject and os.environ.get("RMA_BENCH_CHECK_CORRUPT") == "1" and rank == world - 1:
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
    if os.environ.get("RMA_BENCH_WINDOW_CORRUPT") == "1" and g.me == g.nprocs - 1:
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


# weak-scaling attribution. Self-contained in
# one job: E_in_run = t_fast_iso / t_it = e_gpu * e_coef * e_halo, with
# t_fast_iso the fastest rank's own isotropic solo time (no exchange). The
# N = 1 record of the same tile class (cached by the same driver sweep on the
# same node and build) adds e_box = t(N=1) / t_fast_iso, so that
# E(N) = t(N=1) / t_it = e_box * E_in_run.
def _n1_cache_path() -> str:
    import tempfile

    return os.environ.get("RMA_BENCH_N1_CACHE",
                          os.path.join(tempfile.gettempdir(), "rma_bench_n1_record.json"))


def _build_id() -> str:
    """Hash of the native sources, flags and arch (rocm_mpi_amd/_build.py)."""
    try:
        from rocm_mpi_amd import _build

        return _build.source_stamp()[:12]
    except Exception:  # noqa: BLE001 - informational
        return "unknown"


def _n1_key(nx: int, ny: int, steps: int, warmup: int, K: int, fast: bool, variant: str) -> str:
    """Tile class + build + node: a record from another build or another box
    (another sweep) never matches."""
    import socket

    return (f"{variant}:{nx}x{ny}:s{steps}:w{warmup}:K{K}:f{int(fast)}:b{_build_id()}:"
            f"h{socket.gethostname()}")


def save_n1(key: str, ms_per_step: float, bus: str) -> None:
    try:
        tmp = _n1_cache_path() + f".{os.getpid()}.tmp"
        with open(tmp, "w") as f:
            json.dump({"key": key, "ms_per_step": ms_per_step, "pci_bus_id": bus,
                       "time": time.time()}, f)
        os.replace(tmp, _n1_cache_path())
    except OSError:
        pass


def load_n1(key: str):
    try:
        with open(_n1_cache_path()) as f:
            d = json.load(f)
        return d if d.get("key") == key else None
    except (OSError, ValueError):
        return None


def attribution(t_it: float, solo: float | None, solo_iso: float | None,
                fast_iso: float | None, n1_ms: float | None,
                slow_iso: float | None = None) -> dict:
    """Job-level split of the weak-scaling efficiency (times in s, max over
    ranks unless named otherwise):
      e_halo = solo / t_it        exchange + frame cost, same coefficients
      e_coef = solo_iso / solo    fast-math pass energy at this grid's dx != dy
                                  against dx = dy
      e_gpu  = fast_iso / slow_iso  the slowest GPU against the fastest GPU of
                                  THIS job (each rank's own isotropic solo
                                  time, no exchange): in-run, 1 for one GPU
      e_product = e_halo * e_coef * e_gpu ~ fast_iso / t_it  (in-run E(N);
                                  exact up to the barrier time in solo_iso)
      e_box  = t(N=1) / fast_iso  this job's fastest GPU against the N = 1
                                  record of the same sweep (null without it)
      e_product_vs_n1 = e_box * e_product = t(N=1) / t_it = E(N)."""
    out = {"e_halo": None, "e_coef": None, "e_gpu": None, "e_product": None,
           "e_box": None, "e_product_vs_n1": None,
           "weak_scaling_eff_same_run_iso": None, "fastest_solo_iso_ms_per_step":
               fast_iso * 1e3 if fast_iso else None, "n1_ms_per_step": n1_ms}
    if solo:
        out["e_halo"] = solo / t_it
    if solo and solo_iso:
        out["e_coef"] = solo_iso / solo
        out["weak_scaling_eff_same_run_iso"] = solo_iso / t_it
    if fast_iso and (slow_iso or solo_iso):
        out["e_gpu"] = fast_iso / (slow_iso or solo_iso)
    if all(out[k] is not None for k in ("e_halo", "e_coef", "e_gpu")):
        out["e_product"] = out["e_halo"] * out["e_coef"] * out["e_gpu"]
    if fast_iso and n1_ms:
        out["e_box"] = (n1_ms / 1e3) / fast_iso
        if out["e_product"] is not None:
            out["e_product_vs_n1"] = out["e_box"] * out["e_product"]
    return {k: (round(v, 6) if isinstance(v, float) else v) for k, v in out.items()}


def preflight(dims, K: int, dev: str, world: int, rank: int, gpu: bool, n: int,
              timeout_s: float) -> dict:
    """Before the HBM-sized tile: the ring send/recv of the reference's smoke
    test over the halo transport, then the halo check on a tiny grid."""
    from rocm_mpi_amd.apps import rocmaware_test_selectdevice as smoke

    t0 = time.perf_counter()
    err = ""
    transport = "rccl" if gpu and world == 1 else "auto"
    ring: dict = {}
    try:
        vals = smoke.run(4, transport=transport, verbose=False, self_ring=world == 1, info=ring)
        if any(v != float((rank - 1) % world) for v in vals):
            err = f"ring received {vals}, expected {(rank - 1) % world}"
    except Exception as e:  # noqa: BLE001
        err = f"ring send/recv: {type(e).__name__}: {e}"
    agree(not err, err, world, timeout_s, "preflight ring")
    info = {"ring_ok": True, "ring_ranks": world, "ring_transport": ring.get("transport"),
            "rccl_nranks": ring.get("rccl_nranks")}
    info["halo"] = halo_check(n, dims, K, dev, world, rank, timeout_s,
                              self_rccl=gpu and world == 1, inject=False)
    info["seconds"] = round(time.perf_counter() - t0, 3)
    return info


def _rccl_info() -> dict | None:
    """Which RCCL carries the halo traffic (RMA_RCCL_LIB may swap it)."""
    try:
        from rocm_mpi_amd._native import native

        return {"library": native().rccl_library(), "version": native().rccl_version()}
    except Exception:  # noqa: BLE001 - informational
        return None


def _rccl_nranks(g, pre: dict | None):
    """ncclCommCount of the halo communicator (or of the preflight ring's RCCL
    communicator on the single-GPU RCCL-self path); None without RCCL."""
    try:
        from rocm_mpi_amd.parallel.comm import RcclComm

        if isinstance(g.comm, RcclComm) and g.comm.native is not None:
            return int(g.comm.native.count())
    except Exception:  # noqa: BLE001 - informational
        return None
    return (pre or {}).get("rccl_nranks")


def make_config(a, nx: int, ny: int, dev: str, dims: tuple):
    """The DiffusionConfig of the timed run (the reference-named entry points
    resolve the same one for the BASELINE presets: apps/cli.py auto_temporal,
    tests/test_apps_cpu.py)."""
    from rocm_mpi_amd.models import DiffusionConfig

    K = a.temporal if a.variant != "kp" else 1
    bw = tuple(int(v) for v in a.b_width.split(","))
    return DiffusionConfig(variant=a.variant, nx=nx, ny=ny, nt=a.steps + a.warmup, device=dev,
                           warmup=a.warmup, init="random", b_width=bw, dims=dims,
                           chunk_rows=a.chunk_rows, kernel=a.kernel, nontemporal=a.nontemporal,
                           unroll=a.unroll, vec=a.vec, temporal=K, chunk2=a.chunk2,
                           unroll2=a.unroll2, use_graph=a.graph, quiet=True,
                           fast_math=a.fast_math and a.variant != "kp")


# ---------------------------------------------------------------------------
def main(argv=None) -> int:
    a = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and world == 1:
        # not launched by torchrun: launch ourselves, one rank per GPU
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1", "--master-port",
               os.environ.get("MASTER_PORT", "29613"), os.path.abspath(__file__),
               *(argv if argv is not None else sys.argv[1:])]
        return subprocess.call(cmd)
    rank = int(os.environ.get("RANK", "0"))
    rc = run(a, world, rank)
    record_rc(rank, rc)
    return rc


def run(a, world: int, rank: int) -> int:
    if world != a.gpus:
        log(rank, f"WORLD_SIZE={world} but --gpus {a.gpus}")
        return 2
    if not 1 <= a.temporal <= 24:
        log(rank, f"--temporal must be 1..24, got {a.temporal}")
        return 2

    gpu = a.device == "cuda"
    shared = a.shared_gpu_test and gpu and world > 1
    if shared:
        os.environ["RMA_SHARED_GPU"] = "1"  # select_device: ranks may share cuda:0
        os.environ["RMA_TRANSPORT"] = a.shared_gpu_transport
        if a.shared_gpu_transport == "rccl":  # RCCL's socket transport between the ranks
            os.environ["RMA_RCCL_SHARED_GPU"] = "1"
    elif gpu and world > 1:
        # a scaling point must never silently run on the host-staged transport
        os.environ["RMA_RCCL_STRICT"] = "1"
        os.environ["RMA_TRANSPORT"] = "rccl"
    diag = {k: v for k, v in sorted(os.environ.items())
            if k.startswith("RMA_DIAG") or k in ("RMA_FRAME_SIDES", "RMA_FRAME_ALIGNED",
                                                 "RMA_PASS_COSTS", "RMA_HALO_BATCH",
                                                 "RMA_FRAME_FILL", "RMA_EXEC_STREAMS",
                                                 "RMA_PIPE_FAST", "RMA_HALO_CROSS",
                                                 "RMA_FRAME_BANDS", "RMA_RCCL_LIB",
                                                 "RMA_FRAME_CHUNK_DIV")}
    if gpu and os.environ.get("RMA_PIPE_FAST") == "pipe5":  # an A/B of the lab kernel
        from rocm_mpi_amd._native import load_lab

        load_lab()
    check_on = a.check == 1 or (a.check < 0 and (gpu or world > 1))
    if check_on and os.environ.get("RMA_DIAG_SKIP_EXCHANGE", "0") == "1":
        log(rank, "RMA_DIAG_SKIP_EXCHANGE=1 skips every halo exchange: refused with the halo "
                  "check on (--check 0 for a diagnosis run)")
        return 2

    import torch

    from rocm_mpi_amd.models import Diffusion2D
    from rocm_mpi_amd.parallel import comm as C

    if gpu and not torch.cuda.is_available():
        log(rank, "needs an MI355X (no GPU visible)")
        return 2
    if not gpu and not a.nx:
        log(rank, "--device cpu needs --nx")
        return 2
    if world > 1:
        C.init_distributed(None if gpu and not shared else "gloo")
    local, _ = C.node_local_rank(rank, world)
    dev = str(C.select_device(local)) if gpu else "cpu"
    tmo = a.check_timeout

    # one rank per PHYSICAL GPU: compare PCI bus ids (shared GPUs would make
    # the scaling point meaningless)
    if gpu:
        from rocm_mpi_amd._native import native

        try:
            bus = native().device_pci_bus_id(torch.cuda.current_device())
        except Exception as e:  # noqa: BLE001 - fall back to the device UUID
            uuid = getattr(torch.cuda.get_device_properties(torch.cuda.current_device()),
                           "uuid", None)
            if uuid is None:
                log(rank, f"cannot identify the physical GPU (PCI bus id: {e})")
                return 2
            bus = f"uuid-{uuid}"
    else:
        bus = f"cpu-rank-{rank}"
    buses = gather_obj(bus, world)
    n_gpus = len(set(buses)) if gpu else world
    if gpu and n_gpus != world and not shared:
        log(rank, f"{world} ranks share {n_gpus} physical GPU(s) (PCI bus ids {buses}); "
                  "a scaling point needs one GPU per rank")
        return 2

    def sync():
        if gpu:
            torch.cuda.synchronize()

    dims = tuple(int(v) for v in a.dims.split(",")) + (0,)
    K = a.temporal if a.variant != "kp" else 1
    check_n = a.check_nx or (2050 if gpu else max(130, 6 * K + 2))
    self_rccl = (a.check_self_rccl == 1 or (a.check_self_rccl < 0 and gpu)) and world == 1 and gpu

    # the record is built up as the run goes: a failing phase still reports
    out = {"metric": METRIC + (" [shared-GPU functional test]" if shared else ""),
           "value": None, "unit": "GB/s", "n_gpus": n_gpus, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": None, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "fp64",
           "data": "synthetic: counter-based uniform [0,1) random-init temperature field",
           "config": {"model": f"diffusion_2D_{a.variant}", "ranks": world,
                      "pci_bus_ids": buses if gpu else None, "shared_gpu_test": bool(shared),
                      "diag_env": diag}}
    printed = [False]

    def emit(error: str | None = None) -> None:
        if rank != 0 or printed[0]:
            return
        printed[0] = True
        if error:
            out["error"] = error[:2000]
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")

    def fail_run(what: str, e: Exception, rc: int, wait_s: float | None = None) -> int:
        log(rank, f"{what}: {e}")
        emit(f"{what}: {e}")
        # in the bounded check protocol rank 0 reports within 3 x timeout; after
        # an unexpected error elsewhere it may be blocked in a collective
        finish_failed(rank, world, rc, 3 * tmo + 30 if wait_s is None else wait_s)
        return rc  # not reached

    # --- preflight: before the HBM-sized allocation --------------------------
    if a.preflight and a.variant != "kp":
        wd = Watchdog(rank, world, 3 * tmo, "preflight", emit)
        try:
            out["config"]["preflight"] = preflight(dims[:2], K, dev, world, rank, gpu,
                                                   max(130, 6 * K + 2), tmo)
        except CheckFailed as e:
            out["config"]["preflight"] = {"error": str(e.args[0])}
            return fail_run("preflight", e, 5)
        finally:
            wd.cancel()

    try:
        nx = a.nx or auto_tile(a.hbm_frac, a.max_tile)
        if world > 1 and not a.nx:
            import torch.distributed as dist

            t = torch.tensor([nx], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=C._gloo_group())
            nx = int(t.item())
        ny = a.ny or nx
        cfg = make_config(a, nx, ny, dev, dims)
        t_setup = time.perf_counter()
        gkw = {}
        if a.overlap:
            gkw = {"overlaps": (a.overlap, a.overlap, 2), "halowidths": (K, K, 1)}
        model = Diffusion2D(cfg, grid_kwargs=gkw)
        g = model.g
        comm = g.comm
        if gpu and world > 1 and g.transport != "rccl" and not shared:
            log(rank, f"halo transport is {g.transport!r}, a multi-GPU point needs RCCL")
            return 2
        model.synchronize()
        comm.barrier()
        setup_s = time.perf_counter() - t_setup

        fast_used = bool(model.cfg.fast_math)  # the side measurements below switch it off
        plan_warm = model.plan(a.warmup)
        plan_timed = model.plan(a.steps)
        model.step(a.warmup)
        model.synchronize()
        comm.barrier()
        model.enable_pass_timing(True)  # 5 event records per pass (~us against ~70 ms passes)
        sync()
        t0 = time.perf_counter()
        model.step(a.steps)
        sync()
        own_s = time.perf_counter() - t0  # this rank's own time, before the closing barrier
        comm.barrier()
        local_s = time.perf_counter() - t0
        wall = comm.allreduce(local_s, "max")
        nbrs = any(p >= 0 for side in g.neighbors[:2] for p in side)
        snap = snapshot_windows(model) if a.window_check and a.variant != "kp" else None
        timings = summarize_timings(model.pass_timings(), exchange=nbrs)
        model.enable_pass_timing(False)
        ex = getattr(model, "executor", None)
        # passes of the warmup + timed steps and how many ran as frame-first fused launches
        # (RMA_EXEC_FUSED: with neighbours and >= 2 waves of tasks per pass)
        exec_passes = ({"passes": int(ex.passes_done), "fused": int(ex.fused_passes)}
                       if ex is not None else None)
        bad = float(model.field[:: max(1, ny // 64), :: max(1, nx // 64)].isfinite().logical_not().sum())
        bad = comm.allreduce(bad, "sum")
        a_eff = 3 * nx * ny * 8 / 1e9

        def side_teff(Kside, fast, steps):
            model.set_temporal(Kside, fast_math=fast)
            model.step(2 * Kside)
            model.synchronize()
            comm.barrier()
            sync()
            s0 = time.perf_counter()
            model.step(steps)
            sync()
            comm.barrier()
            s1 = comm.allreduce(time.perf_counter() - s0, "max")
            return a_eff / (s1 / steps)

        # same-run weak-scaling reference: every rank re-times its tile without
        # the exchange (one launch per pass), all ranks concurrently; each rank's
        # own (pre-barrier) solo time identifies a slow GPU independently of the halo
        solo_steps = a.steps if a.solo_steps < 0 else a.solo_steps
        solo = solo_own = solo_iso = solo_iso_own = None
        if solo_steps > 0:
            model.set_solo(True)
            model.step(a.warmup)
            model.synchronize()
            comm.barrier()
            sync()
            s0 = time.perf_counter()
            model.step(solo_steps)
            sync()
            solo_own = (time.perf_counter() - s0) / solo_steps
            comm.barrier()
            solo = comm.allreduce(time.perf_counter() - s0, "max") / solo_steps
            # the same solo re-time at isotropic coefficients (dx = dy = the
            # smaller spacing: the same dt, ry = 1): splits the coefficient
            # energy of an anisotropic grid (4x2, 2x1) from the halo cost
            aniso = comm.allreduce(float(model.dx != model.dy), "max") > 0
            if aniso:
                d = min(model.dx, model.dy)
                model.set_spacing((d, d))
                model.step(a.warmup)
                model.synchronize()
                comm.barrier()
                sync()
                s0 = time.perf_counter()
                model.step(solo_steps)
                sync()
                solo_iso_own = (time.perf_counter() - s0) / solo_steps
                comm.barrier()
                solo_iso = comm.allreduce(time.perf_counter() - s0, "max") / solo_steps
                model.set_spacing(None)
            else:
                solo_iso_own, solo_iso = solo_own, solo
            model.set_solo(False)

        detail = {"rank": rank, "coords": list(g.coords[:2]),
                  "neighbors": [list(p) for p in g.neighbors[:2]], "pci_bus_id": bus,
                  "ms_per_step": round(own_s / a.steps * 1e3, 6),
                  "teff_GBps": round(a_eff / (own_s / a.steps), 2),
                  "solo_ms_per_step": round(solo_own * 1e3, 6) if solo_own else None,
                  "solo_iso_ms_per_step": round(solo_iso_own * 1e3, 6) if solo_iso_own else None,
                  "e_halo": round(solo_own / (own_s / a.steps), 6) if solo_own else None,
                  "e_coef": (round(solo_iso_own / solo_own, 6)
                             if solo_own and solo_iso_own else None),
                  "e_gpu": None, "e_gpu_vs_n1": None,
                  "pass_timing": {k: (round(v, 4) if isinstance(v, float) else v)
                                  for k, v in timings.items() if k != "note"}}
        ranks_detail = gather_obj(detail, world)
        teff_ranks = [d["teff_GBps"] for d in ranks_detail]

        # side measurements on the same tile: the canonical (bitwise) K-step
        # passes and the one-step kernel (24 B/cell/step at the HBM roofline)
        single = canonical = None
        kc = 1
        if K > 1:  # the canonical depth <= K with the lowest measured cost per step
            from rocm_mpi_amd._native import has_native, native

            if has_native():
                cc = native().default_pass_costs(K, False, float(nx) * float(ny))
                kc = min(range(1, K + 1), key=lambda k: cc[k] / k)
            else:
                kc = min(K, 8)
        if a.single_step_steps > 0 and K > 1:
            if a.fast_math:
                canonical = side_teff(kc, False, a.canonical_steps or 2 * kc)
            single = side_teff(1, False, a.single_step_steps)

        kinfo = None
        if K > 1:
            from rocm_mpi_amd import ops
            from rocm_mpi_amd._native import has_native, native

            if has_native():
                depth = max(plan_timed)
                if a.fast_math:
                    kern, kvec, kch = native().fast_kernel_k(depth, ny, tuple(model.coef))
                else:
                    kern, kvec, kch = native().canonical_kernel_k(depth, ny)
                names = {v: k for k, v in ops.KERNELS.items()}
                if kern >= 9:  # the cells per lane the kernel runs (vec 5 needs nx % 5 == 0)
                    kvec = native().pipe_vec(depth, 0, kern - 9, nx, kvec, True)
                kinfo = {"kernel": names[kern], "vec": kvec, "chunk_rows": a.chunk2 or kch,
                         "stages": native().pipe_default_stages(depth) if kern >= 9 else None}
        model.close()
        del model
        if gpu:
            torch.cuda.empty_cache()

        t_it = wall / a.steps
        teff_gpu = a_eff / t_it
        total = teff_gpu * world
        if not nbrs:
            par = "single rank, no halo exchange (one launch per pass)"
        else:
            tdesc = {"rccl": "RCCL send/recv over xGMI", "staged": "host-staged copies + gloo",
                     "gloo": "gloo (CPU twin)", "loopback": "in-process loopback",
                     "self": "periodic self copies"}.get(g.transport, g.transport)
            fused_run = bool(exec_passes and exec_passes["fused"])
            par = f"halo: {tdesc}" + (
                (", frame-first fused launch per pass, exchange on a high-priority stream "
                 "started by the frame tasks' device flag" if fused_run else
                 ", boundary frame + exchange on a high-priority stream overlapped with the "
                 "interior") if a.variant == "perf_hide" else ", exchange after each pass")
        # without a neighbour the solo re-time IS the run: no same-run efficiency
        eff_same = (solo / t_it) if solo and nbrs else None
        if shared:
            par = f"SHARED-GPU FUNCTIONAL TEST, {world} ranks on {n_gpus} GPU, not a scaling point; {par}"
        fast_plan = bool(fast_used)
        n1key = _n1_key(nx, ny, a.steps, a.warmup, K, fast_plan, a.variant)
        n1 = None
        if world == 1 and not nbrs:
            save_n1(n1key, t_it * 1e3, bus)
            n1 = {"ms_per_step": t_it * 1e3}
        elif world > 1:
            n1 = load_n1(n1key)
        n1_ms = n1["ms_per_step"] if n1 else None
        isos = [d["solo_iso_ms_per_step"] for d in ranks_detail if d["solo_iso_ms_per_step"]]
        fast_iso_ms = min(isos) if len(isos) == world else None
        slow_iso_ms = max(isos) if len(isos) == world else None
        for d in ranks_detail:
            if d["solo_iso_ms_per_step"] and fast_iso_ms:
                d["e_gpu"] = round(fast_iso_ms / d["solo_iso_ms_per_step"], 6)
            if d["solo_iso_ms_per_step"] and n1_ms:
                d["e_gpu_vs_n1"] = round(n1_ms / d["solo_iso_ms_per_step"], 6)
        attrib = attribution(t_it, solo, solo_iso,
                             fast_iso_ms / 1e3 if fast_iso_ms else None, n1_ms,
                             slow_iso_ms / 1e3 if slow_iso_ms else None)
        out.update({"value": round(total, 2), "value_kind": "aggregate",
                    "teff_per_gpu": round(teff_gpu, 2), "ms_per_step": round(t_it * 1e3, 6)})
        out["config"].update({
            "global_batch": g.nxyz_g[0] * g.nxyz_g[1],
            "seq_len": None,
            "parallelism": f"2D domain decomposition dims {g.dims[0]}x{g.dims[1]} ({par})",
            "local_grid": [nx, ny],
            "global_grid": [g.nxyz_g[0], g.nxyz_g[1]],
            "teff_per_gpu_GBps": round(teff_gpu, 2),
            "teff_per_gpu_min_GBps": round(min(teff_ranks), 2),
            "teff_per_gpu_max_GBps": round(max(teff_ranks), 2),
            "slowest_rank": int(max(range(world), key=lambda r: ranks_detail[r]["ms_per_step"])),
            "a_eff_GB_per_step": round(a_eff, 6),
            "max_steps_per_pass": K,
            "passes_warmup": plan_warm,
            "passes_timed": plan_timed,
            "kstep_kernel": kinfo,
            "fast_math": fast_used,
            "pass_timing": timings,
            "ranks_detail": ranks_detail,
            "solo_ms_per_step": round(solo * 1e3, 6) if solo else None,
            "solo_iso_ms_per_step": round(solo_iso * 1e3, 6) if solo_iso else None,
            "weak_scaling_eff_same_run": round(eff_same, 4) if eff_same else None,
            "e_attribution": dict(attrib, note=(
                "in-run E ~ fastest_solo_iso/t_it = e_gpu * e_coef * e_halo (e_product); "
                "e_halo = solo/t_it (exchange and frame cost), e_coef = solo_iso/solo "
                "(fast-math pass energy at dx != dy vs dx = dy), e_gpu = fastest/slowest "
                "own isotropic solo time of this job's GPUs (no exchange); e_box = t(N=1)/"
                "fastest_solo_iso against the N = 1 record of the same sweep, node and build "
                "(null without it), e_product_vs_n1 = t(N=1)/t_it; value is the aggregate "
                "N x teff_per_gpu")),
            "headline_window_check": None,
            "rccl_halo_bitwise_ok": None,
            "halo_check": None,
            "fast_math_drift_max": None,
            "drift_check": None,
            "teff_note": ("T_eff = A_eff/t_step with A_eff = 3*nx*ny*8 B (reference "
                          "perf.jl:55-58). With temporal blocking every step of every cell "
                          "is computed, but HBM is read/written once per pass of up to "
                          f"{K} steps, so T_eff exceeds the HBM bandwidth and is a time per "
                          "step, not a memory throughput; teff_single_step_kernel_GBps is "
                          "the one-step kernel on the same tile (the like-for-like memory "
                          "number). fast_math: the passes evaluate the same fp64 update as "
                          "a 5-point sum with one folded per-cell factor and FMAs "
                          "(rounding-level deviation from the canonical update, bounded in "
                          "fast_math_drift_max for this run's length; bitwise "
                          "equal to its CPU twin, tests/test_pipe_gpu.py); "
                          "teff_bitwise_kstep_GBps is the canonical K-step kernel on the "
                          "same tile") if K > 1 else "",
            "teff_single_step_kernel_GBps": round(single, 2) if single else None,
            "teff_bitwise_kstep_GBps": round(canonical, 2) if canonical else None,
            "bitwise_kstep_steps_per_pass": kc if canonical else None,
            "overlap": list(g.overlaps[:2]),
            "transport": g.transport,
            "rccl_nranks": _rccl_nranks(g, out["config"].get("preflight")),
            "rccl": _rccl_info() if gpu else None,
            "hipgraph": bool(a.graph),
            "executor_passes": exec_passes,
            "setup_s": round(setup_s, 3),
            "nonfinite_cells_sampled": int(bad),
        })

        # --- correctness of this run's code paths (bounded; any failure fails all)
        rc = 0 if bad == 0 else 3
        drift_steps = (a.warmup + a.steps) if a.drift_steps < 0 else a.drift_steps
        if (check_on or drift_steps or snap is not None) and a.variant != "kp":
            wd = Watchdog(rank, world, 3 * tmo, "check phase", emit)
            try:
                if drift_steps and fast_used and K > 1:
                    try:
                        di = drift_check(check_n, K, drift_steps, dev, world, tmo)
                    except CheckFailed as e:
                        out["config"]["drift_check"] = e.args[1] if len(e.args) > 1 else None
                        raise
                    out["config"]["drift_check"] = di
                    out["config"]["fast_math_drift_max"] = di["fast_math_drift_max"]
                if snap is not None:
                    try:
                        wc = window_check(snap, world, tmo)
                    except CheckFailed as e:
                        out["config"]["headline_window_check"] = (
                            dict(e.args[1], error=str(e.args[0])) if len(e.args) > 1
                            else {"bitwise": False, "error": str(e.args[0])})
                        raise
                    out["config"]["headline_window_check"] = wc
                if check_on:
                    try:
                        hc = halo_check(check_n, dims[:2], K, dev, world, rank, tmo,
                                        self_rccl=self_rccl)
                    except CheckFailed as e:
                        out["config"]["rccl_halo_bitwise_ok"] = False
                        out["config"]["halo_check"] = dict(e.args[1] if len(e.args) > 1 else {},
                                                           error=str(e.args[0]))
                        raise
                    out["config"]["halo_check"] = hc
                    out["config"]["rccl_halo_bitwise_ok"] = True
            except CheckFailed as e:
                return fail_run("check", CheckFailed(e.args[0]), 4)
            except Exception as e:  # noqa: BLE001 - an unexpected error is a failed check
                return fail_run("check", RuntimeError(f"{type(e).__name__}: {e}"), 4)
            finally:
                wd.cancel()
    except Exception as e:  # noqa: BLE001 - this rank reports and fails; torchrun ends the rest
        import traceback

        traceback.print_exc()
        return fail_run("run", RuntimeError(f"{type(e).__name__}: {e}"), 5, wait_s=10.0)
    emit()
    if world > 1:
        C.shutdown_distributed()
    return rc


if __name__ == "__main__":
    sys.exit(main())
