"""Per-pass timing summary and the weak-scaling attribution of a bench.py run
(in-run e_halo * e_coef * e_gpu and, with the N = 1 record of the same sweep,
e_box)."""
from __future__ import annotations

import json
import os
import time


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


# weak-scaling attribution. Self-contained in
# one job: E_in_run = t_fast_iso / t_it = e_gpu * e_coef * e_halo, with
# t_fast_iso the fastest rank's own isotropic solo time (no exchange). The
# N = 1 record of the same tile class (cached by the same driver sweep on the
# same node and build) adds e_box = t(N=1) / t_fast_iso, so that
# E(N) = t(N=1) / t_it = e_box * E_in_run.
def _n1_cache_path() -> str:
    import tempfile

    from rocm_mpi_amd.config import diag_value

    return (diag_value("bench_n1_cache")
            or os.path.join(tempfile.gettempdir(), "rma_bench_n1_record.json"))


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
