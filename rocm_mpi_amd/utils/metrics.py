"""T_eff metric and run records.

Definition preserved exactly from ``scripts/diffusion_2D_perf.jl:55-58`` (same
lines in perf_hide.jl:108-111 and perf_hide_prof.jl:125-128)::

    A_eff    = (2 + 1)/1e9*nx*ny*sizeof(Float64)   # GB per iteration: read T, write T2, read Cp
    wtime_it = wtime/(nt-10)                       # first 10 iterations untimed
    T_eff    = A_eff/wtime_it                      # GB/s, PER GPU (local nx, ny incl. halo)

Weak-scaling efficiency (not defined by the reference):
``E(N) = T_eff_per_gpu(N) / T_eff_per_gpu(1)`` at fixed local tile.
"""
from __future__ import annotations

import json
import math
import time
from dataclasses import asdict, dataclass, field


def now() -> float:
    """Wall clock for host-side timings (time.perf_counter)."""
    return time.perf_counter()


def a_eff_gb(nx: int, ny: int, nz: int = 1, arrays: int = 3, elem_bytes: int = 8) -> float:
    return arrays / 1e9 * nx * ny * nz * elem_bytes


def t_eff(nx: int, ny: int, wtime: float, timed_steps: int, nz: int = 1) -> float:
    if timed_steps <= 0 or wtime <= 0:
        return float("nan")
    return a_eff_gb(nx, ny, nz) / (wtime / timed_steps)


def round_sig(x: float, sig: int = 3) -> float:
    """Julia ``round(x, sigdigits=sig)``."""
    if x == 0 or not math.isfinite(x):
        return x
    return round(x, sig - int(math.floor(math.log10(abs(x)))) - 1)


def reference_line(nt: int, wtime: float, teff: float) -> str:
    """The reference's printf: ``Executed %d steps in = %1.3e sec (@ T_eff = %1.2f GB/s)``."""
    return f"Executed {nt:d} steps in = {wtime:1.3e} sec (@ T_eff = {round_sig(teff, 3):1.2f} GB/s) "


def weak_scaling_efficiency(teff_per_gpu_n: float, teff_per_gpu_1: float) -> float:
    return teff_per_gpu_n / teff_per_gpu_1 if teff_per_gpu_1 > 0 else float("nan")


@dataclass
class RunResult:
    variant: str
    nprocs: int
    dims: tuple
    nx: int
    ny: int
    nxg: int
    nyg: int
    nt: int
    timed_steps: int
    wtime: float  # seconds for the timed steps (max over ranks via barrier-synced toc)
    t_it: float
    teff: float  # per GPU, GB/s (rank-local tile)
    teff_min: float = float("nan")
    teff_max: float = float("nan")
    teff_total: float = float("nan")  # whole-job aggregate
    transport: str = ""
    device: str = ""
    extra: dict = field(default_factory=dict)

    def to_json(self) -> str:
        d = asdict(self)
        d["dims"] = list(self.dims)
        return json.dumps(d)
