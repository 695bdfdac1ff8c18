"""Profiling helpers (the ``perf_hide_prof`` variant).

The reference wraps its time loop in Julia's sampling profiler and rank 0
writes a flat tree to ``./prof.txt`` (scripts/diffusion_2D_perf_hide_prof.jl:
34,110-121). Here ``--profile`` turns on:

* host-side profiling of the timed loop with ``cProfile`` (rank 0 writes
  ``prof.txt``, top 30 entries by cumulative time — the maxdepth=30 analogue);
* ROCTX ranges from the native executor (rma.step.*, rma.boundary, rma.halo,
  rma.interior) visible in ``rocprofv3 --marker-trace`` timelines.

GPU kernel time is measured with ``rocprofv3 --kernel-trace --stats`` (see
scripts/profile.sh), not from inside the process.
"""
from __future__ import annotations

import contextlib
import cProfile
import io
import pstats


def roctx_enable(on: bool = True) -> bool:
    from .._native import has_native, native

    if not has_native():
        return False
    native().trace_enable(bool(on))
    return bool(native().trace_enabled())


@contextlib.contextmanager
def range_(name: str):
    from .._native import has_native, native

    if has_native() and native().trace_enabled():
        native().trace_push(name)
        try:
            yield
        finally:
            native().trace_pop()
    else:
        yield


class LoopProfiler:
    def __init__(self, enabled: bool, rank: int = 0):
        self.enabled = enabled
        self.rank = rank
        self._p = cProfile.Profile() if enabled else None
        self.roctx = False

    def __enter__(self):
        if self.enabled:
            self.roctx = roctx_enable(True)
            self._p.enable()
        return self

    def __exit__(self, *exc):
        if self.enabled:
            self._p.disable()
            roctx_enable(False)
        return False

    def report(self, limit: int = 30) -> str:
        if not self.enabled:
            return ""
        s = io.StringIO()
        pstats.Stats(self._p, stream=s).sort_stats("cumulative").print_stats(limit)
        return s.getvalue()

    def write(self, path: str = "prof.txt") -> None:
        if self.enabled and self.rank == 0:
            with open(path, "w") as f:
                f.write(self.report())
