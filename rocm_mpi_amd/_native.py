"""Loader for the compiled native core ``rocm_mpi_amd._C``.

GPU code paths call :func:`native` and fail LOUDLY if the extension is missing
(no silent eager fallback on a GPU box). CPU code paths may use the CPU twins
from the same extension, or pure-torch implementations when it is absent.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        # torch first: the extension links libamdhip64.so.7 / librccl.so.1 by
        # SONAME and must bind to the copies torch already loaded (one HIP
        # runtime per process).
        import torch  # noqa: F401

        try:
            _mod = importlib.import_module("rocm_mpi_amd._C")
        except ImportError as e:  # not built yet
            if os.environ.get("RMA_AUTOBUILD", "1") != "0":
                try:
                    from rocm_mpi_amd import _build

                    _build.build()
                    _mod = importlib.import_module("rocm_mpi_amd._C")
                    return
                except Exception as be:  # pragma: no cover - reported below
                    _err = RuntimeError(f"native core missing and build failed: {be}")
                    return
            _err = e


def has_native() -> bool:
    _load()
    return _mod is not None


def native():
    """Return the native module or raise (never a silent fallback)."""
    _load()
    if _mod is None:
        raise RuntimeError(
            "rocm_mpi_amd native core (_C) is not available: run "
            "`python -m rocm_mpi_amd._build` (hipcc, gfx950). Cause: " + repr(_err)
        )
    return _mod


def native_path() -> str | None:
    _load()
    return getattr(_mod, "__file__", None)


_lab = None


def load_lab():
    """Load librma_lab.so (csrc/lab: the superseded / experimental kernels kept
    as test oracles and for sweeps); it installs them in the core's K-step
    dispatchers. Idempotent; loud failure if the library is missing."""
    global _lab
    native()  # the core first: the lab library binds to this process's librma_core.so
    with _lock:
        if _lab is None:
            import ctypes

            path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librma_lab.so")
            if not os.path.exists(path):
                raise RuntimeError(f"{path} is missing: run `python -m rocm_mpi_amd._build`")
            _lab = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    return _lab


def lab_loaded() -> bool:
    return _lab is not None
