"""Environment configuration, Python side (C++ side: csrc/include/rma/config.h).

Tuning knobs are documented variables of their own (docs/TUNING.md): RMA_TRANSPORT,
RMA_IPC_MODE, RMA_IPC_MAILBOX_MB, RMA_COMM_TIMEOUT, RMA_TEARDOWN_TIMEOUT,
RMA_RCCL_BLOCKING, RMA_RCCL_LIB, RMA_RCCL_STRICT, RMA_RCCL_SHARED_GPU,
RMA_SHARED_GPU, RMA_EXEC_FUSED, RMA_EXEC_FUSED_TIMEOUT, RMA_GATHER_MAX_BYTES,
RMA_NUM_THREADS, RMA_OFFLOAD_ARCH, RMA_AUTOBUILD.

Every diagnostic / A-B switch / test injection is a key of ONE variable::

    RMA_DIAG="key[=value],key[=value],..."      e.g. RMA_DIAG=no_lag,exec_streams=hifirst

An unknown key is an error (both sides check the same list, DIAG_KEYS here and
kDiagKeys in csrc/runtime/config.cpp). Values may not contain ','.
The reference's whole configuration surface is 8 constants per script
(scripts/diffusion_2D_perf.jl:15-25) and IGG_ROCMAWARE_MPI (scripts/setenv.sh:13).
"""
from __future__ import annotations

import os

# key -> what it does (mirrors kDiagKeys, csrc/runtime/config.cpp)
DIAG_KEYS = {
    # executor / planner (C++)
    "skip_exchange": "every halo exchange skipped (WRONG multi-rank results)",
    "exec_streams": "pool | lofirst | hifirst | plain: executor stream creation",
    "exec_verbose": "print the executor's stream priorities",
    "no_prime": "no kernel priming at executor construction",
    "no_lag": "every pass waits for the previous exchange",
    "no_halo_cross": "one-step passes: one RCCL group per dimension",
    "no_halo_merged": "x+y neighbours: one group per dimension (C++ and Python)",
    "no_halo_batch": "one pack / unpack launch per plane",
    "frame_sides": "all: frame rects on every side once any neighbour exists",
    "frame_chunk_div": "N: aligned frame tasks of 1/N the interior's rows",
    "frame_aligned": "0 | 1: force the frame layout",
    "frame_bands": "task | ol: force the aligned y-band height",
    "no_frame_fill": "frame bands not filled into the interior",
    "pipe_fast": "pipe | pipe5: the LDS-ring fast kernel at every depth",
    "pass_costs": "K:cost/K:cost/...: planner cost overrides",
    # communication (C++)
    "rccl_data_blocking": "blocking RCCL data path of a non-blocking communicator",
    "rccl_graph": "allow hipGraph capture over RCCL",
    "no_ipc_graph": "refuse hipGraph capture over the IPC transport",
    # Python side
    "hostname": "node name for the local-rank exchange (tests)",
    "rccl_fallback": "an RCCL init failure falls back to the staged transport",
    "bench_rc_dir": "bench.py: every rank writes its exit status into this directory",
    "bench_n1_cache": "bench.py: path of the N = 1 record",
    "bench_check_raise": "bench.py: before | after: injected halo-check failure",
    "bench_check_corrupt": "bench.py: corrupt one halo-check cell",
    "bench_window_corrupt": "bench.py: corrupt one headline-window cell",
    "bench_field_corrupt": "bench.py: nan | hot | cold: one bad timed-field cell",
    "bench_rccl_log_dir": "bench.py: RCCL log directory of the link probe",
}


def diag_entries(s: str | None = None) -> dict:
    """{key: value} of RMA_DIAG (a bare key has value "1"); unknown keys raise."""
    s = os.environ.get("RMA_DIAG", "") if s is None else s
    out = {}
    for item in filter(None, (p.strip() for p in s.split(","))):
        k, _, v = item.partition("=")
        if k not in DIAG_KEYS:
            raise ValueError(f"RMA_DIAG: unknown key {k!r} (known: {', '.join(DIAG_KEYS)})")
        out[k] = v if "=" in item else "1"
    return out


def diag_flag(key: str) -> bool:
    """``key`` (or ``key=<not 0>``) in RMA_DIAG."""
    assert key in DIAG_KEYS, key
    v = diag_entries().get(key)
    return v is not None and v != "0"


def diag_value(key: str, default: str = "") -> str:
    """The value of ``key=value`` in RMA_DIAG, else ``default``."""
    assert key in DIAG_KEYS, key
    return diag_entries().get(key, default)


def diag_with(base: str | None = None, **kv) -> str:
    """An RMA_DIAG string with these keys set (True: bare key; None / False:
    removed), e.g. for a child process's environment."""
    d = diag_entries(base)
    for k, v in kv.items():
        if k not in DIAG_KEYS:
            raise ValueError(f"unknown RMA_DIAG key {k!r}")
        if v is None or v is False:
            d.pop(k, None)
        else:
            d[k] = "1" if v is True else str(v)
    return ",".join(k if v == "1" else f"{k}={v}" for k, v in d.items())
