"""bench.py's full-field check: one pass over every cell
of the timed field (non-finite count, min, max: ``ops.field_stats``, native
CPU twin here, the HIP kernel on the GPU: tests/test_kernels_gpu.py) and the
explicit scheme's maximum principle against the initial field's bounds."""
import json
import math
import os
import subprocess
import sys

import pytest
import torch

from helpers import ROOT
from rocm_mpi_amd import ops
from rocm_mpi_amd.benchmark import checks
from rocm_mpi_amd.benchmark.common import CheckFailed


class _Self:  # a one-rank communicator
    def allreduce(self, v, op="sum"):
        return float(v)


def test_field_stats_cpu_twin():
    g = torch.Generator().manual_seed(3)
    a = torch.rand((37, 53), generator=g, dtype=torch.float64) * 4 - 1
    assert ops.field_stats(a) == (0.0, float(a.min()), float(a.max()))
    a[5, 7] = float("nan")
    a[30, 1] = float("inf")
    a[0, 0] = -float("inf")
    bad, lo, hi = ops.field_stats(a)
    fin = a[torch.isfinite(a)]
    assert (bad, lo, hi) == (3.0, float(fin.min()), float(fin.max()))
    odd = torch.arange(7, dtype=torch.float64)  # odd length: the scalar tail
    assert ops.field_stats(odd) == (0.0, 0.0, 6.0)


def test_full_field_check_passes_a_diffused_field():
    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig

    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=130, ny=98, nt=30, warmup=0,
                                    device="cpu", quiet=True, init="random", temporal=6))
    init = checks.field_stats_global(m.field, _Self())
    m.step(30)
    info = checks.full_field_check(m.field, init, m.steps_done, _Self(), 1, 0, 10.0)
    m.close()
    assert info["ok"] and info["nonfinite"] == 0 and info["cells"] == 130 * 98
    assert init[1] <= info["min"] and info["max"] <= init[2]
    assert info["max"] < init[2]  # diffusion shrinks the range of a random field


@pytest.mark.parametrize("kind", ["nan", "hot", "cold"])
def test_full_field_check_fails_on_injected_cell(monkeypatch, kind):
    f = torch.full((20, 30), 0.5, dtype=torch.float64)
    f[3, 4], f[9, 9] = 0.0, 1.0
    init = checks.field_stats_global(f, _Self())
    monkeypatch.setenv("RMA_DIAG", f"bench_field_corrupt={kind}")
    with pytest.raises(CheckFailed) as ei:
        checks.full_field_check(f, init, 10, _Self(), 1, 0, 10.0)
    info = ei.value.args[1]
    assert info["ok"] is False and info["injected"] == kind
    assert ("non-finite" in info["error"]) == (kind == "nan")


def test_full_field_check_tolerance_is_rounding_sized():
    f = torch.full((4, 4), 0.25, dtype=torch.float64)
    init = (0.0, 0.0, 1.0)
    f[1, 1] = 1.0 + 8 * 2.0 ** -52  # within 8 ulps per step
    checks.full_field_check(f, init, 1, _Self(), 1, 0, 10.0)
    f[1, 1] = 1.0 + 1e-12
    with pytest.raises(CheckFailed, match="maximum principle"):
        checks.full_field_check(f, init, 10, _Self(), 1, 0, 10.0)


@pytest.mark.parametrize("corrupt", ["", "nan"])
def test_bench_cpu_records_full_field_check(tmp_path, corrupt):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    env.pop("RMA_DIAG", None)
    if corrupt:
        env["RMA_DIAG"] = f"bench_field_corrupt={corrupt}"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu",
                        "--nx", "130", "--steps", "12", "--warmup", "2",
                        "--single-step-steps", "2"], capture_output=True, text=True,
                       timeout=600, cwd=str(tmp_path), env=env)
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    ffc = rec["config"]["full_field_check"]
    if corrupt:
        assert r.returncode == 3 and ffc["ok"] is False and "non-finite" in rec["error"]
    else:
        assert r.returncode == 0, r.stderr[-2000:]
        assert ffc["ok"] and ffc["cells"] == 130 * 130 and ffc["steps"] == 14
        assert ffc["init_min"] <= ffc["min"] <= ffc["max"] <= ffc["init_max"]
        assert math.isfinite(ffc["seconds"])


# RCCL INFO lines in the shapes RCCL 2.2x logs them (connection setup of the
# ring/tree channels and of point-to-point send/recv channels)
P2P_LOG = """\
node:4101:4101 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC comm 0x55d1 nRanks 04
node:4101:4101 [0] NCCL INFO Channel 01/0 : 3[3] -> 0[0] via P2P/IPC comm 0x55d1 nRanks 04
node:4101:4188 [0] NCCL INFO Channel 00/1 : 0[0] -> 2[2] [send] via P2P/IPC/read
node:4101:4188 [0] NCCL INFO Channel 00/1 : 2[2] -> 0[0] [receive] via P2P/IPC/read
node:4101:4188 [0] NCCL INFO Channel 02/1 : 0[3e000] -> 1[4e000] [send] via P2P/direct pointer
node:4101:4101 [0] NCCL INFO Connected all rings comm 0x55d1 nRanks 04
"""
SOCKET_LOG = """\
box:77:77 [0] NCCL INFO NET/Socket : Using [0]lo:127.0.0.1<0>
box:77:77 [0] NCCL INFO Channel 00/0 : 1[0] -> 0[0] [receive] via NET/Socket/0
box:77:77 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[0] [send] via NET/Socket/0
box:77:91 [0] NCCL INFO Channel 01/1 : 0[0] -> 2[0] [send] via NET/Socket/0
"""


def test_rccl_connection_parser_p2p_and_socket():
    from rocm_mpi_amd.benchmark import preflight as P

    c = P.parse_rccl_connections(P2P_LOG, rank=0)
    assert c == {1: ["P2P"], 2: ["P2P"], 3: ["P2P"]}
    assert P.classify_links(c, [1, 2])["verdict"] == "p2p"
    s = P.parse_rccl_connections(SOCKET_LOG, rank=0)
    assert s == {1: ["NET/Socket"], 2: ["NET/Socket"]}
    assert P.classify_links(s, [1, 2]) == {"verdict": "socket", "kinds": ["NET/Socket"],
                                           "peers_without_log": []}
    # one socket link among P2P links makes the rank non-P2P; a peer without
    # any logged connection leaves it unknown
    mixed = P.parse_rccl_connections(P2P_LOG + SOCKET_LOG, rank=0)
    assert P.classify_links(mixed, [1, 2, 3])["verdict"] == "socket"
    assert P.classify_links(c, [1, 5])["verdict"] == "unknown"
    assert P.parse_rccl_connections(P2P_LOG, rank=3) == {0: ["P2P"]}


def test_rccl_debug_env_never_uses_stdout(tmp_path):
    from rocm_mpi_amd.benchmark import preflight as P

    env = P.rccl_debug_env(str(tmp_path))
    assert env["NCCL_DEBUG"] == "INFO" and "P2P" in env["NCCL_DEBUG_SUBSYS"]
    assert env["NCCL_DEBUG_FILE"].startswith(str(tmp_path)) and "%p" in env["NCCL_DEBUG_FILE"]
    import os as _os
    import socket

    f = env["NCCL_DEBUG_FILE"].replace("%h", socket.gethostname()).replace("%p", str(_os.getpid()))
    open(f, "w").write(SOCKET_LOG)
    old = _os.environ.get("NCCL_DEBUG_FILE")
    assert P.read_own_rccl_log(env["NCCL_DEBUG_FILE"]) == SOCKET_LOG
    assert old == _os.environ.get("NCCL_DEBUG_FILE")
