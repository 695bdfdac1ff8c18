"""Node-local device selection on every entry path.

The reference selects the GPU from the node-local rank of a shared-memory
communicator split (``scripts/rocmaware_test_selectdevice.jl:5-9``). Here:
``select_device`` refuses more local ranks than visible GPUs unless a
shared-GPU test mode is on, and importing the package sets the IPC mode the
driver needs before any GPU call. CPU only: the GPU count is faked."""
import os
import subprocess
import sys

import pytest
import torch

from helpers import ROOT
from rocm_mpi_amd.parallel import comm as C


@pytest.fixture
def fake_gpus(monkeypatch):
    picked = []
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: picked.append(d))

    def with_n(n):
        monkeypatch.setattr(C, "visible_devices", lambda: n)
        return picked

    return with_n


def test_one_rank_per_gpu(fake_gpus, monkeypatch):
    monkeypatch.delenv("RMA_SHARED_GPU", raising=False)
    monkeypatch.delenv("RMA_RCCL_SHARED_GPU", raising=False)
    picked = fake_gpus(8)
    for lr in range(8):
        assert C.select_device(lr) == torch.device("cuda", lr)
    assert picked == [torch.device("cuda", lr) for lr in range(8)]


@pytest.mark.parametrize("n,lr", [(1, 1), (4, 4), (8, 9)])
def test_oversubscription_is_an_error(fake_gpus, monkeypatch, n, lr):
    monkeypatch.delenv("RMA_SHARED_GPU", raising=False)
    monkeypatch.delenv("RMA_RCCL_SHARED_GPU", raising=False)
    picked = fake_gpus(n)
    with pytest.raises(RuntimeError, match=rf"node-local rank {lr} but only {n} visible GPU"):
        C.select_device(lr)
    assert picked == []  # refused before touching any device
    with pytest.raises(ValueError):
        C.select_device(-1)


@pytest.mark.parametrize("var", ["RMA_SHARED_GPU", "RMA_RCCL_SHARED_GPU"])
def test_shared_gpu_test_modes_wrap(fake_gpus, monkeypatch, var):
    monkeypatch.delenv("RMA_SHARED_GPU", raising=False)
    monkeypatch.delenv("RMA_RCCL_SHARED_GPU", raising=False)
    monkeypatch.setenv(var, "1")
    fake_gpus(1)
    assert C.shared_gpu_allowed()
    assert C.select_device(3) == torch.device("cuda", 0)


def test_local_rank_sources(monkeypatch):
    """torchrun's LOCAL_RANK, else SLURM / Open MPI / MPICH node-local ids;
    never the global rank."""
    for k in ("LOCAL_RANK", "SLURM_LOCALID", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
              "RANK", "SLURM_PROCID"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("SLURM_PROCID", "13")
    assert C.env_world()[2] is None
    monkeypatch.setenv("SLURM_LOCALID", "5")
    assert C.env_world()[:1] == (13,) and C.env_world()[2] == 5
    monkeypatch.setenv("LOCAL_RANK", "2")
    assert C.env_world()[2] == 2


def test_package_import_sets_ipc_mode_default():
    """``import rocm_mpi_amd`` alone (no setenv.sh, no bench.py) sets
    HSA_ENABLE_IPC_MODE_LEGACY=0, and keeps a value the user set."""
    code = "import os, rocm_mpi_amd; print(os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY'))"
    env = {k: v for k, v in os.environ.items() if k != "HSA_ENABLE_IPC_MODE_LEGACY"}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT,
                       env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == "0"
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "1"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT,
                       env=env, timeout=120)
    assert r.stdout.strip().splitlines()[-1] == "1"
