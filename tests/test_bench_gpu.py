"""bench.py on one GPU: the driver's command shape, its record, and the
in-run halo check path with real RCCL traffic (periodic grid, RCCL send/recv
to self vs local self copies), which a multi-GPU run uses across GPUs."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench(*args, timeout=300):
    from helpers import free_port

    env = dict(os.environ, MASTER_PORT=str(free_port()))  # multi-rank runs self-launch
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                       capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_small_tile_with_self_rccl_halo_check():
    d = bench("--steps", "20", "--warmup", "5", "--nx", "4096", "--single-step-steps", "8",
              "--check", "1", "--check-self-rccl", "--check-nx", "1026")
    c = d["config"]
    assert d["n_gpus"] == 1 and c["ranks"] == 1
    # the planner's choice for this tile class (its own cost table)
    from rocm_mpi_amd._native import native
    costs = native().default_pass_costs(24, True, 4096.0 * 4096.0)
    plan = list(native().plan_passes(20, costs))
    assert sum(plan) == 20 and c["passes_timed"] == plan
    assert c["passes_warmup"] == list(native().plan_passes(5, costs))
    # the deepest pass's kernel: register factors (piper) from K = 14 on (4096^2)
    assert c["kstep_kernel"]["kernel"] == ("piper" if max(plan) >= 14 else "pipe")
    assert c["rccl_halo_bitwise_ok"] is True
    hc = c["halo_check"]
    assert hc["transport"] == "rccl" and hc["self_rccl"] and hc["tiles_mismatched"] == 0
    pt = c["pass_timing"]
    assert pt["passes"] == len(plan) and pt["depths"] == plan and pt["interior_ms"] > 0
    assert pt["overlap_fraction"] is None and "no neighbour" in pt["note"]  # nothing exchanged
    # no neighbour: the solo re-time is the run itself (no same-run efficiency)
    assert c["weak_scaling_eff_same_run"] is None and c["solo_ms_per_step"] > 0
    # preflight over RCCL (ring to self + tiny periodic halo check), drift bound
    pf = c["preflight"]
    assert pf["ring_ok"] and pf["halo"]["transport"] == "rccl" and pf["halo"]["self_rccl"]
    assert pf["halo"]["tiles_mismatched"] == 0
    assert c["drift_check"]["steps"] == 25 and c["fast_math_drift_max"] <= 1e-14
    rd = c["ranks_detail"]
    assert len(rd) == 1 and rd[0]["pci_bus_id"] == c["pci_bus_ids"][0]
    assert c["teff_single_step_kernel_GBps"] > 0 and c["teff_bitwise_kstep_GBps"] > 0
    assert c["pci_bus_ids"] and len(c["pci_bus_ids"]) == 1
    # every cell of the timed field: finite, inside the initial bounds (max principle)
    ff = c["full_field_check"]
    assert ff["ok"] and ff["nonfinite"] == 0 and ff["cells"] == 4096 * 4096 and ff["steps"] == 25
    assert ff["init_min"] <= ff["min"] <= ff["max"] <= ff["init_max"]
    # per-link probe at the timed tile's message sizes (one GPU: RCCL to itself)
    lk = pf["links"]
    assert lk["sizes"]["x_plane"] == 24 * 4096 * 8 and lk["all_p2p"] is None
    r0 = lk["ranks"][0]
    assert r0["transport"].startswith("self") and r0["peers"] == [0]
    assert [t["message"] for t in r0["timed"]] == ["latency_8B", "x_plane", "y_plane"]
    assert all(t["data_ok"] and t["us"] > 0 for t in r0["timed"])
    # the timed field itself: three full-width row windows bitwise vs the CPU twin
    wc = c["headline_window_check"]
    assert wc["windows"] == 3 and wc["bitwise"] is True and wc["full_width"] is True
    assert wc["steps"] == 25 and wc["arithmetic"] == "fast-math twin"
    # N = 1: isotropic grid, no exchange -> e_halo = e_coef = 1 by construction
    assert d["value_kind"] == "aggregate" and d["teff_per_gpu"] == c["teff_per_gpu_GBps"]
    ea = c["e_attribution"]
    assert ea["e_coef"] == 1.0 and c["solo_iso_ms_per_step"] == c["solo_ms_per_step"]
    assert ea["e_gpu"] == 1.0  # one GPU: the fastest is the slowest
    assert c["rccl"]["version"] > 0 and c["rccl"]["library"]
    # the preflight ring went through an RCCL communicator of exactly 1 rank
    # (ncclCommCount)
    assert pf["ring_transport"] == "rccl" and pf["rccl_nranks"] == 1 == d["n_gpus"]
    assert c["rccl_nranks"] == 1


def test_bench_default_check_on_one_gpu():
    """The driver's N=1 command shape: the RCCL-self halo check and the drift
    bound run by default."""
    d = bench("--steps", "48", "--warmup", "4", "--nx", "2048", "--single-step-steps", "0",
              "--check-nx", "530")
    c = d["config"]
    assert c["rccl_halo_bitwise_ok"] is True and c["halo_check"]["self_rccl"]
    assert c["halo_check"]["transport"] == "rccl"
    assert c["drift_check"]["steps"] == 52 and c["fast_math_drift_max"] <= 1e-14


@pytest.mark.parametrize("transport", ["staged", "ipc", "rccl"])
def test_bench_two_processes_sharing_the_gpu(tmp_path, transport):
    """The multi-process bench flow on one GPU (torchrun-style ranks, staged or
    HIP-IPC halo transport, per-rank timings, solo re-time, in-run halo check):
    a functional test, labelled so it can never pass for a scaling point."""
    d = bench("--gpus", "2", "--shared-gpu-test", "--shared-gpu-transport", transport, "--nx",
              "4096", "--steps", "24", "--warmup", "5", "--single-step-steps", "4", "--check-nx",
              "530", timeout=600)
    c = d["config"]
    assert c["shared_gpu_test"] is True and "shared-GPU" in d["metric"]
    assert c["ranks"] == 2 and d["n_gpus"] == 1 and c["transport"] == transport
    assert c["rccl_halo_bitwise_ok"] is True and c["halo_check"]["tiles_mismatched"] == 0
    assert c["pass_timing"]["passes"] == len(c["passes_timed"]) and sum(c["passes_timed"]) == 24
    assert len(c["pci_bus_ids"]) == 2 and c["full_field_check"]["ok"]
    assert c["scaling_point"] is False
    lk = c["preflight"]["links"]
    assert [r["peers"] for r in lk["ranks"]] == [[1], [0]]
    assert all(t["data_ok"] for r in lk["ranks"] for t in r["timed"])
    if transport == "rccl":  # RCCL between processes sharing cuda:0: its socket transport
        assert [r["transport"] for r in lk["ranks"]] == ["socket", "socket"]
        assert lk["all_p2p"] is False and "NET/Socket" in lk["ranks"][0]["transport_kinds"]
    assert [r["rank"] for r in c["ranks_detail"]] == [0, 1]
    assert c["preflight"]["ring_ok"] and c["preflight"]["halo"]["transport"] == transport
    assert c["headline_window_check"]["bitwise"] is True


@pytest.mark.parametrize("gpus,dims", [(4, (2, 2)), (8, (4, 2))])
def test_bench_rehearsal_of_the_scaling_run_over_rccl(gpus, dims):
    """The driver's N-GPU command shape (bench.py --gpus N: torchrun ranks,
    preflight device ring, RCCL halo exchange, in-run halo / window / drift
    checks, per-rank timings, E(N) attribution) with N real RCCL ranks on the
    one GPU of this box (RMA_RCCL_SHARED_GPU: RCCL's socket transport instead
    of xGMI). Functional, never a scaling point: the record says so."""
    d = bench("--gpus", str(gpus), "--shared-gpu-test", "--shared-gpu-transport", "rccl",
              "--nx", "2048", "--steps", "48", "--warmup", "4", "--single-step-steps", "0",
              "--check-nx", "530", timeout=600)
    c = d["config"]
    assert c["shared_gpu_test"] is True and c["ranks"] == gpus and c["transport"] == "rccl"
    assert c["global_grid"] == [dims[0] * (2048 - 48) + 48, dims[1] * (2048 - 48) + 48]
    assert c["rccl_nranks"] == gpus and c["preflight"]["rccl_nranks"] == gpus
    assert c["preflight"]["ring_ok"] and c["preflight"]["halo"]["tiles_mismatched"] == 0
    assert c["rccl_halo_bitwise_ok"] is True and c["halo_check"]["transport"] == "rccl"
    assert c["headline_window_check"]["bitwise"] is True
    assert c["pass_timing"]["halo_ms"] > 0 and sum(c["passes_timed"]) == 48
    ea = c["e_attribution"]
    assert ea["e_gpu"] is not None and ea["e_product"] is not None
    assert [r["rank"] for r in c["ranks_detail"]] == list(range(gpus))
    # the record proves its own transport and links
    lk = c["preflight"]["links"]
    assert {r["transport"] for r in lk["ranks"]} == {"socket"} and lk["all_p2p"] is False
    assert all(len(r["timed"]) == 3 * len(r["peers"]) and r["peers"] for r in lk["ranks"])
    assert c["scaling_point"] is False and c["full_field_check"]["ok"]
    assert "socket" in c["parallelism"] or "NET" in c["parallelism"] or "socket" in str(lk)
