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
import json  # noqa: E402
import math  # noqa: E402
import subprocess  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "T_eff (GB/s) + weak-scaling eff., 2D diffusion 1000 steps at 1/2/4/8 MI355X"


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
    ap.add_argument("--link-probe", type=int, default=1,
                    help="preflight: time one exchange per halo neighbour at the timed tile's "
                         "message sizes and record RCCL's transport per connection (1/0)")
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
    ap.add_argument("--full-field-check", type=int, default=1,
                    help="after the timed run, one device pass over every cell of the timed "
                         "field: finite and within the initial field's bounds (maximum "
                         "principle of the explicit scheme) (1/0)")
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


from rocm_mpi_amd.benchmark.attribution import (_n1_key, attribution, load_n1,  # noqa: E402
                                                save_n1, summarize_timings)
from rocm_mpi_amd.benchmark.checks import (DRIFT_BOUND, drift_check,  # noqa: E402,F401
                                           field_stats_global, full_field_check, halo_check,
                                           snapshot_windows, window_check)
from rocm_mpi_amd.benchmark.common import (CheckFailed, Watchdog, finish_failed,  # noqa: E402
                                           gather_obj, log, record_rc)
from rocm_mpi_amd.benchmark.preflight import _rccl_info, _rccl_nranks, preflight  # noqa: E402
from rocm_mpi_amd.config import diag_entries, diag_flag, diag_value  # noqa: E402


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
    if gpu and a.link_probe and (os.environ.get("NCCL_DEBUG", "").upper() in ("", "VERSION", "WARN")
                                 or not os.environ.get("NCCL_DEBUG_FILE")):
        # RCCL's connection log (which transport each peer link uses), one file
        # per process, before this process's first RCCL call
        import tempfile

        from rocm_mpi_amd.benchmark.preflight import rccl_debug_env

        ld = diag_value("bench_rccl_log_dir") or os.path.join(
            tempfile.gettempdir(), f"rma_rccl_{os.environ.get('MASTER_PORT', 'solo')}")
        os.makedirs(ld, exist_ok=True)
        os.environ.update(rccl_debug_env(ld))
    if shared:
        os.environ["RMA_SHARED_GPU"] = "1"  # select_device: ranks may share cuda:0
        os.environ["RMA_TRANSPORT"] = a.shared_gpu_transport
        if a.shared_gpu_transport == "rccl":  # RCCL's socket transport between the ranks
            os.environ["RMA_RCCL_SHARED_GPU"] = "1"
    elif gpu and world > 1:
        # a scaling point must never silently run on the host-staged transport
        os.environ["RMA_RCCL_STRICT"] = "1"
        os.environ["RMA_TRANSPORT"] = "rccl"
    # every diagnostic switch of this run (RMA_DIAG, validated) and the tuning
    # knobs that change what the timed passes run
    diag = {k: v for k, v in sorted(os.environ.items())
            if k in ("RMA_DIAG", "RMA_RCCL_LIB", "RMA_EXEC_FUSED", "RMA_EXEC_FUSED_TIMEOUT")}
    diag_entries()  # an unknown RMA_DIAG key fails the run here, before any work
    if gpu and diag_value("pipe_fast") == "pipe5":  # an A/B of the lab kernel
        from rocm_mpi_amd._native import load_lab

        load_lab()
    check_on = a.check == 1 or (a.check < 0 and (gpu or world > 1))
    if check_on and diag_flag("skip_exchange"):
        log(rank, "RMA_DIAG=skip_exchange skips every halo exchange: refused with the halo "
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
                      "scaling_point": (not shared) if world > 1 and gpu else None,
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
            # the halo messages of the timed tile: K-wide x- and y-planes
            nx_est = a.nx or (auto_tile(a.hbm_frac, a.max_tile) if gpu else 130)
            ny_est = a.ny or nx_est
            sizes = ({"latency_8B": 8, "x_plane": K * ny_est * 8, "y_plane": K * nx_est * 8}
                     if a.link_probe else None)
            out["config"]["preflight"] = preflight(dims[:2], K, dev, world, rank, gpu,
                                                   max(130, 6 * K + 2), tmo, sizes)
        except CheckFailed as e:
            out["config"]["preflight"] = {"error": str(e.args[0])}
            return fail_run("preflight", e, 5)
        finally:
            wd.cancel()
        lk = out["config"]["preflight"].get("links") or {}
        if gpu and world > 1 and not shared and lk.get("all_p2p") is False:
            # RCCL chose a host path (sockets, shared memory) for a halo connection
            out["config"]["scaling_point"] = False
            out["config"]["non_scaling_reason"] = (
                "RCCL halo connections are not all GPU-direct P2P: " +
                ", ".join(f"rank {r['rank']}: {r['transport']}" for r in lk["ranks"]))
            log(rank, out["config"]["non_scaling_reason"])

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
        init_stats = field_stats_global(model.field, comm) if a.full_field_check else None

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
        # every cell of the timed field, before the side measurements step it further
        ffc = None
        if init_stats is not None:
            try:
                ffc = full_field_check(model.field, init_stats, model.steps_done, comm, world,
                                       rank, tmo)
            except CheckFailed as e:
                out["config"]["full_field_check"] = e.args[1] if len(e.args) > 1 else None
                return fail_run("check", CheckFailed(e.args[0]), 3)
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

                if kern >= 9:  # the cells per lane the kernel runs (vec 5 needs nx % 5 == 0)
                    kvec = native().pipe_vec(depth, 0, kern - 9, nx, kvec, True)
                kinfo = {"kernel": ops.kernel_name(kern), "vec": kvec, "chunk_rows": a.chunk2 or kch,
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
            lk = (out["config"].get("preflight") or {}).get("links") or {}
            verdicts = sorted({r["transport"] for r in lk.get("ranks", [])})
            rccl_desc = ("RCCL send/recv over xGMI (every connection P2P in RCCL's log)"
                         if lk.get("all_p2p") else
                         f"RCCL send/recv (RCCL-logged transport: {', '.join(verdicts)})"
                         if verdicts else "RCCL send/recv")
            tdesc = {"rccl": rccl_desc, "staged": "host-staged copies + gloo",
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
        elif out["config"].get("scaling_point") is False:
            par = f"NOT A SCALING POINT ({out['config']['non_scaling_reason']}); {par}"
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
            "full_field_check": ffc,
        })

        # --- correctness of this run's code paths (bounded; any failure fails all)
        rc = 0
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
