#!/usr/bin/env python
"""Headline benchmark: T_eff (GB/s) of 2D diffusion on 1..8 MI355X, weak scaling.

BASELINE.json metric: "T_eff (GB/s) + weak-scaling eff., 2D diffusion 1000 steps
at 1/2/4/8 MI355X"; flagship config "diffusion_2D_perf_hide ... per-GPU tile
sized to 288 GB HBM". One process per GPU (torch.distributed.run), halo
exchange GPU-direct over RCCL/xGMI overlapped with the interior kernel.

    python bench.py                                   # 1 GPU, 1000 steps, 10 warmup
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29600 bench.py --gpus 8

T_eff per GPU follows the reference exactly (scripts/diffusion_2D_perf.jl:55-58):
A_eff = 3*nx*ny*8 B per step on the LOCAL tile (halo included), divided by the
time per step. W warmup steps run untimed (the reference skips 10); K steps
are timed between barrier+device-sync pairs; the step time is the MAX over
ranks; ``value`` is the whole-job aggregate = N x per-GPU T_eff (weak scaling:
the local tile is the same for every N). Data: synthetic random-init field.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

_TRANSPORT_DESC = {"rccl": "RCCL send/recv over xGMI", "staged": "host-staged copies + gloo",
                   "self": "single rank, no exchange", "gloo": "gloo (CPU twin)",
                   "loopback": "in-process loopback"}

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
    ap.add_argument("--temporal", type=int, default=16, choices=[1, 2, 3, 4, 6, 8, 12, 16],
                    help="K: K time steps per kernel pass (register temporal blocking), "
                         "width-K halo exchange per pass, grid overlap 2K (12, 16: fast-math)")
    ap.add_argument("--chunk2", type=int, default=0,
                    help="K-step kernel rows per wave-task (0: auto, models.diffusion.default_chunk2)")
    ap.add_argument("--unroll2", type=int, default=2, choices=[2, 4])
    ap.add_argument("--fast-math", dest="fast_math", action="store_true", default=True,
                    help="K-step passes with fast-math fp64 arithmetic (5-point sum, one folded "
                         "per-cell factor, FMAs): same scheme, not bitwise equal to the "
                         "canonical update (default; the bitwise K-step (K <= 8) and one-step "
                         "kernels are timed too)")
    ap.add_argument("--no-fast-math", dest="fast_math", action="store_false")
    ap.add_argument("--overlap", type=int, default=0,
                    help="grid overlap (0: 2 x steps-per-pass, the minimum)")
    ap.add_argument("--single-step-steps", type=int, default=100,
                    help="after the timed run, also time this many steps of the one-step "
                         "kernel on the same tile (reported in config; 0 = skip)")
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
    if world != a.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}", file=sys.stderr)
        return 2

    import torch

    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import comm as C
    from rocm_mpi_amd.parallel import implicit_grid as gg

    gpu = a.device == "cuda"
    if gpu and not torch.cuda.is_available():
        print("bench.py needs an MI355X (no GPU visible)", file=sys.stderr)
        return 2
    if not gpu and not a.nx:
        print("bench.py --device cpu needs --nx", file=sys.stderr)
        return 2
    if world > 1:
        C.init_distributed(None if gpu else "gloo")
    rank = int(os.environ.get("RANK", "0"))
    local, _ = C.node_local_rank(rank, world)
    dev = str(C.select_device(local)) if gpu else "cpu"

    def sync():
        if gpu:
            torch.cuda.synchronize()

    nx = a.nx or auto_tile(a.hbm_frac, a.max_tile)
    if world > 1 and not a.nx:
        import torch.distributed as dist

        t = torch.tensor([nx], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=C._gloo_group())
        nx = int(t.item())
    ny = a.ny or nx
    dims = tuple(int(v) for v in a.dims.split(",")) + (0,)
    bw = tuple(int(v) for v in a.b_width.split(","))
    cfg = DiffusionConfig(variant=a.variant, nx=nx, ny=ny, nt=a.steps + a.warmup, device=dev,
                          warmup=a.warmup, init="random", b_width=bw, dims=dims,
                          chunk_rows=a.chunk_rows, kernel=a.kernel, nontemporal=a.nontemporal,
                          unroll=a.unroll, vec=a.vec, temporal=a.temporal, chunk2=a.chunk2,
                          unroll2=a.unroll2, use_graph=a.graph, quiet=True,
                          fast_math=a.fast_math and a.temporal > 1)
    t_setup = time.perf_counter()
    gkw = {}
    if a.overlap:
        gkw = {"overlaps": (a.overlap, a.overlap, 2),
               "halowidths": (max(1, a.temporal), max(1, a.temporal), 1)}
    model = Diffusion2D(cfg, grid_kwargs=gkw)
    chunk2_main = model.chunk2
    g = model.g
    comm = g.comm
    model.synchronize()
    comm.barrier()
    setup_s = time.perf_counter() - t_setup

    model.step(a.warmup)
    model.synchronize()
    comm.barrier()
    sync()
    t0 = time.perf_counter()
    model.step(a.steps)
    sync()
    comm.barrier()
    t1 = time.perf_counter()
    local_s = t1 - t0
    wall = comm.allreduce(local_s, "max")
    bad = float(model.field[:: max(1, ny // 64), :: max(1, nx // 64)].isfinite().logical_not().sum())
    bad = comm.allreduce(bad, "sum")

    # secondary: the one-step kernel (24 B/cell/step at the HBM roofline) on the
    # same tile, so the temporal-blocking gain is visible in one record
    def side_teff(K, fast, steps):
        model.set_temporal(K, fast_math=fast)
        model.step(2 * K)
        model.synchronize()
        comm.barrier()
        sync()
        s0 = time.perf_counter()
        model.step(steps)
        sync()
        comm.barrier()
        s1 = comm.allreduce(time.perf_counter() - s0, "max")
        return 3 * nx * ny * 8 / 1e9 / (s1 / steps)

    single = canonical = None
    kc = min(a.temporal, 8)  # the canonical K-step kernels go up to 8 steps per pass
    if a.single_step_steps > 0 and a.temporal > 1:
        if a.fast_math:  # the bitwise-canonical K-step kernel on the same tile
            canonical = side_teff(kc, False, max(kc, a.single_step_steps // kc * kc))
        single = side_teff(1, False, a.single_step_steps)

    kstep = None  # the K-step kernel the executor runs (csrc/runtime/executor.cpp fast_tune_k)
    if a.temporal > 1:
        from rocm_mpi_amd import ops
        from rocm_mpi_amd._native import native

        if a.fast_math and gpu:
            kern, kvec, _ = native().fast_kernel_k(a.temporal, ny, tuple(model.coef))
            kstep = {"kernel": {v: k for k, v in ops.KERNELS.items()}[kern], "vec": kvec,
                     "chunk_rows": chunk2_main}
        else:
            kstep = {"kernel": "canonical", "chunk_rows": chunk2_main}

    t_it = wall / a.steps
    teff_gpu = 3 * nx * ny * 8 / 1e9 / t_it
    total = teff_gpu * world
    out = {
        "metric": METRIC,
        "value": round(total, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(t_it * 1e3, 6),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp64",
        "data": "synthetic: counter-based uniform [0,1) random-init temperature field",
        "config": {
            "model": f"diffusion_2D_{a.variant}",
            "global_batch": g.nxyz_g[0] * g.nxyz_g[1],
            "seq_len": None,
            "parallelism": f"2D domain decomposition dims {g.dims[0]}x{g.dims[1]} "
                           f"(halo: {_TRANSPORT_DESC.get(g.transport, g.transport)}"
                           + (", boundary/interior overlap)" if a.variant == "perf_hide" else ")"),
            "local_grid": [nx, ny],
            "global_grid": [g.nxyz_g[0], g.nxyz_g[1]],
            "teff_per_gpu_GBps": round(teff_gpu, 2),
            "a_eff_GB_per_step": round(3 * nx * ny * 8 / 1e9, 6),
            "kernel": a.kernel,
            "kstep_kernel": kstep,
            "chunk_rows": a.chunk_rows,
            "unroll": a.unroll,
            "vec": a.vec,
            "nontemporal": a.nontemporal,
            "b_width": list(bw),
            "hipgraph": bool(a.graph),
            "temporal_blocking": a.temporal,
            "chunk2": chunk2_main,
            "steps_per_kernel_pass": a.temporal,
            "teff_note": ("T_eff = A_eff/t_step with A_eff = 3*nx*ny*8 B (reference "
                          "perf.jl:55-58). With temporal blocking every step of every cell "
                          "is still computed (bitwise equal to one-step updates) but HBM is "
                          f"read/written once per {a.temporal} steps, so T_eff exceeds the "
                          "HBM bandwidth; teff_single_step_kernel_GBps is the one-step "
                          "kernel on the same tile. fast_math: the K-step passes evaluate "
                          "the same fp64 update as a 5-point sum with one folded per-cell "
                          "factor and FMAs (rounding-level deviation from the canonical "
                          "update, tests/test_temporal_gpu.py); teff_bitwise_kstep_GBps is "
                          "the bitwise-canonical K-step kernel on the same tile")
                         if a.temporal > 1 else "",
            "teff_single_step_kernel_GBps": round(single, 2) if single else None,
            "fast_math": bool(a.fast_math and a.temporal > 1),
            "teff_bitwise_kstep_GBps": round(canonical, 2) if canonical else None,
            "bitwise_kstep_steps_per_pass": kc if canonical else None,
            "overlap": list(g.overlaps[:2]),
            "setup_s": round(setup_s, 3),
            "nonfinite_cells_sampled": int(bad),
        },
    }
    if g.me == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    model.close()
    if world > 1:
        C.shutdown_distributed()
    return 0 if bad == 0 else 3


if __name__ == "__main__":
    sys.exit(main())
