"""Diagnose: one-step throughput over consecutive segments, executor rebuilds."""
import os
import sys
import time

import torch

sys.path.insert(0, ".")
from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"), flush=True)


def seg(m, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.step(steps)
    torch.cuda.synchronize()
    return 3 * n * n * 8 / 1e9 / ((time.perf_counter() - t0) / steps)


for variant in ("perf_hide", "perf"):
    m = Diffusion2D(DiffusionConfig(variant=variant, nx=n, ny=n, nt=1, quiet=True,
                                    init="random"))
    out = []
    for s in (20, 1, 20, 20, 1, 20, 2, 20):
        out.append((s, round(seg(m, s))))
    print(variant, "segments (steps, GB/s):", out, flush=True)
    m.set_temporal(1)
    out = [(s, round(seg(m, s))) for s in (20, 1, 20, 20)]
    print(variant, "after rebuild:", out, flush=True)
    m.close()
