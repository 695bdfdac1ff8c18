#!/usr/bin/env python
"""Multi-rank halo-path overhead with REAL RCCL traffic on one GPU.

RCCL refuses two ranks on one GPU, so the 2-8 GPU weak-scaling run is the
driver's. This probe runs the production configuration on one MI355X twice:
  * open boundaries (no neighbour: one launch per K-step pass), and
  * periodic in x and y with every halo plane routed through RCCL send/recv to
    self (4 neighbours: frame kernel + x-plane pack/unpack + 4 RCCL messages of
    K rows/columns per pass, overlapped with the interior on the low-priority
    stream) -- the message pattern of an interior rank of the 4x2 grid.
The ratio of the two step times bounds what the distributed path costs per
rank (xGMI wire time aside: self messages stay on the GPU).

    python bench/rccl_self_overhead.py [--n 0 (auto: 288 GB tile)] [--steps 320]
    python bench/rccl_self_overhead.py --n 16384 --K 1 --variants perf,perf_hide --steps 400

Also reported per configuration: the host time to ENQUEUE the steps (the
executor's per-step launch + RCCL group overhead, measured as the time until
step() returns) and the per-pass HIP-event split (frame / halo / interior /
exposed halo) of the executor.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(n: int, K: int, steps: int, periodic: bool, variant: str = "perf_hide",
        chunk2: int = 0, dims: str = "xy", via_rccl: bool = True, init: str = "random",
        spacing=None, direct: bool = False) -> dict:
    import torch

    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg

    px = 1 if periodic and "x" in dims else 0
    py = 1 if periodic and "y" in dims else 0
    gg.init_global_grid(n, n, 1, periodx=px, periody=py, quiet=True, transport="rccl",
                        overlaps=(max(2, 2 * K), max(2, 2 * K), 2), halowidths=(K, K, 1),
                        self_via_transport=periodic and via_rccl and not direct)
    m = Diffusion2D(DiffusionConfig(variant=variant, nx=n, ny=n, nt=steps, quiet=True,
                                    init=init, periods=(px, py, 0), temporal=K,
                                    fast_math=K > 1, chunk2=chunk2, spacing=spacing,
                                    halo_direct=periodic and direct))
    m.step(2 * K)
    m.synchronize()
    t0 = time.perf_counter()
    m.step(steps)
    t_enq = time.perf_counter() - t0
    m.synchronize()
    dt = (time.perf_counter() - t0) / steps
    # pass split on a second, shorter run
    m.enable_pass_timing(True)
    m.step(min(steps, 8 * K))
    ts = m.pass_timings()
    m.enable_pass_timing(False)
    m.close()
    gg.finalize_global_grid()
    torch.cuda.empty_cache()
    nps = len(ts)
    split = {k: sum(t[k] for t in ts) / nps for k in ("frame_ms", "halo_ms", "interior_ms",
                                                     "exposed_halo_ms", "pass_ms")} if nps else {}
    return {"ms_per_step": dt * 1e3, "enqueue_ms_per_step": t_enq / steps * 1e3,
            "pass_split_ms": split}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=0, help="tile edge (0: 80%% of free HBM)")
    ap.add_argument("--K", type=int, default=16)
    ap.add_argument("--steps", type=int, default=320)
    ap.add_argument("--variants", default="perf_hide")
    ap.add_argument("--chunk2", type=int, default=0, help="rows per task of the K-step passes (0: table)")
    ap.add_argument("--periodic", default="xy", choices=["xy", "x", "y"],
                    help="dimensions routed through RCCL-self in the periodic runs (x: the "
                         "two x-neighbours of a middle rank of a 4x1 row, no y-neighbour)")
    ap.add_argument("--self-copies", action="store_true",
                    help="periodic halos by local copies instead of RCCL send/recv to self "
                         "(separates the exchange transport from the geometry)")
    ap.add_argument("--init", default="random", choices=["random", "gaussian"])
    ap.add_argument("--pattern", default="opop",
                    help="run order: o = open boundaries, p = periodic (each run allocates "
                         "its own tile), d = periodic with direct-store halos (the pass's "
                         "kernel stores the periodic images itself, no exchange)")
    ap.add_argument("--spacing", default="grid", choices=["grid", "equal", "anisotropic"],
                    help="grid: dx = 10/nx_g, dy = 10/ny_g of each run (a periodic dim has "
                         "nx_g = n - 2K, so dx != dy and the coefficients differ from the open "
                         "run's); equal: dx = dy = 10/n in every run (same coefficients, the "
                         "halo path alone); anisotropic: dx = 10/(n - 2K), dy = 10/n in every "
                         "run (the x-periodic coefficients everywhere)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    import torch

    n = a.n
    if not n:
        free, _ = torch.cuda.mem_get_info()
        n = int(math.isqrt(int(0.8 * free / 24))) // 256 * 256
    spacing = {"grid": None, "equal": (10.0 / n, 10.0 / n),
               "anisotropic": (10.0 / (n - 2 * a.K), 10.0 / n)}[a.spacing]
    out = {"tile": n, "K": a.K, "steps": a.steps, "periodic_dims": a.periodic,
           "spacing": a.spacing,
           "periodic_via": "local copies" if a.self_copies else "rccl self send/recv",
           "init": a.init,
           "frame_sides": os.environ.get("RMA_DIAG", "") or "neighbours", "variants": {}}
    for variant in a.variants.split(","):
        rows = []
        for c in a.pattern:
            periodic, direct = c in "pd", c == "d"
            r = run(n, a.K, a.steps, periodic, variant, a.chunk2, a.periodic, not a.self_copies,
                    a.init, spacing, direct)
            r.update({"periodic_rccl_self": periodic and not direct, "periodic_direct": direct,
                      "teff_GBps": 3 * n * n * 8 / 1e9 / (r["ms_per_step"] / 1e3)})
            rows.append(r)
            print(json.dumps({"variant": variant, **r}), flush=True)
        op = [r["ms_per_step"] for r in rows if not r["periodic_rccl_self"] and not r["periodic_direct"]]
        pe = [r["ms_per_step"] for r in rows if r["periodic_rccl_self"]]
        pd = [r["ms_per_step"] for r in rows if r["periodic_direct"]]
        out["variants"][variant] = {
            "runs": rows, "overhead": min(pe) / min(op) - 1.0 if pe and op else None,
            "overhead_direct": min(pd) / min(op) - 1.0 if pd and op else None}
    print(json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
