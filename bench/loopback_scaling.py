"""Halo-exchange overhead on ONE GPU: N logical ranks (threads) share the card.

The real weak-scaling run needs N GPUs (the driver's 8-GPU `bench.py` pass).
This emulation measures what the distributed path costs on top of the compute:
N ranks run the native executor (frame on a high-priority stream, halo
exchange through the device loopback transport = D2D copies with RCCL's
completion semantics, interior on a low-priority stream) on N tiles of the
same size, concurrently on one GPU. Aggregate T_eff(N) / T_eff(1) is then the
fraction of the single-rank throughput that survives the extra frames,
pack/unpack kernels, copies and cross-stream synchronisation (1.0 = fully
hidden). Transport latency across xGMI is not part of it.

    python bench/loopback_scaling.py --n 8192 --ranks 1,2,4 --temporal 1,8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(N: int, n: int, K: int, steps: int, variant: str, fast: bool = False) -> dict:
    import torch

    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg
    from rocm_mpi_amd.parallel.comm import LoopbackHub

    hub = LoopbackHub(N, timeout_s=300)
    out = [None] * N
    err = []
    go = threading.Barrier(N)

    def body(r):
        try:
            ol = 2 * K
            gg.init_global_grid(n, n, 1, overlaps=(ol, ol, 2), halowidths=(K, K, 1), quiet=True,
                                loopback=(hub, r))
            m = Diffusion2D(DiffusionConfig(variant=variant, nx=n, ny=n, nt=steps, quiet=True,
                                            init="random", temporal=K,
                                            fast_math=K > 1 and (fast or K > 8)))
            m.step(2 * K)
            m.synchronize()
            go.wait()
            t0 = time.perf_counter()
            m.step(steps)
            m.synchronize()
            go.wait()
            out[r] = (time.perf_counter() - t0, m.g.dims)
            m.close()
            gg.finalize_global_grid()
        except BaseException as e:  # noqa: BLE001
            err.append((r, repr(e)))
            go.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(N)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if err:
        raise RuntimeError(f"rank failures: {err}")
    wall = max(o[0] for o in out)
    agg = N * 3 * n * n * 8 / 1e9 / (wall / steps)
    torch.cuda.empty_cache()
    return {"ranks": N, "dims": list(out[0][1]), "tile": n, "temporal": K, "steps": steps,
            "fast_math": K > 1 and (fast or K > 8),
            "ms_per_step": wall / steps * 1e3, "aggregate_teff_GBps": agg}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--ranks", default="1,2,4")
    ap.add_argument("--temporal", default="1,8")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--variant", default="perf_hide")
    ap.add_argument("--fast-math", action="store_true",
                    help="fast-math K-step passes (always on for K = 12, 16)")
    ap.add_argument("--out", default="")
    a = ap.parse_args(argv)
    rows = []
    for K in [int(v) for v in a.temporal.split(",")]:
        base = None
        for N in [int(v) for v in a.ranks.split(",")]:
            r = run(N, a.n, K, a.steps, a.variant, a.fast_math)
            base = base or r["aggregate_teff_GBps"]
            r["fraction_of_1_rank"] = r["aggregate_teff_GBps"] / base
            rows.append(r)
            print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
