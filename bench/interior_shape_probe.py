"""Pass time of the K-step interior launch vs the rect it covers (288 GB tile):
the owned rect of an open tile, of one with x / y / x+y neighbours, and the
interior left by the frame strips, to see whether the rect's origin or
extent (not the concurrent frame + exchange) makes a rank with neighbours
slower.

    python bench/interior_shape_probe.py --K 24 --out gpurun_out/shape.json
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocm_mpi_amd import ops  # noqa: E402
from rocm_mpi_amd._native import native  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--n", type=int, default=0)
    ap.add_argument("--K", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--init", default="random", choices=["random", "gaussian"])
    ap.add_argument("--coef", default="probe", choices=["probe", "physics"],
                    help="physics: the run's coefficients (lx = 10, dt = dx^2/4.1)")
    ap.add_argument("--alternate", type=int, default=0,
                    help="P > 0: per rect, P passes alternating T <-> T2 (the executor's "
                         "buffer sequence on an evolving field), timed one by one")
    ap.add_argument("--rects", default="", help="comma list of rect names (default: all)")
    ap.add_argument("--nosync", action="store_true",
                    help="with --alternate: enqueue the P passes back to back (events only)")
    ap.add_argument("--stream", default="default", choices=["default", "low", "high"],
                    help="run the passes on a new stream of this priority (the executor's "
                         "interior runs on a low-priority stream)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    n = a.n
    if not n:
        free, _ = torch.cuda.mem_get_info()
        n = int(math.isqrt(int(0.8 * free / 24))) // 256 * 256
    K = a.K
    T = torch.empty((n, n), dtype=torch.float64, device="cuda")
    T2 = torch.empty_like(T)
    iCp = torch.empty_like(T)
    geom = ops.TileGeometry(0, 0, n, n, 1.0, 1.0)
    def init(A):
        if a.init == "random":
            ops.init_random_(A, geom, seed=1)
        else:
            ops.init_gaussian_(A, geom, 10.0, 10.0)

    init(T)
    ops.fill_(iCp, 1.0)
    ops.fill_(T2, 0.0)
    coef = ops.StencilCoef(-1.0, 1.0 / 0.01, 1.0 / 0.01, 1e-5)
    if a.coef == "physics":
        dx = 10.0 / n
        coef = ops.StencilCoef.from_physics(1.0, dx, dx, dx * dx / 4.1)
    kern, vec, ch = native().fast_kernel_k(K, n, tuple(coef))
    tn = ops.StencilTuning(chunk_rows=ch, kernel=ops.kernel_name(kern), vec=vec, xcd_remap=1)
    f = 128 - 2 * K + K  # interior start next to an ol-wide frame strip (frame fill)
    rects = {
        "open": (1, n - 1, 1, n - 1),
        "owned_x": (K, n - K, 1, n - 1),
        "owned_y": (1, n - 1, K, n - K),
        "owned_xy": (K, n - K, K, n - K),
        "interior_x_strips": (f, n - f, 1, n - 1),
        "interior_y_strips": (1, n - 1, 2 * K, n - 2 * K),
        "interior_xy_strips": (f, n - f, 2 * K, n - 2 * K),
        "open_shift_x8": (9, n - 1, 1, n - 1),
        "owned_x_origin_only": (K, n - 1, 1, n - 1),
        "owned_x_far_only": (1, n - K, 1, n - 1),
        "owned_x_split_y24": [(K, n - K, 1, K), (K, n - K, K, n - 1)],
        "owned_y_split_x24": [(1, K, K, n - K), (K, n - 1, K, n - K)],
        # r3 interior rects of the aligned layouts (K = 24, vec 4: strip 208 columns)
        "al_x": (K + 208, n - K - 208, 1, n - 1),
        "band_y": (1, n - 1, 2 * K, n - 2 * K),
        "hyb_xy": (K + 208, n - K - 208, 2 * K, n - 2 * K),
        "al1536_xy": (K + 208, n - K - 208, K + 1536, n - K - 1536),
        "hyb_xy_rowphase": (K + 208, n - K - 208, 1 + 3072, n - 1 - 3072),
    }
    if a.rects:
        rects = {k: rects[k] for k in a.rects.split(",")}
    res = {"n": n, "K": K, "init": a.init, "kernel": names[kern], "vec": vec, "chunk_rows": ch,
           "coef": a.coef, "alternate": a.alternate, "ms": {}}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    stream = torch.cuda.current_stream()
    if a.stream != "default":  # torch: lower number = higher priority
        lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") \
            else (0, -1)
        stream = torch.cuda.Stream(priority=lo if a.stream == "low" else hi)
    res["stream"] = a.stream
    res["nosync"] = a.nosync
    if a.alternate:
        # every rect starts from the same random field; passes alternate the
        # buffers like the executor (halo cells keep their values: no exchange)
        for rep in range(a.reps):
            for name, r in rects.items():
                rl = r if isinstance(r, list) else [r]
                init(T)  # no room for a saved copy at the 288 GB tile
                T2.copy_(T)
                src, dst = T, T2
                torch.cuda.synchronize()
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(a.alternate)]
                with torch.cuda.stream(stream):
                    for e0, e1 in evs:
                        if not a.nosync:
                            torch.cuda.synchronize()
                        e0.record()
                        ops.stencilk_step(K, dst, src, iCp, coef, rl, tn)
                        e1.record()
                        src, dst = dst, src
                torch.cuda.synchronize()
                ts = [round(e0.elapsed_time(e1), 3) for e0, e1 in evs]
                res["ms"].setdefault(name, []).append(ts)
                print(json.dumps({name: ts}), flush=True)
        if a.out:
            with open(a.out, "w") as fo:
                json.dump(res, fo, indent=1)
        return 0
    for rep in range(a.reps):
        for name, r in rects.items():
            rl = r if isinstance(r, list) else [r]
            ops.stencilk_step(K, T2, T, iCp, coef, rl, tn)
            torch.cuda.synchronize()
            ev[0].record()
            ops.stencilk_step(K, T2, T, iCp, coef, rl, tn)
            ev[1].record()
            torch.cuda.synchronize()
            res["ms"].setdefault(name, []).append(round(ev[0].elapsed_time(ev[1]), 3))
        print(json.dumps(res["ms"]), flush=True)
    if a.out:
        with open(a.out, "w") as fo:
            json.dump(res, fo, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
