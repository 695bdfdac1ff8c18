"""Halo pack / unpack time: both x-planes of a tile as two launches
(``copy_plane`` each) vs one batched launch (``copy_planes``, what the halo
engine issues per dimension since r2), for width-K fp64 planes.

    python bench/pack_time.py --n 16384 --K 1,24 --out gpurun_out/pack.json

Times are device time per exchange phase (HIP events over ``--reps``
back-to-back repetitions; the planes stay cache-resident between repetitions,
as they are after the frame kernel wrote them) and host enqueue time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from rocm_mpi_amd import ops  # noqa: E402


def timed(fn, reps: int) -> tuple[float, float]:
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    h0 = time.perf_counter()
    for _ in range(reps):
        fn()
    h1 = time.perf_counter()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3, (h1 - h0) / reps * 1e6  # device us, host us


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--K", default="1,24")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    n = a.n
    T = torch.empty((n, n), dtype=torch.float64, device="cuda")
    ops.fill_(T, 1.0)
    rows = []
    for K in (int(k) for k in a.K.split(",")):
        bl = torch.empty((n, K), dtype=torch.float64, device="cuda")
        bh = torch.empty_like(bl)
        lo, hi = T[:, K:2 * K], T[:, n - 2 * K:n - K]
        hl, hh = T[:, :K], T[:, n - K:]

        def pack2():
            ops.copy_plane(bl, lo)
            ops.copy_plane(bh, hi)

        def unpack2():
            ops.copy_plane(hl, bh)
            ops.copy_plane(hh, bl)

        r = {"n": n, "K": K, "plane_MB": n * K * 8 / 1e6}
        for name, fn in (("pack_2_launches", pack2),
                         ("pack_batched", lambda: ops.copy_planes([(bl, lo), (bh, hi)])),
                         ("unpack_2_launches", unpack2),
                         ("unpack_batched", lambda: ops.copy_planes([(hl, bh), (hh, bl)]))):
            dev_us, host_us = timed(fn, a.reps)
            r[name + "_us"] = round(dev_us, 2)
            r[name + "_host_us"] = round(host_us, 2)
        r["pack_GBps_batched"] = round(2 * 2 * n * K * 8 / (r["pack_batched_us"] * 1e3), 1)
        rows.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(), "rows": rows}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
