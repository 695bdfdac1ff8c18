#!/usr/bin/env python
"""Root-cause probe of the executor stream-creation-order effect.

Creates several executors in ONE process, one after the other (the previous
one destroyed) and two alive together, and times the one-step kernel on each
(16384^2, perf_hide without neighbours = one launch per step on the
low-priority stream). Each stream-creation mode runs in its own subprocess:

  lofirst  low-priority stream created first (the executor default)
  hifirst  high-priority first (r1: every second instance ~25 % slower)
  plain    two unprioritised streams
  pool     the executor's process-wide stream pool (streams of destroyed
           executors are reused, created low-priority first)

Run under ``rocprofv3 --kernel-trace`` to see the hardware queue of every
dispatch; the JSON line per mode lists GB/s per instance and the HIP stream
handles the executor reported (RMA_DIAG exec_verbose).

    python bench/probe_stream_order.py --n 16384 --modes lofirst,hifirst,plain,pool
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(n: int, steps: int) -> dict:
    import torch

    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig

    def seg(m):
        m.step(2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m.step(steps)
        torch.cuda.synchronize()
        return round(3 * n * n * 8 / 1e9 / ((time.perf_counter() - t0) / steps))

    seq = []
    for _ in range(4):  # one after the other
        m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=n, ny=n, nt=1, quiet=True,
                                        init="random"))
        seq.append(seg(m))
        m.close()
        del m
    a = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=n, ny=n, nt=1, quiet=True,
                                    init="random"))
    # a second grid cannot be created while a owns the process grid: reuse it
    b = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=n, ny=n, nt=1, quiet=True,
                                    init="random"))
    both = [seg(a), seg(b), seg(a), seg(b)]
    b.close()
    a.close()
    return {"sequential_GBps": seq, "two_alive_GBps": both}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--modes", default="lofirst,hifirst,plain,pool")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args(argv)
    if a.child:
        print("RESULT " + json.dumps(child(a.n, a.steps)), flush=True)
        return 0
    out = {}
    for mode in a.modes.split(","):
        env = dict(os.environ, RMA_DIAG=f"exec_streams={mode},exec_verbose")
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--n",
                            str(a.n), "--steps", str(a.steps)], capture_output=True, text=True,
                           env=env, timeout=600)
        res = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
        streams = [ln for ln in r.stderr.splitlines() if ln.startswith("[executor]")]
        out[mode] = json.loads(res[0][7:]) if res else {"error": r.stderr[-800:]}
        out[mode]["streams"] = streams
        print(json.dumps({mode: out[mode]}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
