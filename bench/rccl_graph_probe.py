#!/usr/bin/env python
"""RCCL point-to-point inside hipGraph capture, torch's RCCL vs the system RCCL.

The multi-rank one-step path is host-bound on small tiles: every step enqueues
a frame launch, the pack, one RCCL group and the unpack.
hipGraph replay removes that host cost, but RCCL P2P under capture crashed
with the RCCL 2.26 that torch bundles. This probe runs, each configuration in
its own child process (a crash stays contained, each child has a time limit):

  lib = linked  (the RCCL the core binds to in a torch process: torch's)
  lib = system  (RMA_RCCL_LIB=system: /opt/rocm/lib/librccl.so.1 loaded
                 privately for the native communicators)
  x graph = 0 / 1 (RMA_DIAG=rccl_graph lets the executor capture the exchange)

on one GPU: a periodic perf_hide tile whose four halo planes go through RCCL
send/recv to self, one-step passes (the small-tile regime). A child reports
its RCCL version and library, ms per step, host enqueue ms per step and
whether its field equals the eager run with the linked RCCL (bitwise).

    python bench/rccl_graph_probe.py --n 4096 --steps 400 --out gpurun_out/g.json
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


def child(n: int, steps: int, graph: bool, field_out: str) -> dict:
    import numpy as np
    import torch

    from rocm_mpi_amd._native import native
    from rocm_mpi_amd.models import Diffusion2D, DiffusionConfig
    from rocm_mpi_amd.parallel import implicit_grid as gg

    gg.init_global_grid(n, n, 1, periodx=1, periody=1, quiet=True, transport="rccl",
                        self_via_transport=True)
    m = Diffusion2D(DiffusionConfig(variant="perf_hide", nx=n, ny=n, nt=steps, quiet=True,
                                    init="random", periods=(1, 1, 0), use_graph=graph,
                                    graph_steps=20))
    used_graph = bool(m.use_graph)
    m.step(40)
    m.synchronize()
    t0 = time.perf_counter()
    m.step(steps)
    t_enq = time.perf_counter() - t0
    m.synchronize()
    dt = time.perf_counter() - t0
    np.save(field_out, m.field.cpu().numpy())
    m.close()
    gg.finalize_global_grid()
    return {"rccl_version": native().rccl_version(), "rccl_library": native().rccl_library(),
            "graph": used_graph, "ms_per_step": dt / steps * 1e3,
            "enqueue_ms_per_step": t_enq / steps * 1e3}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--timeout", type=float, default=120)
    ap.add_argument("--configs", default="linked:0,system:0,system:1",
                    help="lib:graph pairs, run in this order (linked:1 segfaulted in round 2 and "
                         "is not run by default); the first failing child ends the probe")
    ap.add_argument("--out", default="")
    ap.add_argument("--child", default="", help=argparse.SUPPRESS)
    a = ap.parse_args(argv)
    if a.child:
        graph, field_out = a.child.split(",", 1)
        print("RESULT " + json.dumps(child(a.n, a.steps, graph == "1", field_out)), flush=True)
        return 0
    import numpy as np

    outdir = os.path.dirname(os.path.abspath(a.out)) if a.out else "/tmp"
    res = {"n": a.n, "steps": a.steps, "runs": []}
    ref = None
    for cfg in a.configs.split(","):
        lib, graph = cfg.split(":")
        env = dict(os.environ, RMA_DIAG="rccl_graph" if graph == "1" else "", RMA_RCCL_BLOCKING="1")
        if lib == "system":
            env["RMA_RCCL_LIB"] = "system"
        else:
            env.pop("RMA_RCCL_LIB", None)
        fo = os.path.join(outdir, f"rccl_graph_{lib}_{graph}.npy")
        cmd = [sys.executable, os.path.abspath(__file__), "--n", str(a.n), "--steps",
               str(a.steps), "--child", f"{graph},{fo}"]
        t0 = time.perf_counter()
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, env=env)
            rc, out, err = r.returncode, r.stdout, r.stderr
        except subprocess.TimeoutExpired as e:
            rc, out, err = "timeout", e.stdout or "", e.stderr or ""
            out = out.decode() if isinstance(out, bytes) else out
            err = err.decode() if isinstance(err, bytes) else err
        row = {"lib": lib, "graph_requested": graph == "1", "rc": rc,
               "seconds": round(time.perf_counter() - t0, 1)}
        line = [ln for ln in out.splitlines() if ln.startswith("RESULT ")]
        if rc == 0 and line:
            row.update(json.loads(line[0][7:]))
            f = np.load(fo)
            if ref is None:
                ref = f
            row["field_equals_first_run"] = bool(np.array_equal(f, ref))
            os.remove(fo)
        else:
            row["stderr_tail"] = err[-1500:]
        res["runs"].append(row)
        print(json.dumps(row), flush=True)
        if rc != 0:  # a crash / timeout is the finding: nothing more on the GPU
            break
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
