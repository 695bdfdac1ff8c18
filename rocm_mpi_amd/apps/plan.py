"""Show what a run would execute: the pass plan, kernel tuning and predicted
time of ``n`` steps on a local tile (the executor's planner, no GPU needed).

    python -m rocm_mpi_amd.apps.plan --nx 101376 --steps 1000
    python -m rocm_mpi_amd.apps.plan --nx 16384 --steps 20 --temporal 24 --canonical

The predicted time uses the measured one-step kernel time of the tile class
(ms per HBM sweep of the three arrays) and the planner's relative pass costs
(csrc/runtime/plan.cpp, profiles/pass_sweep_*_r2_final.json); box-to-box
spread is a few percent (the deep passes run at the package power cap).
"""
from __future__ import annotations

import argparse
import collections
import json
import sys

# one-step march kernel time per cell on MI355X (24 B/cell at ~6.2 TB/s):
# the planner's cost unit, scaled by the tile's cell count
_MS_PER_CELL = 39.6 / (101376.0 * 101376.0)


def describe(nx: int, ny: int, steps: int, temporal: int = 24, fast_math: bool = True) -> dict:
    from .. import ops
    from .._native import native

    N = native()
    cells = float(nx) * float(ny)
    costs = list(N.default_pass_costs(temporal, fast_math, cells))
    plan = list(N.plan_passes(int(steps), costs))
    unit_ms = _MS_PER_CELL * cells
    kernels = {}
    for K in sorted(set(plan)):
        if fast_math:
            kern, vec, ch = N.fast_kernel_k(K, ny, (-1.0, 1.0, 1.0, 0.1))
        elif K == 1:
            kern, vec, ch = 0, 2, N.default_chunk_k(1, ny)
        else:
            kern, vec, ch = N.canonical_kernel_k(K, ny)
        kernels[K] = {"kernel": ops.kernel_name(kern), "vec": vec, "chunk_rows": ch,
                      "stages": N.pipe_default_stages(K) if kern >= 9 else None,
                      "rel_cost": round(costs[K], 3), "pred_ms_per_pass": round(costs[K] * unit_ms, 3)}
    pred = sum(costs[K] for K in plan) * unit_ms
    a_eff = 3 * cells * 8 / 1e9
    return {"tile": [nx, ny], "steps": steps, "max_steps_per_pass": temporal,
            "arithmetic": "fast-math" if fast_math else "canonical",
            "passes": dict(collections.Counter(plan)), "n_passes": len(plan),
            "kernels": kernels, "pred_ms": round(pred, 3),
            "pred_ms_per_step": round(pred / max(steps, 1), 5),
            "pred_teff_GBps": round(a_eff / (pred / max(steps, 1) / 1e3), 1) if steps else None}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--nx", type=int, required=True, help="local tile x size (halo incl.)")
    ap.add_argument("--ny", type=int, default=0)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--temporal", type=int, default=24, help="max steps per pass (1..24)")
    ap.add_argument("--canonical", action="store_true", help="the bitwise-canonical arithmetic")
    a = ap.parse_args(argv)
    if not 1 <= a.temporal <= 24 or a.nx < 3 or a.steps < 0:
        ap.error("need 1 <= --temporal <= 24, --nx >= 3, --steps >= 0")
    d = describe(a.nx, a.ny or a.nx, a.steps, a.temporal, not a.canonical)
    print(json.dumps(d, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
