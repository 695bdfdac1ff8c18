#!/usr/bin/env python
"""Per-pass timeline of frame-first fused passes from a rocprofv3 kernel trace
(``--kernel-trace -d DIR -o run``; ``scripts/gpu_steps.sh trace_fused``): for
each large pipelined launch, when (after its start) the exchange stream's
frame-flag wait ended, when the pack / RCCL / unpack kernels of that pass ran,
and when the launch itself ended -- i.e. how much of the launch the exchange
overlapped.

    python scripts/fused_timeline.py gpurun_out/tf/trace_fused/run_results.db --last 6
"""
from __future__ import annotations

import argparse
import sqlite3


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0].split("::")[-1][:22]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=6)
    ap.add_argument("--min-grid", type=int, default=200, help="workgroups of a pass launch")
    a = ap.parse_args(argv)
    cur = sqlite3.connect(a.db).cursor()
    rows = list(cur.execute("select name, start, end, grid_x / max(workgroup_x, 1), queue_id "
                            "from kernels order by start"))
    passes = [r for r in rows if "pipe_kernel" in r[0] and r[3] >= a.min_grid]
    out = ["| pass | launch us | flag wait ends at us | exchange kernels (start-end us) | "
           "exchange done at us | exposed us |", "|---|---|---|---|---|---|"]
    for k, (name, s0, e0, grid, q) in enumerate(passes[-a.last:]):
        nxt = passes[passes.index((name, s0, e0, grid, q)) + 1][1] if \
            passes.index((name, s0, e0, grid, q)) + 1 < len(passes) else None
        win = [r for r in rows if r[1] >= s0 and (nxt is None or r[1] < nxt) and r[0] != name]
        # this pass's wait was enqueued after the previous exchange: it ENDS in the launch
        wait = sorted((r for r in rows if "flag_wait" in r[0] and s0 <= r[2] <= e0),
                      key=lambda r: r[2])
        ex = [r for r in win if "flag" not in r[0]]
        done = max((r[2] for r in ex), default=None)
        desc = ", ".join(f"{short(r[0])} "
                         f"{(r[1] - s0) / 1e3:.0f}-{(r[2] - s0) / 1e3:.0f}" for r in ex)
        out.append(f"| {k} | {(e0 - s0) / 1e3:.0f} | "
                   f"{(wait[0][2] - s0) / 1e3:.0f} | {desc} | "
                   f"{(done - s0) / 1e3:.0f} | {max(0.0, (done - e0) / 1e3):.0f} |"
                   if wait and done else f"| {k} | {(e0 - s0) / 1e3:.0f} | - | {desc} | - | - |")
    print("\n".join(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
