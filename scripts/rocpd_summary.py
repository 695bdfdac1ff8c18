#!/usr/bin/env python
"""Markdown summary of a rocprofv3 SQLite database (``rocprofv3 --kernel-trace
--stats -d DIR -o run``): the top kernels, then every dispatch of the kernels
matching --match with its duration, grid, LDS, VGPRs and scratch.

    python scripts/rocpd_summary.py gpurun_out/r3i/prof20/run_results.db --match pipe_kernel
"""
from __future__ import annotations

import argparse
import sqlite3


def short_name(name: str) -> str:
    return name.replace("(anonymous namespace)::", "").split("(")[0]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="pipe_kernel")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--min-ms", type=float, default=1.0, help="dispatches shorter than this are counted, not listed")
    a = ap.parse_args(argv)
    cur = sqlite3.connect(a.db).cursor()
    out = ["| kernel | calls | total ms | mean ms | % |", "|---|---|---|---|---|"]
    for name, calls, tot, avg, pct in cur.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels "
            "order by total_duration desc limit ?", (a.top,)):
        # (top_kernels durations are in microseconds, the kernels table's in nanoseconds)
        out.append(f"| `{short_name(name)}` | {calls} | {tot / 1e3:.3f} | {avg / 1e3:.3f} | {pct:.1f} |")
    out += ["", f"Dispatches of `{a.match}` >= {a.min_ms} ms (in order):", "",
            "| # | kernel | ms | grid (workgroups) | LDS B | scratch |", "|---|---|---|---|---|---|"]
    short = 0
    rows = cur.execute("select name, duration, grid_x, workgroup_x, lds_size, vgpr_count, scratch_size "
                       "from kernels where name like ? order by start", (f"%{a.match}%",))
    for i, (name, dur, gx, wx, lds, vgpr, scr) in enumerate(rows):
        if dur / 1e6 < a.min_ms:
            short += 1
            continue
        out.append(f"| {i} | `{short_name(name)}` | {dur / 1e6:.3f} | {gx // max(wx, 1)} | {lds} | "
                   f"{scr} |")
    out.append(f"\n({short} shorter dispatches not listed)")
    print("\n".join(out))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
