"""Diagnosis: repeat the one-step perf_hide loopback cases that mismatched
intermittently (2x1 vs golden, 2x2 periodic perf_hide vs perf) in ONE process
and count mismatches; run under RMA_DIAG frame_sides / no_halo_batch variants."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import golden  # noqa: E402
from helpers import run_loopback  # noqa: E402
from test_multirank_gpu import spmd  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
bad = {"2x1_golden": 0, "2x2_periodic": 0, "4x2_golden": 0}
G21 = None
for i in range(reps):
    Tv, (nxg, nyg, _) = run_loopback(2, spmd, "perf_hide", 200, 100, 8, (2, 1), timeout=60)[0]
    if G21 is None:
        G21 = golden.run(nxg, nyg, 8)[1:-1, 1:-1]
    bad["2x1_golden"] += int(not np.array_equal(Tv, G21))
    a = run_loopback(4, spmd, "perf_hide", 200, 100, 30, (2, 2), periods=(1, 1, 0),
                     init="random")[0][0]
    b = run_loopback(4, spmd, "perf", 200, 100, 30, (2, 2), periods=(1, 1, 0),
                     init="random")[0][0]
    if not np.array_equal(a, b):
        bad["2x2_periodic"] += 1
        d = np.argwhere(a != b)
        print("2x2 mismatch cells", len(d), "first", d[:3].tolist(), "last", d[-3:].tolist(),
              flush=True)
    Tv, (nxg, nyg, _) = run_loopback(8, spmd, "perf_hide", 100, 68, 11, (4, 2), timeout=60)[0]
    bad["4x2_golden"] += int(not np.array_equal(Tv, golden.run(nxg, nyg, 11)[1:-1, 1:-1]))
print(json.dumps({"reps": reps, "mismatches": bad,
                  "env": {"RMA_DIAG": os.environ.get("RMA_DIAG")}}),
      flush=True)
