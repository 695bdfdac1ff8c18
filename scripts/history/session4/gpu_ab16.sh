#!/bin/bash
# bitwise GPU tests + K=16 fast5p4 pass at 101376^2 + bench.py default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=${OUT:-gpurun_out/ab16}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_temporal_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 &&
tail -1 "$OUT/tests.log" &&
timeout -k 10 400 python bench/stencil_sweep.py --n 101376 --rounds 3 --iters 2 --no-roof --no-march --tbk 16 --tbk-chunks 1536 --tbk-xcds 1 --tbk-vecs 4 --tbk-kernels fast5p4 --out "$OUT/sweep_101k.json" > "$OUT/sweep_101k.log" 2>&1 &&
grep -A3 '"tbk16_c1536' "$OUT/sweep_101k.json" | grep median_ms &&
timeout -k 10 400 python bench.py --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 &&
tail -1 "$OUT/bench.log" | cut -c1-260
