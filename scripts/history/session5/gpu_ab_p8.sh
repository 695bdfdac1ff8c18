#!/bin/bash
# fast5p8 (8 pipelined stages of 2 levels, 4 waves/SIMD) vs fast5p4 at K=16:
# bitwise GPU tests, then an interleaved sweep at 16384^2 and 101376^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=${OUT:-gpurun_out/ab_p8}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_temporal_gpu.py tests/test_guard_bands_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fast5 or bounds" > "$OUT/tests.log" 2>&1 &&
tail -1 "$OUT/tests.log" &&
timeout -k 10 300 python bench/stencil_sweep.py --n 16384 --rounds 3 --iters 4 --no-roof --no-march --tbk 16 --tbk-chunks 256,1024 --tbk-xcds 1 --tbk-vecs 4 --tbk-kernels fast5p4,fast5p8 --out "$OUT/sweep_16k.json" > "$OUT/sweep_16k.log" 2>&1 &&
timeout -k 10 500 python bench/stencil_sweep.py --n 101376 --rounds 3 --iters 2 --no-roof --no-march --tbk 16 --tbk-chunks 1024,1536 --tbk-xcds 1 --tbk-vecs 4 --tbk-kernels fast5p4,fast5p8 --out "$OUT/sweep_101k.json" > "$OUT/sweep_101k.log" 2>&1 &&
echo sweeps ok
