#!/bin/bash
# fast5 K-step kernel: correctness (tests) then A/B sweep against kernel 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=gpurun_out/fast5; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_temporal_gpu.py tests/test_guard_bands_gpu.py -k "fast or stay_in_bounds" > $OUT/tests.log 2>&1 &&
echo "tests ok" && tail -2 $OUT/tests.log &&
timeout -k 10 300 python bench/stencil_sweep.py --n 16384 --rounds 3 --iters 4 --no-march --no-roof \
    --tbk 6,8 --tbk-chunks 128 --tbk-xcds 1 --tbk-vecs 2,4 --tbk-kernels fast,fast5,fast5o4 \
    --out $OUT/sweep16k.json > $OUT/sweep16k.log 2>&1 &&
echo "sweep16k ok" &&
timeout -k 10 400 python bench/stencil_sweep.py --n 101376 --rounds 3 --iters 2 --no-march --no-roof \
    --tbk 6,8 --tbk-chunks 1024 --tbk-xcds 1 --tbk-vecs 2,4 --tbk-kernels fast,fast5,fast5o4 \
    --out $OUT/sweep101k.json > $OUT/sweep101k.log 2>&1 &&
echo "sweep101k ok"
