#!/bin/bash
# 8-stage pipelined fast5: tests, sweeps vs fast5p4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=gpurun_out/fast5p8; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_temporal_gpu.py tests/test_guard_bands_gpu.py -k "pipelined or stay_in_bounds" > $OUT/tests.log 2>&1 &&
echo "tests ok" && tail -1 $OUT/tests.log &&
timeout -k 10 300 python bench/stencil_sweep.py --n 16384 --rounds 3 --iters 4 --no-march --no-roof \
    --tbk 16 --tbk-chunks 128,256 --tbk-xcds 1 --tbk-vecs 2,4 --tbk-kernels fast5p4,fast5p8 \
    --out $OUT/sweep16k.json > $OUT/sweep16k.log 2>&1 &&
echo "sweep16k ok" &&
timeout -k 10 500 python bench/stencil_sweep.py --n 101376 --rounds 3 --iters 2 --no-march --no-roof \
    --tbk 8,16 --tbk-chunks 512,1024,2048 --tbk-xcds 1 --tbk-vecs 2,4 --tbk-kernels fast5p4,fast5p8 \
    --out $OUT/sweep101k.json > $OUT/sweep101k.log 2>&1 &&
echo "sweep101k ok"
