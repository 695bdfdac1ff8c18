#!/bin/bash
# two-row prefetch in every K-step kernel: full GPU tests, canonical K-step sweep, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=gpurun_out/pf2_all; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 &&
echo "tests ok" && tail -1 $OUT/tests.log &&
timeout -k 10 400 python bench/stencil_sweep.py --n 101376 --rounds 3 --iters 2 --no-march --no-roof \
    --tbk 6,8 --tbk-chunks 512,1024 --tbk-xcds 1 --tbk-vecs 2 --tbk-kernels lds_dpp \
    --out $OUT/sweep101k.json > $OUT/sweep101k.log 2>&1 &&
echo "sweep101k ok" &&
timeout -k 10 400 python bench.py --json-out $OUT/bench.json > $OUT/bench.log 2>&1 && echo "bench ok" && tail -1 $OUT/bench.log | cut -c1-400
