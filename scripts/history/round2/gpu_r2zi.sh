#!/bin/bash
# r2: the multi-process bench flow on one GPU (shared-GPU functional test)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zi
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests/test_bench_gpu.py -m gpu -q -x --timeout 650 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
