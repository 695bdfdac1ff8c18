#!/bin/bash
# r2: kernel tests after moving strip planning into the pipe instantiations
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2q
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_pipe_gpu.py tests/test_guard_bands_gpu.py tests/test_temporal_gpu.py tests/test_multirank_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
tail -1 $OUT/bench.log | cut -c1-250
