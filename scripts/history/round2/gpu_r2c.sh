#!/bin/bash
# r2 session: pipe tests with the 1/2/4-stage defaults, pass sweep with chunk
# variants, then the whole GPU suite (stops at the first GPU step that fails)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2c
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_pipe_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_pipe.log 2>&1; rc=$?
echo "== pytest_pipe rc=$rc"; tail -3 $OUT/pytest_pipe.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u bench/pass_sweep.py --pipec 3-12,16,20,24 --chunks 16:1024/2048,20:1024/2048/3072,24:1024/2048/3072 --out $OUT/pass_sweep_101k.json > $OUT/pass_sweep.log 2>&1; rc=$?
echo "== sweep rc=$rc"; tail -2 $OUT/pass_sweep.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 30 --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "== pytest_gpu rc=$rc"; tail -40 $OUT/pytest_gpu.log | grep -E "FAILED|ERROR|passed|failed"
exit 0
