#!/bin/bash
# r2 session: any-K pipelined kernel correctness + per-depth pass sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2b
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_pipe_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_pipe.log 2>&1; rc=$?
echo "== pytest_pipe rc=$rc"; tail -3 $OUT/pytest_pipe.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench/pass_sweep.py --out $OUT/pass_sweep_101k.json > $OUT/pass_sweep.log 2>&1; rc=$?
echo "== sweep rc=$rc"; tail -3 $OUT/pass_sweep.log
exit $rc
