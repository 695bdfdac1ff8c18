#!/bin/bash
# r2: validate the tile-aware planner + deep guard-band tests; driver bench; 16k bench; loopback scaling
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2k
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest ${PYTEST_SEL:-tests} -m gpu -q --maxfail 20 --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/bench_20_5.json > $OUT/bench_20_5.log 2>&1 || exit $?
tail -1 $OUT/bench_20_5.log
timeout -k 10 300 python -u bench.py --json-out $OUT/bench_default.json > $OUT/bench_default.log 2>&1 || exit $?
tail -1 $OUT/bench_default.log
timeout -k 10 300 python -u bench.py --nx 16384 --steps 1000 --warmup 50 --json-out $OUT/bench_16k.json > $OUT/bench_16k.log 2>&1 || exit $?
tail -1 $OUT/bench_16k.log
timeout -k 10 300 python -u bench/loopback_scaling.py --n 16384 --ranks 1,2,4,8 --temporal 1,16,24 --steps 480 --out $OUT/loopback_16k.json > $OUT/loopback.log 2>&1 || exit $?
tail -5 $OUT/loopback.log
