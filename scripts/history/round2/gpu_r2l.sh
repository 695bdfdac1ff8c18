#!/bin/bash
# r2: mirrored factor ring (one LDS base per stage): bitwise tests, pass sweep, power probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2l
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_pipe_gpu.py tests/test_guard_bands_gpu.py tests/test_temporal_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python -u bench/pass_sweep.py --rounds 3 --pipe 10-24 --pipec 12,13,14,16 --ldsdpp "" --old "" --alt "" --out $OUT/pass_sweep.json > $OUT/sweep.log 2>&1 || exit $?
tail -3 $OUT/sweep.log
timeout -k 10 300 python -u bench/power_probe.py --configs pipe:12,pipe:16,pipe:20,pipe:24 --seconds 6 --out $OUT/power.json > $OUT/power.log 2>&1 || exit $?
tail -1 $OUT/power.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/bench_20_5.json > $OUT/bench_20_5.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --json-out $OUT/bench_default.json > $OUT/bench_default.log 2>&1 || exit $?
tail -1 $OUT/bench_20_5.log | cut -c1-300
tail -1 $OUT/bench_default.log | cut -c1-300
