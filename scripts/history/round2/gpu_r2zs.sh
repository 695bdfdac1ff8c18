#!/bin/bash
# r2: single-stream passes when there is no frame (no cross-queue round trip per pass)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zs
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_executor_gpu.py tests/test_multirank_gpu.py tests/test_temporal_gpu.py tests/test_bench_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for n in 2048 4096 8192 16384; do
  timeout -k 10 200 python -u bench.py --nx $n --steps 1000 --warmup 48 --single-step-steps 20 --json-out $OUT/b_$n.json > $OUT/b_$n.log 2>&1 || exit 1
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/b_20_5.json > $OUT/b_20_5.log 2>&1 || exit 1
python - <<'PY'
import json
for n in ("2048", "4096", "8192", "16384", "20_5"):
    d = json.load(open(f"gpurun_out/r2zs/b_{n}.json"))
    print(n, d["value"], d["ms_per_step"], d["config"]["teff_single_step_kernel_GBps"])
PY
