#!/bin/bash
# bench.py at 16384^2 (K=16): new default chunk (1024) vs the old one (256), twice each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=${OUT:-gpurun_out/b16k}
mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 200 python bench.py --nx 16384 --single-step-steps 0 --json-out "$OUT/new$i.json" > "$OUT/new$i.log" 2>&1 &&
  timeout -k 10 200 python bench.py --nx 16384 --single-step-steps 0 --chunk2 256 --json-out "$OUT/old$i.json" > "$OUT/old$i.log" 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_executor_gpu.py tests/test_temporal_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 && tail -1 "$OUT/tests.log"
