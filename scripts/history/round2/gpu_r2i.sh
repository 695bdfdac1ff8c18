#!/bin/bash
# r2: mixed-depth multi-rank loopback tests, full GPU suite, C++ example (no Python)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2i
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300
  return $rc
}
step pytest_mr 600 python -u -m pytest tests/test_multirank_gpu.py -x -q -k "planned or pass_timing" --timeout 200 --timeout-method thread -p no:cacheprovider &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 200 --timeout-method thread -p no:cacheprovider &&
step example_k24 300 ./build/examples/diffusion_2D_perf_hide 16384 1010 1 24 1 &&
step example_k1 300 ./build/examples/diffusion_2D_perf_hide 16384 1010 1 1 0
