#!/bin/bash
# r2: x-neighbour pass cost with the exchange skipped (geometry kept; diagnosis only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6n
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -4 | tr '\n' ' '; echo
  return $rc
}
RMA_DIAG_SKIP_EXCHANGE=1 step x_skip 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --variants perf --self-copies --init gaussian --out $OUT/x_skip.json &&
step x_ref 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --variants perf --self-copies --init gaussian --out $OUT/x_ref.json &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
