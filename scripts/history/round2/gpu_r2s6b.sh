#!/bin/bash
# r2: batched halo pack/unpack (one launch per dimension phase): GPU suite, pack timing,
# RCCL-self one-step overhead at 16384^2 (compare rccl_self_16k_k1_r2.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6b
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-300
  return $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step pack_16k 120 python -u bench/pack_time.py --n 16384 --K 1,8,24 --out $OUT/pack_16384.json &&
step pack_101k 180 python -u bench/pack_time.py --n 101376 --K 16,24 --reps 50 --out $OUT/pack_101376.json &&
step rccl_self_16k 600 python -u bench/rccl_self_overhead.py --n 16384 --K 1 --variants perf,perf_hide --steps 400 --out $OUT/rccl_self_16k_k1.json
