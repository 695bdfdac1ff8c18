#!/bin/bash
# r2: x-neighbour pass slowdown at the 288 GB tile: RCCL vs local self copies, x and y
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6i
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"overhead": [-0-9.e]*' "$OUT/$name.log" | tr '\n' ' '; echo
  return $rc
}
step x_copies 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --variants perf,perf_hide --self-copies --out $OUT/x_copies.json &&
step y_copies 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic y --variants perf --self-copies --out $OUT/y_copies.json &&
step y_rccl 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic y --variants perf --out $OUT/y_rccl.json
