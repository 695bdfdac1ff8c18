#!/bin/bash
# r2: x-neighbour pass slowdown vs rows per task (perf, local copies, smooth field)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6o
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -4 | tr '\n' ' '; echo
  return $rc
}
step x_c1536 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --variants perf --self-copies --init gaussian --chunk2 1536 --out $OUT/x_c1536.json &&
step x_c4096 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --variants perf --self-copies --init gaussian --chunk2 4096 --out $OUT/x_c4096.json
