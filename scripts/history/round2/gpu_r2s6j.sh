#!/bin/bash
# r2: is the "periodic is slower" pattern the run order (each run allocates a 230 GB tile)?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6j
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.log" | head -8 | tr '\n' ' '; echo
  return $rc
}
step oooo 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --variants perf --self-copies --pattern oooo --out $OUT/oooo.json &&
step ppoo 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --variants perf --self-copies --pattern ppoo --out $OUT/ppoo.json
