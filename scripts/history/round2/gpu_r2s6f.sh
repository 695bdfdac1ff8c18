#!/bin/bash
# r2: diagnosis of the intermittent one-step perf_hide loopback mismatches (frame sides x
# halo batching), then the interior rect-shape probe at the 288 GB tile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6f
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300
  return $rc
}
step stress_default 240 python -u scripts/stress_loopback.py 12 &&
RMA_HALO_BATCH=0 step stress_nobatch 240 python -u scripts/stress_loopback.py 12 &&
RMA_FRAME_SIDES=all step stress_allsides 240 python -u scripts/stress_loopback.py 12 &&
RMA_FRAME_SIDES=all RMA_HALO_BATCH=0 step stress_old 240 python -u scripts/stress_loopback.py 12 &&
step shape 300 python -u bench/interior_shape_probe.py --K 24 --out $OUT/shape_k24.json
