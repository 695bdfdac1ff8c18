#!/bin/bash
# r2: GPU suite after the loopback gather fix; same-box RCCL-self halo overhead at the 288 GB
# tile for periodic x / y / xy with the default frame strips vs aligned 1536-row tasks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6g
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"overhead": [-0-9.e]*' "$OUT/$name.log" | tr '\n' ' '; tail -1 "$OUT/$name.log" | cut -c1-160
  return $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ;
for d in x xy y; do
  step ${d}_strips 300 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic $d --out $OUT/${d}_strips.json || exit 1
  RMA_FRAME_ALIGNED=1 step ${d}_al1536 300 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic $d --chunk2 1536 --out $OUT/${d}_al1536.json || exit 1
done
