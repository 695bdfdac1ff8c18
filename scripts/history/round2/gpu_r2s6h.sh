#!/bin/bash
# r2: is the x-periodic overhead at the 288 GB tile the concurrency of frame + exchange with
# the interior? perf (exchange after the one-launch pass) vs perf_hide, periodic x and xy
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6h
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"overhead": [-0-9.e]*' "$OUT/$name.log" | tr '\n' ' '; echo
  return $rc
}
for d in x xy; do
  step ${d}_perf_hide 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic $d --variants perf,perf_hide --out $OUT/${d}.json || exit 1
done
RMA_FRAME_ALIGNED=1 step x_al1536 400 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --variants perf,perf_hide --chunk2 1536 --out $OUT/x_al1536.json
