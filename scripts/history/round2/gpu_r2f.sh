#!/bin/bash
# r2: GPU suite after the halo-plan / C ABI refactor, stream-order probe (+ kernel
# trace with queue ids), RCCL-self overhead at 16384^2 one-step and 288 GB K<=24
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out/r2f
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "$OUT/$name.log" | cut -c1-600
  return $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 120 --timeout-method thread -p no:cacheprovider &&
step stream_order 600 python -u bench/probe_stream_order.py --n 16384 &&
(cd /tmp && export TMPDIR=/tmp && for m in hifirst lofirst; do
   RMA_EXEC_STREAMS=$m RMA_EXEC_VERBOSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
     -d "$R/$OUT/trace_$m" -o run -- python3 "$R/bench/probe_stream_order.py" --child --n 16384 \
     > "$R/$OUT/trace_$m.log" 2>&1 || exit $?; echo "== trace $m ok"; done) &&
step rccl_self_16k 600 python -u bench/rccl_self_overhead.py --n 16384 --K 1 --variants perf,perf_hide --steps 400 --out $OUT/rccl_self_16k_k1.json &&
step rccl_self_101k 600 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --out $OUT/rccl_self_101k_k24.json
