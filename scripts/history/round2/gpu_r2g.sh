#!/bin/bash
# r2: RCCL host overhead with the blocking data communicator (default) vs the
# polled non-blocking one; GPU suite; stream pool default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2g
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400
  return $rc
}
step rccl_self_16k_blocking 600 python -u bench/rccl_self_overhead.py --n 16384 --K 1 --variants perf,perf_hide --steps 400 --out $OUT/rccl_self_16k_k1_blocking.json &&
RMA_RCCL_DATA_NONBLOCKING=1 step rccl_self_16k_polled 600 python -u bench/rccl_self_overhead.py --n 16384 --K 1 --variants perf_hide --steps 400 --out $OUT/rccl_self_16k_k1_polled.json &&
step stream_order 600 python -u bench/probe_stream_order.py --n 16384 --modes pool,lofirst &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 120 --timeout-method thread -p no:cacheprovider
