#!/bin/bash
# r2: host cost of an RCCL send/recv group (self) idle vs GPU busy, and RCCL env variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6c
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -E "^(idle|busy)" "$OUT/$name.log" | cut -c1-200
  return $rc
}
step default 120 python -u bench/rccl_enqueue_probe.py --out $OUT/default.json &&
step small 120 python -u bench/rccl_enqueue_probe.py --mb 0.13 --out $OUT/small.json &&
NCCL_GRAPH_MIXING_SUPPORT=0 step nomix 120 python -u bench/rccl_enqueue_probe.py --out $OUT/nomix.json &&
NCCL_LAUNCH_MODE=GROUP step launch_group 120 python -u bench/rccl_enqueue_probe.py --out $OUT/launch_group.json &&
RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 step nomscl 120 python -u bench/rccl_enqueue_probe.py --out $OUT/nomscl.json &&
NCCL_PROTO=Simple step simple 120 python -u bench/rccl_enqueue_probe.py --out $OUT/simple.json &&
RMA_RCCL_BLOCKING=1 step blocking 120 python -u bench/rccl_enqueue_probe.py --out $OUT/blocking.json
