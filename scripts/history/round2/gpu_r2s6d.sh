#!/bin/bash
# r2: is the one-step path's "enqueue" time host work or a full GPU queue? short runs
# (queue never fills) and a small tile (GPU faster than the host)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6d
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 "$OUT/$name.log" | cut -c1-400
  return $rc
}
for st in 10 40 100 400; do
  step rs16k_s$st 300 python -u bench/rccl_self_overhead.py --n 16384 --K 1 --variants perf_hide --steps $st --out $OUT/rs16k_s$st.json || exit 1
done
step rs2k 300 python -u bench/rccl_self_overhead.py --n 2048 --K 1 --variants perf,perf_hide --steps 400 --out $OUT/rs2k.json &&
step rs4k 300 python -u bench/rccl_self_overhead.py --n 4096 --K 1 --variants perf,perf_hide --steps 400 --out $OUT/rs4k.json
