#!/bin/bash
# Kernel trace + stats of bench/rccl_self_overhead.py runs, one rocprofv3 run
# per pattern letter (o open, p periodic RCCL-self, d periodic direct-store):
#   N=4096 K=24 PATS="o d p" OUT=gpurun_out/prof bash scripts/prof_pattern.sh
set -eo pipefail
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=${OUT:-gpurun_out/prof_pattern}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for p in ${PATS:-o d p}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$p" -o run -- \
      python3 bench/rccl_self_overhead.py --n "${N:-4096}" --K "${K:-24}" --pattern "$p" \
      --steps "${STEPS:-240}" --spacing equal > "$OUT/$p.log" 2>&1
done
