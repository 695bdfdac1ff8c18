#!/bin/bash
# r2: planner cost tables after the mirrored factor ring (all 4 tile classes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2m
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 0 16384 8192 4096; do
  timeout -k 10 400 python -u bench/pass_sweep.py --n $n --rounds 3 --pipe 1-24 --pipec 5-12,16,20 --ldsdpp 3,4,6,8 --old "" --alt "" --out $OUT/pass_sweep_$n.json > $OUT/sweep_$n.log 2>&1 || exit $?
  echo "== sweep $n ok"
done
