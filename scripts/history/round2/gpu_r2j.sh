#!/bin/bash
# r2: pass cost per depth at smaller tiles (planner table validity)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2j
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 16384 8192 4096; do
  timeout -k 10 300 python -u bench/pass_sweep.py --n $n --rounds 5 --pipe 1-24 --pipec 5-12,16,20 --ldsdpp 3,4,6,8 --old "" --alt "" --out $OUT/pass_sweep_$n.json > $OUT/sweep_$n.log 2>&1 || exit $?
  echo "== sweep $n ok"
done
