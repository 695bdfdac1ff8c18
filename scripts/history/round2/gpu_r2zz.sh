#!/bin/bash
# r2: chunk rows vs the task tail at the 288 GB tile: chunk sizes whose task count per XCD
# fills the last round of block slots (2 blocks per CU at K=20/24) vs the table's 3072
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zz
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u bench/pass_sweep.py --n 0 --rounds 5 --pipe "20,24" --pipec "" --ldsdpp "" --old= --alt= \
  --chunks "20:2560/2740/3380/3899/4055/4608,24:2358/2560/3168/3380/4608/4828" \
  --out $OUT/chunk_tail_101376.json > $OUT/chunk_tail.log 2>&1
