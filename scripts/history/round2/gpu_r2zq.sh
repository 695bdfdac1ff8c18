#!/bin/bash
# r2: the 2048^2 class: chunk rows per depth, then the pass costs with the chosen chunks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zq
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
C="16/32/48/64/96/128/192/256/384/512"
SPEC=""; for K in 2 4 6 8 10 12 14 16 18 20 22 24; do SPEC="$SPEC${SPEC:+,}$K:$C"; done
SPECC=""; for K in 6 8 12 16 20; do SPECC="$SPECC${SPECC:+,}$K:$C"; done
timeout -k 10 400 python -u bench/pass_sweep.py --n 2048 --rounds 11 --pipe "" --pipec "" --ldsdpp "" --old= --alt= --chunks "$SPEC" --chunksc "$SPECC" --out $OUT/chunks_2048.json > $OUT/chunks_2048.log 2>&1 || exit $?
echo "== done"
