#!/bin/bash
# r2: chunk rows x depth x tile class for the pipelined passes (fast5 + canonical)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2za
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
CS="32/64/128/192/256/384/512/768/1024/1536/2048/3072"
for n in 4096 8192 16384 32768 0; do
  case $n in 4096) C="32/64/128/192/256/384/512/768/1024/1536/2048"; R=9;; 8192|16384) C="32/64/128/192/256/384/512/768/1024/1536/2048/3072"; R=7;; *) C=$CS; R=3;; esac
  SPEC=""; for K in 4 6 8 10 12 14 16 18 20 22 24; do SPEC="$SPEC${SPEC:+,}$K:$C"; done
  SPECC=""; for K in 8 12 16; do SPECC="$SPECC${SPECC:+,}$K:$C"; done
  timeout -k 10 400 python -u bench/pass_sweep.py --n $n --rounds $R --pipe "" --pipec "" --ldsdpp "" --old= --alt= --chunks "$SPEC" --chunksc "$SPECC" --out $OUT/chunks_$n.json > $OUT/chunks_$n.log 2>&1 || exit $?
  echo "== $n ok"
done
