#!/bin/bash
# K=16 fast5p4 at the 288 GB tile: XCD-aware block remap on/off, chunk 1536/2048
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=${OUT:-gpurun_out/xcd101k}
mkdir -p "$OUT"
timeout -k 10 500 python bench/stencil_sweep.py --n 101376 --rounds 3 --iters 2 --no-roof --no-march --tbk 16 --tbk-chunks 1536,2048 --tbk-xcds 0,1 --tbk-vecs 4 --tbk-kernels fast5p4 --out "$OUT/sweep.json" > "$OUT/sweep.log" 2>&1 && echo sweep ok
