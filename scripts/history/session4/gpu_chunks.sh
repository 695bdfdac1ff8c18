#!/bin/bash
# row-chunk length of the K=16 fast5p4 pass at the 288 GB tile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=${OUT:-gpurun_out/chunks}
mkdir -p "$OUT"
timeout -k 10 500 python bench/stencil_sweep.py --n 101376 --rounds 3 --iters 2 --no-roof --no-march --tbk 16 --tbk-chunks 512,1024,1536,2048,3072,4096 --tbk-xcds 1 --tbk-vecs 4 --tbk-kernels fast5p4 --out "$OUT/sweep_101k.json" > "$OUT/sweep_101k.log" 2>&1
