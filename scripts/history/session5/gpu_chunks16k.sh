#!/bin/bash
# chunk rows of the pipelined K-step kernels (executor defaults: K=16 fast5p4,
# K=12 fast5p2) at 16384^2 and 32768^2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=${OUT:-gpurun_out/chunks16k}
mkdir -p "$OUT"
timeout -k 10 300 python bench/stencil_sweep.py --n 16384 --rounds 3 --iters 4 --no-roof --no-march --tbk 16 --tbk-chunks 256,512,768,1024,2048 --tbk-xcds 1 --tbk-vecs 4 --tbk-kernels fast5p4 --out "$OUT/k16_16k.json" > "$OUT/k16_16k.log" 2>&1 &&
timeout -k 10 300 python bench/stencil_sweep.py --n 16384 --rounds 3 --iters 4 --no-roof --no-march --tbk 12 --tbk-chunks 256,512,1024 --tbk-xcds 1 --tbk-vecs 4 --tbk-kernels fast5p2 --out "$OUT/k12_16k.json" > "$OUT/k12_16k.log" 2>&1 &&
timeout -k 10 300 python bench/stencil_sweep.py --n 32768 --rounds 3 --iters 3 --no-roof --no-march --tbk 16 --tbk-chunks 1024,2048 --tbk-xcds 1 --tbk-vecs 4 --tbk-kernels fast5p4 --out "$OUT/k16_32k.json" > "$OUT/k16_32k.log" 2>&1 &&
echo sweeps ok
