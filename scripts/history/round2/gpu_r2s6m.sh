#!/bin/bash
# r2: owned-rect origin effect on the K=24 pass kernel alone, smooth field
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6m
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench/interior_shape_probe.py --K 24 --init gaussian --reps 3 --out $OUT/shape_gauss.json > $OUT/shape.log 2>&1; rc=$?
tail -1 $OUT/shape.log; exit $rc
