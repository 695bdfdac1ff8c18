#!/bin/bash
# r2: kernel + memory-copy timeline of 2 loopback ranks (perf_hide, K<=24 passes,
# 16384^2 tiles on one GPU): does the frame + exchange hide under the interior?
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/r2t; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench/loopback_scaling.py --n 16384 --ranks 2 --temporal 24 --steps 96 --out $OUT/loopback.json > $OUT/trace.log 2>&1 && echo "== trace ok"
