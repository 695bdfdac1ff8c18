#!/bin/bash
# r2: HBM bytes of the final deep passes (rocprofv3 FETCH_SIZE / WRITE_SIZE, one pass each)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/r2zx; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
SW="$R/bench/pass_sweep.py --pipe 20,24 --pipec 12 --ldsdpp= --old= --alt= --rounds 1"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -o run -- python3 $SW > $OUT/f.log 2>&1 && echo "== fetch ok" &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -o run -- python3 $SW > $OUT/w.log 2>&1 && echo "== write ok"
