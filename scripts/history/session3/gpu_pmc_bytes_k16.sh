#!/bin/bash
# HBM bytes of the default K=16 pass (fast5p4, 101376^2): FETCH_SIZE / WRITE_SIZE.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
OUT=$R/gpurun_out/pmc_bytes; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export RMA_PROBE_SET=fast RMA_PROBE_N=101376 RMA_PROBE_REPS=2 RMA_PROBE_K=16 RMA_PROBE_KERNELS=fast5p4
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -o run -- python3 $R/bench/pmc_probe.py > $OUT/f.log 2>&1 && echo "== fetch ok" &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -o run -- python3 $R/bench/pmc_probe.py > $OUT/w.log 2>&1 && echo "== write ok"
