#!/bin/bash
# r2: kernel timelines for the overlap evidence: 4 loopback ranks (16384^2, K<=24)
# and one rank with RCCL send/recv to itself on a periodic 101376^2 tile (K<=24)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/r2u; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lb4 -o run -- python3 $R/bench/loopback_scaling.py --n 16384 --ranks 4 --temporal 24 --steps 96 --out $OUT/lb4.json > $OUT/lb4.log 2>&1 && echo "== lb4 ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rccl -o run -- python3 $R/bench/rccl_self_overhead.py --n 0 --K 24 --steps 96 --out $OUT/rccl.json > $OUT/rccl.log 2>&1 && echo "== rccl ok"
