#!/bin/bash
# 2 ranks on the one GPU (host-staged halos) through bench.py's multi-rank path,
# ending in comm.shutdown_distributed (barrier before destroy); then the GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=${OUT:-gpurun_out/teardown}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
RMA_TRANSPORT=staged timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29650 bench.py --gpus 2 --nx 16384 --steps 200 --single-step-steps 0 --json-out "$OUT/bench2.json" > "$OUT/bench2.log" 2>&1 &&
echo "== bench2 ok" && tail -1 "$OUT/bench2.log" | cut -c1-200 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
tail -1 "$OUT/pytest_gpu.log"
