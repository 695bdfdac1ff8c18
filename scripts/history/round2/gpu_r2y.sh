#!/bin/bash
# r2: P2P smoke test through RCCL on one GPU + fuzz
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2y
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_multirank_gpu.py -k "p2p_smoke or rccl" -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -u -m rocm_mpi_amd.apps.rocmaware_test_selectdevice --transport rccl --self-ring > $OUT/app.log 2>&1 || { cat $OUT/app.log; exit 1; }
cat $OUT/app.log
