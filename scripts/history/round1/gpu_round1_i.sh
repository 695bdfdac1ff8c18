set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/i
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/i/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/i/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/baseline_configs.py --max-gpus 1 --out gpurun_out/i/baseline_configs_1gpu.json > gpurun_out/i/baseline.log 2>&1; rc=$?
tail -8 gpurun_out/i/baseline.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/i/bench.log 2>&1; rc=$?
tail -3 gpurun_out/i/bench.log; exit $rc
