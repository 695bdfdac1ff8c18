set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/o
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -m pytest tests/test_multirank_gpu.py tests/test_executor_gpu.py tests/test_temporal_gpu.py -x -q > gpurun_out/o/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/o/pytest.log; [ $rc -eq 0 ] || exit $rc
for tb in 1 2 4 6 8; do
  timeout -k 10 120 python bench.py --nx 16384 --temporal $tb > gpurun_out/o/bench_16k_tb${tb}.log 2>&1; rc=$?
  echo "16k perf_hide tb$tb: $(grep -o '"value": [0-9.]*' gpurun_out/o/bench_16k_tb${tb}.log)"; [ $rc -eq 0 ] || exit $rc
done
for tb in 6 8; do
  timeout -k 10 300 python bench.py --temporal $tb > gpurun_out/o/bench_auto_tb${tb}.log 2>&1; rc=$?
  echo "auto perf_hide tb$tb: $(grep -o '"value": [0-9.]*' gpurun_out/o/bench_auto_tb${tb}.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/o/bench_auto_tb${tb}.log)"; [ $rc -eq 0 ] || exit $rc
done
