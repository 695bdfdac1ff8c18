set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/k
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -m pytest tests/test_temporal_gpu.py tests/test_multirank_gpu.py tests/test_executor_gpu.py -x -q > gpurun_out/k/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/k/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in perf perf_hide; do
  for tb in 1 2; do
    timeout -k 10 120 python bench.py --variant $v --nx 16384 --temporal $tb > gpurun_out/k/bench_16k_${v}_tb${tb}.log 2>&1; rc=$?
    echo "16k $v tb$tb: $(grep -o '"value": [0-9.]*' gpurun_out/k/bench_16k_${v}_tb${tb}.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 python bench.py --temporal 2 > gpurun_out/k/bench_auto_tb2.log 2>&1; rc=$?
tail -1 gpurun_out/k/bench_auto_tb2.log; exit $rc
