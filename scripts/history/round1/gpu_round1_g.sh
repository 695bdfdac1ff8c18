set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py tests/test_multirank_gpu.py -q -x > gpurun_out/pytest_gpu_k.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_k.log
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_k.log | head; exit 1;; *) exit $rc;; esac
for v in perf_hide perf; do
  timeout -k 10 300 python bench.py --nx 16384 --steps 1000 --warmup 10 --variant $v > gpurun_out/bench16k_$v.log 2>&1 || { tail -20 gpurun_out/bench16k_$v.log; exit 1; }
  tail -1 gpurun_out/bench16k_$v.log | cut -c100-200
done
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c100-200
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hide16k -o run -- python3 bench.py --nx 16384 --steps 50 --warmup 5 > gpurun_out/prof_hide16k.log 2>&1 || { tail -20 gpurun_out/prof_hide16k.log; exit 1; }
echo done
