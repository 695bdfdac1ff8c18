set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head; exit 1;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --nx 16384 --steps 1000 --warmup 10 --variant kp > gpurun_out/bench16k_kp.log 2>&1 || { tail -20 gpurun_out/bench16k_kp.log; exit 1; }
tail -1 gpurun_out/bench16k_kp.log | cut -c100-200
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kp16k -o run -- python3 bench.py --nx 16384 --steps 30 --warmup 3 --variant kp > gpurun_out/prof_kp16k.log 2>&1 || { tail -20 gpurun_out/prof_kp16k.log; exit 1; }
head -5 gpurun_out/prof_kp16k/run_kernel_stats.csv | cut -c1-150
echo done
