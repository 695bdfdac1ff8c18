set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== rocm-smi"; (rocm-smi --showproductname --showmeminfo vram 2>&1 | head -30) > gpurun_out/smi.log || true
echo "== smoke"
timeout -k 10 400 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -50 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
echo "== pytest gpu"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "not int64" > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "== bench 16k perf_hide"
timeout -k 10 300 python bench.py --nx 16384 --steps 300 --warmup 10 > gpurun_out/bench16k_hide.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench16k_hide.log; exit 1; }
cat gpurun_out/bench16k_hide.log
timeout -k 10 300 python bench.py --nx 16384 --steps 300 --warmup 10 --variant perf > gpurun_out/bench16k_perf.log 2>&1 && cat gpurun_out/bench16k_perf.log
timeout -k 10 300 python bench.py --nx 16384 --steps 300 --warmup 10 --variant perf --kernel lds > gpurun_out/bench16k_lds.log 2>&1 && cat gpurun_out/bench16k_lds.log
timeout -k 10 300 python bench.py --nx 16384 --steps 300 --warmup 10 --variant kp > gpurun_out/bench16k_kp.log 2>&1 && cat gpurun_out/bench16k_kp.log
echo "== rocprof"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof16k -o run -- python3 bench.py --nx 16384 --steps 100 --warmup 5 > gpurun_out/prof16k.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof16k.log; }
find gpurun_out/prof16k -name "*stats*" | head
echo "== bench auto-size"
timeout -k 10 400 python bench.py --steps 60 --warmup 5 > gpurun_out/bench_auto.log 2>&1 && cat gpurun_out/bench_auto.log
