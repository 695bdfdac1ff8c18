set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench/probe_set_temporal.py 16384 > gpurun_out/t/probe.log 2>&1; rc=$?; tail -4 gpurun_out/t/probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/t/bench.log 2>&1; rc=$?; tail -1 gpurun_out/t/bench.log | cut -c1-300; grep -o '"teff_single_step_kernel_GBps": [0-9.]*' gpurun_out/t/bench.log; exit $rc
