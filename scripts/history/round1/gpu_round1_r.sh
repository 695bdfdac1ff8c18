set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench/probe_set_temporal.py 16384 > gpurun_out/r/probe16k.log 2>&1; rc=$?; cat gpurun_out/r/probe16k.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/probe_set_temporal.py 65536 > gpurun_out/r/probe64k.log 2>&1; rc=$?; cat gpurun_out/r/probe64k.log | tail -6; exit $rc
