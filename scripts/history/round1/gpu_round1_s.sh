set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
export HSA_ENABLE_IPC_MODE_LEGACY=0 RMA_EXEC_VERBOSE=1
for m in plain lofirst; do
  RMA_EXEC_STREAMS=$m timeout -k 10 300 python bench/probe_set_temporal.py 16384 > gpurun_out/s/probe_$m.log 2>&1; rc=$?; tail -9 gpurun_out/s/probe_$m.log; [ $rc -eq 0 ] || exit $rc
done
