set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/p/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/p/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/p/smoke.log 2>&1; rc=$?
tail -2 gpurun_out/p/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/p/bench.log 2>&1; rc=$?
tail -1 gpurun_out/p/bench.log; exit $rc
