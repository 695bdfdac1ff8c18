set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/w
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/w/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/w/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/w/smoke.log 2>&1; rc=$?
tail -1 gpurun_out/w/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/w/bench.log 2>&1; rc=$?
tail -1 gpurun_out/w/bench.log | cut -c1-330; grep -o '"teff_single_step_kernel_GBps": [0-9.]*' gpurun_out/w/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --nx 16384 > gpurun_out/w/bench16k.log 2>&1; rc=$?
grep -o '"value": [0-9.]*' gpurun_out/w/bench16k.log; exit $rc
