set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/j
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_temporal_gpu.py tests/test_executor_gpu.py -x -q > gpurun_out/j/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/j/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/stencil_sweep.py --n 16384 --rounds 5 --iters 20 --chunks 4 --unrolls 4 --nts 3 --xcds 0 --tb-chunks 6,8,14,16,30 --tb-unrolls 2,4 --tb-xcds 0,1 --out gpurun_out/j/sweep_tb_16k.json > gpurun_out/j/sweep.log 2>&1; rc=$?
grep -E '"best|GBps_equiv|copy_GBps|triad_GBps' gpurun_out/j/sweep.log; exit $rc
