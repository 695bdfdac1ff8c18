set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/n
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_temporal_gpu.py tests/test_kernels_gpu.py -x -q > gpurun_out/n/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/n/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench/stencil_sweep.py --n 16384 --rounds 5 --iters 10 --chunks 4 --unrolls 4 --nts 3 --xcds 0 --no-roof --tb-chunks 16 --tb-unrolls 2 --tb-xcds 0 --tbk 2,3,4,6,8 --tbk-chunks 64,128,256 --tbk-xcds 1 --tbk-vecs 1,2 --out gpurun_out/n/sweep_tbk_16k.json > gpurun_out/n/sweep.log 2>&1; rc=$?
grep -E '"best' gpurun_out/n/sweep.log; exit $rc
