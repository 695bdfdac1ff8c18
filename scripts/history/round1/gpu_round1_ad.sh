set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ad
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_temporal_gpu.py tests/test_guard_bands_gpu.py -x -q > gpurun_out/ad/pytest.log 2>&1; rc=$?
tail -1 gpurun_out/ad/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/stencil_sweep.py --n 16384 --rounds 5 --iters 10 --chunks 4 --unrolls 4 --nts 3 --xcds 0 --no-roof --tbk 8 --tbk-chunks 128,256 --tbk-xcds 1 --tbk-vecs 2 --tbk-kernels fast,fast_w4 --out gpurun_out/ad/sweep16k.json > gpurun_out/ad/sweep16k.log 2>&1; rc=$?
grep -E '"best' gpurun_out/ad/sweep16k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/stencil_sweep.py --n 101376 --rounds 3 --iters 2 --chunks 4 --unrolls 4 --nts 3 --xcds 1 --no-roof --tbk 8 --tbk-chunks 512,1024 --tbk-xcds 1 --tbk-vecs 2 --tbk-kernels fast,fast_w4 --out gpurun_out/ad/sweep101k.json > gpurun_out/ad/sweep101k.log 2>&1; rc=$?
grep -E '"best' gpurun_out/ad/sweep101k.log; exit $rc
