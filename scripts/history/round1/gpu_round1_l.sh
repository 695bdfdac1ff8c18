set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/l
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m pytest tests/test_temporal_gpu.py -x -q > gpurun_out/l/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/l/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench/stencil_sweep.py --n 16384 --rounds 5 --iters 10 --chunks 4 --unrolls 4 --nts 3 --xcds 0 --no-roof --tbk 2,3,4 --tbk-chunks 16,32,64,128 --tbk-xcds 0,1 --tbk-vecs 2,4 --out gpurun_out/l/sweep_tbk_16k.json > gpurun_out/l/sweep.log 2>&1; rc=$?
grep -E '"best' gpurun_out/l/sweep.log; exit $rc
