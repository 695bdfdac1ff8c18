set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/z
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2048 4096 8192; do
  timeout -k 10 300 python bench/stencil_sweep.py --n $n --rounds 5 --iters 20 --chunks 4 --unrolls 4 --nts 3 --xcds 0 --no-roof --tb-chunks 8,16 --tb-unrolls 2 --tb-xcds 0 --tbk 3,4,6,8 --tbk-chunks 16,32,64,128 --tbk-xcds 1 --tbk-vecs 2 --tbk-kernels lds --out gpurun_out/z/sweep_$n.json > gpurun_out/z/sweep_$n.log 2>&1; rc=$?
  echo "n=$n rc=$rc"; grep -E '"best' gpurun_out/z/sweep_$n.log; [ $rc -eq 0 ] || exit $rc
done
