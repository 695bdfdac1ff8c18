set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== pytest gpu (kernels only)"
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_executor_gpu.py -q -x > gpurun_out/pytest_gpu_k.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu_k.log
case $rc in 0) ;; 1) grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_k.log | head; exit 1;; *) exit $rc;; esac
echo "== sweep 16k fused + interior-like rect"
timeout -k 10 300 python bench/stencil_sweep.py --n 16384 --rounds 3 --iters 8 --chunks 4,8 --unrolls 4 --nts 3 --xcds 0,1 --vecs 2 --out gpurun_out/sweep16k_xcd.json > gpurun_out/sweep16k_xcd.log 2>&1 || { tail -20 gpurun_out/sweep16k_xcd.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sweep16k_xcd.json')); r=d['results']; [print(k, round(r[k]['GBps_median'])) for k in sorted(r, key=lambda k:-r[k]['GBps_median'])[:14]]"
timeout -k 10 300 python bench/stencil_sweep.py --n 16384 --x0 128 --y0 5 --no-roof --rounds 3 --iters 8 --chunks 4,8 --unrolls 4 --nts 3 --xcds 0,1 --vecs 2 --out gpurun_out/sweep16k_int.json > gpurun_out/sweep16k_int.log 2>&1 || { tail -20 gpurun_out/sweep16k_int.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sweep16k_int.json')); r=d['results']; [print('interior', k, round(r[k]['GBps_median'])) for k in sorted(r, key=lambda k:-r[k]['GBps_median'])]"
echo "== sweep big tile 65536"
timeout -k 10 400 python bench/stencil_sweep.py --n 65536 --rounds 2 --iters 3 --chunks 4,8,16 --unrolls 4 --nts 1,3 --xcds 0,1 --vecs 2 --out gpurun_out/sweep64k.json > gpurun_out/sweep64k.log 2>&1 || { tail -20 gpurun_out/sweep64k.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sweep64k.json')); r=d['results']; [print('64k', k, round(r[k]['GBps_median'])) for k in sorted(r, key=lambda k:-r[k]['GBps_median'])[:16]]"
echo "== bench 16k hide/perf + auto"
for v in perf_hide perf; do
  timeout -k 10 300 python bench.py --nx 16384 --steps 1000 --warmup 10 --variant $v > gpurun_out/bench16k_$v.log 2>&1 || { tail -20 gpurun_out/bench16k_$v.log; exit 1; }
  tail -1 gpurun_out/bench16k_$v.log | cut -c1-200
done
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-200
