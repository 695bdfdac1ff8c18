set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== sweep 101376 fused"
timeout -k 10 400 python bench/stencil_sweep.py --n 101376 --no-roof --rounds 2 --iters 3 --chunks 4,8 --unrolls 4 --nts 3 --xcds 0,1 --vecs 2 --out gpurun_out/sweep101k.json > gpurun_out/sweep101k.log 2>&1 || { tail -20 gpurun_out/sweep101k.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sweep101k.json')); r=d['results']; [print('101k', k, round(r[k]['GBps_median'])) for k in sorted(r, key=lambda k:-r[k]['GBps_median'])]"
echo "== sweep 101376 interior"
timeout -k 10 400 python bench/stencil_sweep.py --n 101376 --x0 128 --y0 5 --no-roof --rounds 2 --iters 3 --chunks 4,8 --unrolls 4 --nts 3 --xcds 0,1 --vecs 2 --out gpurun_out/sweep101k_int.json > gpurun_out/sweep101k_int.log 2>&1 || { tail -20 gpurun_out/sweep101k_int.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/sweep101k_int.json')); r=d['results']; [print('101k int', k, round(r[k]['GBps_median'])) for k in sorted(r, key=lambda k:-r[k]['GBps_median'])]"
echo "== trace perf 16k"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_perf16k -o run -- python3 bench.py --nx 16384 --steps 60 --warmup 5 --variant perf > gpurun_out/prof_perf16k.log 2>&1 || { tail -20 gpurun_out/prof_perf16k.log; exit 1; }
echo done
