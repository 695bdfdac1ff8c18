set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
echo "== pytest gpu"
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
if fatal $rc; then echo "FATAL pytest rc=$rc"; exit $rc; fi
[ $rc -ne 0 ] && grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head -20
echo "== sweep 16384"
timeout -k 10 300 python bench/stencil_sweep.py --n 16384 --rounds 4 --iters 8 --out gpurun_out/sweep16k.json > gpurun_out/sweep16k.log 2>&1 || { echo SWEEP_FAIL; tail -30 gpurun_out/sweep16k.log; exit 1; }
python - <<'PY'
import json
d=json.load(open("gpurun_out/sweep16k.json"))
r=d["results"]
for k in sorted(r, key=lambda k:-r[k]["GBps_median"])[:12]: print(k, round(r[k]["GBps_median"],1), round(r[k]["GBps_best"],1))
print("copy", d["best_copy"], round(d["copy_GBps"],1), "triad", d["best_triad"], round(d["triad_GBps"],1), "lds", round(r["lds"]["GBps_median"],1))
PY
echo "== native example"
timeout -k 10 120 ./build/examples/diffusion_2D_perf_hide 16384 300 1 > gpurun_out/example.log 2>&1; cat gpurun_out/example.log
echo "== pmc"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench/pmc_probe.py > gpurun_out/pmc_fetch.log 2>&1 || { echo PMC1_FAIL; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench/pmc_probe.py > gpurun_out/pmc_write.log 2>&1 || { echo PMC2_FAIL; tail -20 gpurun_out/pmc_write.log; exit 1; }
ls -R gpurun_out/pmc_fetch | head
exit $rc
