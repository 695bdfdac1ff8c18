#!/bin/bash
# r2: full GPU suite + smoke + benches on every tile class with the per-tile chunks and tables
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zc
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/bench_20_5.json > $OUT/bench_20_5.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --json-out $OUT/bench_default.json > $OUT/bench_default.log 2>&1 || exit $?
for n in 16384 8192 4096; do
  timeout -k 10 300 python -u bench.py --nx $n --steps 1000 --warmup 50 --json-out $OUT/bench_$n.json > $OUT/bench_$n.log 2>&1 || exit $?
done
python - <<'PY'
import json
for f in ("bench_20_5", "bench_default", "bench_16384", "bench_8192", "bench_4096"):
    d = json.load(open(f"gpurun_out/r2zc/{f}.json"))
    c = d["config"]
    print(f, d["value"], d["ms_per_step"], c["passes_timed"][:3], len(c["passes_timed"]), c["kstep_kernel"])
PY
