#!/bin/bash
# r2: x-frames widened to the strip capacity (RMA_FRAME_FILL A/B) + correctness
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zg
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_fuzz_gpu.py tests/test_executor_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
for ff in 0 1; do
  export RMA_FRAME_FILL=$ff
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 16384 --K 24 --steps 2400 --out $OUT/r16_${ff}_$rep.json > $OUT/r16_${ff}_$rep.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 0 --K 24 --steps 240 --out $OUT/r101_${ff}_$rep.json > $OUT/r101_${ff}_$rep.log 2>&1 || exit $?
done
done
unset RMA_FRAME_FILL
python - <<'PY'
import json
for rep in (1, 2):
    for ff in (0, 1):
        for t in ("r16", "r101"):
            d = json.load(open(f"gpurun_out/r2zg/{t}_{ff}_{rep}.json"))
            runs = d["variants"]["perf_hide"]["runs"]
            o = min(r["ms_per_step"] for r in runs if not r["periodic_rccl_self"])
            p = min(r["ms_per_step"] for r in runs if r["periodic_rccl_self"])
            print(rep, "fill" if ff else "nofill", t, round(o, 5), round(p, 5), "%.2f%%" % (100 * (p / o - 1)))
PY
