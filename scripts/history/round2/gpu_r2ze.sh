#!/bin/bash
# r2: frame strips split by shape (wide: 4 cells/lane, tall: 2 cells/lane + interior chunk):
# correctness tests, then the RCCL-self halo overhead at 101376^2 and 16384^2 (K=24)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2ze
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_fuzz_gpu.py tests/test_guard_bands_gpu.py tests/test_executor_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 0 --K 24 --steps 240 --out $OUT/rccl_101k.json > $OUT/rccl_101k.log 2>&1 || exit $?
timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 16384 --K 24 --steps 2400 --out $OUT/rccl_16k.json > $OUT/rccl_16k.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("rccl_101k", "rccl_16k"):
    d = json.load(open(f"gpurun_out/r2ze/{f}.json"))
    for v, x in d["variants"].items():
        for r in x["runs"]:
            print(f, v, r["periodic_rccl_self"], round(r["ms_per_step"], 5), r["pass_split_ms"])
PY
