#!/bin/bash
# r2: validation of the aligned frames (auto rule): multi-rank + fuzz + executor tests, overheads
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zn
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_multirank_gpu.py tests/test_fuzz_gpu.py tests/test_executor_gpu.py tests/test_guard_bands_gpu.py tests/test_capi_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 16384 --K 24 --steps 2400 --out $OUT/r16.json > $OUT/r16.log 2>&1 || exit $?
timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 0 --K 24 --steps 240 --out $OUT/r101.json > $OUT/r101.log 2>&1 || exit $?
timeout -k 10 300 python -u bench/loopback_scaling.py --n 16384 --ranks 1,2,4,8 --temporal 24 --steps 480 --out $OUT/loopback.json > $OUT/loopback.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("r16", "r101"):
    d = json.load(open(f"gpurun_out/r2zn/{f}.json"))
    runs = d["variants"]["perf_hide"]["runs"]
    o = min(r["ms_per_step"] for r in runs if not r["periodic_rccl_self"])
    p = min(r["ms_per_step"] for r in runs if r["periodic_rccl_self"])
    print(f, round(o, 5), round(p, 5), "%.2f%%" % (100 * (p / o - 1)))
for r in json.load(open("gpurun_out/r2zn/loopback.json")):
    print("loopback", r["ranks"], r["temporal"], round(r["fraction_of_1_rank"], 4))
PY
