#!/bin/bash
# r2: two column waves per stage (8-wave blocks): bitwise + guard tests, sweep vs one column
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2n
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_pipe_gpu.py tests/test_guard_bands_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 python -u bench/pass_sweep.py --rounds 3 --pipe 13-24 --pipe2 13-24 --chunks2 20:1536/6144,24:1536/6144 --pipec "" --ldsdpp "" --old "" --alt "" --out $OUT/sweep_101k.json > $OUT/sweep_101k.log 2>&1 || exit $?
timeout -k 10 600 python -u bench/pass_sweep.py --n 16384 --rounds 5 --pipe 13-24 --pipe2 13-24 --chunks2 16:128/512,20:128/512,24:128/512 --pipec "" --ldsdpp "" --old "" --alt "" --out $OUT/sweep_16k.json > $OUT/sweep_16k.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/r2n/sweep_101k.json", "gpurun_out/r2n/sweep_16k.json"):
    d = json.load(open(f))
    print(f, d["one_step_ms"])
    for r in d["rows"]:
        print(" ", r["kernel"], r["K"], r["chunk_rows"], r["ms_per_pass"], r["rel"])
PY
