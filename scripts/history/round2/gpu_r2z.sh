#!/bin/bash
# r2: chunk rows of the deep passes on the smaller tile classes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2z
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 16384 8192; do
timeout -k 10 300 python -u bench/pass_sweep.py --n $n --rounds 7 --pipe 12,16,20,24 --chunks 24:128/384/512/768/1024,20:128/384/512/768,16:128/384/512,12:128/384/512 --pipec "" --ldsdpp "" --old= --alt= --out $OUT/sweep_$n.json > $OUT/sweep_$n.log 2>&1 || exit $?
done
python - <<'PY'
import json
for n in (16384, 8192):
    d = json.load(open(f"gpurun_out/r2z/sweep_{n}.json"))
    print(n, d["one_step_ms"])
    for r in d["rows"]:
        print(" ", r["kernel"], r["K"], r["chunk_rows"], r["ms_per_pass"], round(r["ms_per_step"], 4))
PY
