#!/bin/bash
# r2: longer chunks at the 288 GB tile; 12288^2 (the reference's perf tile) and 24576^2 checks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zd
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench/pass_sweep.py --n 0 --rounds 5 --pipe 20,24 --pipec "" --ldsdpp "" --old= --alt= --chunks 24:2048/3072/4096/5120/6144,20:2048/3072/4096/6144 --out $OUT/c101k.json > $OUT/c101k.log 2>&1 || exit $?
for n in 12288 24576; do
timeout -k 10 400 python -u bench/pass_sweep.py --n $n --rounds 7 --pipe 12,16,20,24 --pipec "" --ldsdpp "" --old= --alt= --chunks 24:256/384/512/768/1024/1536,16:256/384/512/768/1024,12:256/512/1024 --out $OUT/c$n.json > $OUT/c$n.log 2>&1 || exit $?
done
python - <<'PY'
import json
for f in ("c101k", "c12288", "c24576"):
    d = json.load(open(f"gpurun_out/r2zd/{f}.json"))
    print(f, d["tile"], d["one_step_ms"])
    for r in d["rows"]:
        if r["kernel"] == "pipe":
            print(" ", r["K"], r["chunk_rows"], r["ms_per_pass"])
PY
