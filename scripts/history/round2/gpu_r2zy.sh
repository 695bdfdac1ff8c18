#!/bin/bash
# r2: 288 GB tile with neighbours: strips + 3072-row chunks (default) vs aligned frames with
# 1536 / 1024-row chunks (absolute ms per step with RCCL-self periodic halos), K=24
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zy
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
  unset RMA_FRAME_ALIGNED
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 0 --K 24 --steps 240 --out $OUT/def_$rep.json > $OUT/def_$rep.log 2>&1 || exit $?
  export RMA_FRAME_ALIGNED=1
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 0 --K 24 --steps 240 --chunk2 1536 --out $OUT/a1536_$rep.json > $OUT/a1536_$rep.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 0 --K 24 --steps 240 --chunk2 1024 --out $OUT/a1024_$rep.json > $OUT/a1024_$rep.log 2>&1 || exit $?
done
unset RMA_FRAME_ALIGNED
python - <<'PY'
import json
for rep in (1, 2):
    for t in ("def", "a1536", "a1024"):
        d = json.load(open(f"gpurun_out/r2zy/{t}_{rep}.json"))
        runs = d["variants"]["perf_hide"]["runs"]
        o = min(r["ms_per_step"] for r in runs if not r["periodic_rccl_self"])
        p = min(r["ms_per_step"] for r in runs if r["periodic_rccl_self"])
        print(rep, t, "open", round(o, 5), "periodic", round(p, 5), "%.2f%%" % (100 * (p / o - 1)))
PY
