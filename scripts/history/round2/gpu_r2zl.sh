#!/bin/bash
# r2: aligned vs strip frames (RMA_FRAME_ALIGNED) at 32768^2 / 65536^2 / 101376^2, K=24
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zl
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
for ff in 0 1; do
  export RMA_FRAME_ALIGNED=$ff
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 32768 --K 24 --steps 720 --out $OUT/r32_${ff}_$rep.json > $OUT/r32_${ff}_$rep.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 65536 --K 24 --steps 240 --out $OUT/r65_${ff}_$rep.json > $OUT/r65_${ff}_$rep.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 0 --K 24 --steps 240 --out $OUT/r101_${ff}_$rep.json > $OUT/r101_${ff}_$rep.log 2>&1 || exit $?
done
done
unset RMA_FRAME_ALIGNED
python - <<'PY'
import json
for rep in (1, 2):
    for ff in (0, 1):
        for t in ("r32", "r65", "r101"):
            d = json.load(open(f"gpurun_out/r2zl/{t}_{ff}_{rep}.json"))
            runs = d["variants"]["perf_hide"]["runs"]
            o = min(r["ms_per_step"] for r in runs if not r["periodic_rccl_self"])
            p = min(r["ms_per_step"] for r in runs if r["periodic_rccl_self"])
            ps = [r for r in runs if r["periodic_rccl_self"]][0]["pass_split_ms"]
            print(rep, "aligned" if ff else "strips", t, round(o, 5), round(p, 5), "%.2f%%" % (100 * (p / o - 1)), "frame", round(ps["frame_ms"], 2), "halo", round(ps["halo_ms"], 2))
PY
