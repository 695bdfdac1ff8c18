#!/bin/bash
# r2: aligned frames with capped band height (RMA_FRAME_ALIGNED=0 strips | <band rows>) at 101376^2 / 16384^2, K=24
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zm
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
for ff in 0 256 1024 3072; do
  export RMA_FRAME_ALIGNED=$ff
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 0 --K 24 --steps 240 --out $OUT/r101_${ff}_$rep.json > $OUT/r101_${ff}_$rep.log 2>&1 || exit $?
done
done
for ff in 0 256 512; do
  export RMA_FRAME_ALIGNED=$ff
  timeout -k 10 300 python -u bench/rccl_self_overhead.py --n 16384 --K 24 --steps 2400 --out $OUT/r16_${ff}_1.json > $OUT/r16_${ff}_1.log 2>&1 || exit $?
done
unset RMA_FRAME_ALIGNED
python - <<'PY'
import json, os
for f in sorted(os.listdir("gpurun_out/r2zm")):
    if not f.endswith(".json"):
        continue
    d = json.load(open(f"gpurun_out/r2zm/{f}"))
    runs = d["variants"]["perf_hide"]["runs"]
    o = min(r["ms_per_step"] for r in runs if not r["periodic_rccl_self"])
    p = min(r["ms_per_step"] for r in runs if r["periodic_rccl_self"])
    ps = [r for r in runs if r["periodic_rccl_self"]][0]["pass_split_ms"]
    print(f, round(o, 5), round(p, 5), "%.2f%%" % (100 * (p / o - 1)), "frame", round(ps["frame_ms"], 2), "halo", round(ps["halo_ms"], 2))
PY
