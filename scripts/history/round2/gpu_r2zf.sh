#!/bin/bash
# (experiment record: RMA_FRAME_TUNE was removed after this run; the kept tuning is "64")
# r2 experiment: frame tunings A/B (RMA_FRAME_TUNE) by the RCCL-self halo overhead, K=24
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zf
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for ft in old new 64 256 1024; do
  for n in 0 16384; do
    S=240; [ $n = 16384 ] && S=2400
    if [ $ft = new ]; then unset RMA_FRAME_TUNE; else export RMA_FRAME_TUNE=$ft; fi
    timeout -k 10 300 python -u bench/rccl_self_overhead.py --n $n --K 24 --steps $S --out $OUT/r_${ft}_$n.json > $OUT/r_${ft}_$n.log 2>&1 || exit $?
  done
done
unset RMA_FRAME_TUNE
python - <<'PY'
import json
for ft in ("old", "new", "64", "256", "1024"):
    for n in (0, 16384):
        d = json.load(open(f"gpurun_out/r2zf/r_{ft}_{n}.json"))
        runs = d["variants"]["perf_hide"]["runs"]
        o = [r["ms_per_step"] for r in runs if not r["periodic_rccl_self"]]
        p = [r for r in runs if r["periodic_rccl_self"]]
        print(ft, n, "open", round(min(o), 5), "periodic", round(min(r["ms_per_step"] for r in p), 5),
              "overhead %.2f%%" % (100 * (min(r["ms_per_step"] for r in p) / min(o) - 1)),
              "frame_ms", round(p[0]["pass_split_ms"]["frame_ms"], 3))
PY
