#!/bin/bash
# r2: pass costs per tile class with the per-tile pipe chunk table; tests; 16k/8k benches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zb
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
true
true
for n in 0 16384 8192 4096; do
  R=5; [ $n = 0 ] && R=3
  timeout -k 10 400 python -u bench/pass_sweep.py --n $n --rounds $R --pipe 1-24 --pipec 5-24 --ldsdpp 3,4,6,8 --old= --alt= --out $OUT/pass_sweep_$n.json > $OUT/sweep_$n.log 2>&1 || exit $?
  echo "== sweep $n ok"
done
exit 0
tail -1 $OUT/bench_16k.log | cut -c1-200
timeout -k 10 300 python -u bench.py --nx 8192 --steps 1000 --warmup 50 --json-out $OUT/bench_8k.json > $OUT/bench_8k.log 2>&1 || exit $?
tail -1 $OUT/bench_8k.log | cut -c1-200
