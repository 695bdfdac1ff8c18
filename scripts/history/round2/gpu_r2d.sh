#!/bin/bash
# r2: driver-command bench (planner: one 20-step pass), full GPU suite, smoke,
# and a rocprofv3 kernel trace of the driver command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=gpurun_out/r2d
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-400
  return $rc
}
step bench_20_5 300 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/bench_20_5.json &&
step bench_default 300 python bench.py --json-out $OUT/bench_default.json &&
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$OUT/trace" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 \
    > "$R/$OUT/trace.log" 2>&1; rc=$?; echo "== trace rc=$rc"; exit $rc)
