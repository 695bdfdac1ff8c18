#!/bin/bash
# r2 final tree: GPU suite, smoke(), the driver's bench command, the default bench, and the
# 1-GPU RCCL-self halo-check bench path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6k
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300
  return $rc
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench_20_5 300 python bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/bench_20_5.json &&
step bench_default 400 python bench.py --json-out $OUT/bench_default.json &&
step bench_check_self 300 python bench.py --steps 48 --warmup 24 --check 1 --check-self-rccl --json-out $OUT/bench_check_self.json
