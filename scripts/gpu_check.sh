#!/bin/bash
# One-GPU validation + measurement pass (run on the GPU box, e.g.
#   gpurun --timeout 1200 -- bash scripts/gpu_check.sh):
# GPU test suite, smoke(), default bench (16 fast-math steps/pass at the 288 GB tile, also
# reporting the one-step kernel), the BASELINE presets that fit one GPU, and a
# rocprofv3 kernel trace of a short bench. Every GPU step has its own time
# limit; the script stops at the first failure, fault or timeout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=${OUT:-gpurun_out/check}
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-240
  return $rc
}
step pytest_gpu 700 python -m pytest tests -m gpu -x -q &&
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench 400 python bench.py --json-out "$OUT/bench.json" &&
step baseline_presets 400 python bench/baseline_configs.py --max-gpus 1 --out "$OUT/baseline_configs.json" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$R/$OUT/trace" -o run -- python3 "$R/bench.py" --steps 120 --single-step-steps 24 \
    > "$R/$OUT/trace.log" 2>&1; rc=$?; echo "== trace rc=$rc"; exit $rc)
