#!/bin/bash
# r2: pipeb (ds_bpermute lane moves) correctness + power / clock of the deep passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2h
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "$OUT/$name.log" | cut -c1-300
  return $rc
}
rocm-smi --showpower --showclocks --showmaxpower > $OUT/smi_idle.txt 2>&1
step pytest_pipe 600 python -u -m pytest tests/test_pipe_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider &&
step power 400 python -u bench/power_probe.py --configs march:1,pipe:16,pipe:20,pipe:24,pipeb:16,pipeb:20,pipeb:24,pipe:12,pipe:8 --seconds 6 --out $OUT/power.json
