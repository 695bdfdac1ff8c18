#!/bin/bash
# r2: bench.py T_eff vs local tile size (1 GPU, 1000 steps, K<=24 fast-math passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zp
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2048 4096 8192 12288 16384 24576 32768 49152 65536; do
  timeout -k 10 300 python -u bench.py --nx $n --steps 1000 --warmup 48 --single-step-steps 20 --json-out $OUT/b_$n.json > $OUT/b_$n.log 2>&1 || exit $?
  echo "== $n"
done
python - <<'PY'
import json
for n in (2048, 4096, 8192, 12288, 16384, 24576, 32768, 49152, 65536):
    d = json.load(open(f"gpurun_out/r2zp/b_{n}.json"))
    c = d["config"]
    print(n, d["value"], d["ms_per_step"], c["teff_single_step_kernel_GBps"], c["kstep_kernel"]["chunk_rows"], c["passes_timed"][:2], len(c["passes_timed"]))
PY
