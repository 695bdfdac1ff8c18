#!/bin/bash
# r2: BASELINE presets on 1 GPU, sustained 6000-step bench, canonical (bitwise) bench, app path
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2r
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u bench/baseline_configs.py --max-gpus 1 --out $OUT/baseline_configs.json > $OUT/baseline.log 2>&1 || { tail -20 $OUT/baseline.log; exit 1; }
echo "== presets ok"
timeout -k 10 300 python -u bench.py --steps 6000 --warmup 24 --single-step-steps 0 --solo-steps 240 --json-out $OUT/bench_6000.json > $OUT/bench_6000.log 2>&1 || exit $?
tail -1 $OUT/bench_6000.log | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 1000 --no-fast-math --temporal 12 --single-step-steps 0 --json-out $OUT/bench_canonical.json > $OUT/bench_canonical.log 2>&1 || exit $?
tail -1 $OUT/bench_canonical.log | cut -c1-200
timeout -k 10 300 python -u -m rocm_mpi_amd.launch -n 1 -m rocm_mpi_amd.apps.diffusion_2D_perf_hide -- --nx 16384 --ny 16384 --nt 1000 --temporal 24 --fast-math --init random --no-vis --json --quiet > $OUT/app_hide16k.log 2>&1 || exit $?
tail -2 $OUT/app_hide16k.log | cut -c1-300
