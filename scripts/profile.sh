#!/bin/bash
# rocprofv3 recipes (run on the GPU box). Kernel trace + stats of a bench run,
# then PMC passes (one counter family per pass; never combined with sys/runtime
# traces) for the per-dispatch HBM bytes of the stencil vs the T_eff model.
set -eo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/prof}
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --nx ${NX:-16384} --steps ${STEPS:-100} --warmup 5
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench/pmc_probe.py
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench/pmc_probe.py
