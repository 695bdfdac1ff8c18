#!/bin/bash
# Per-job entry (counterpart of the reference's scripts/runme.sh): pick the
# variant by argument instead of (un)commenting lines.
#   ./scripts/runme.sh 4 perf_hide --nx 16384      # 4 ranks, one per GPU
set -e
cd "$(dirname "$0")/.."
source scripts/setenv.sh
N=${1:-1}; VARIANT=${2:-ap}; shift 2 || true
python -m rocm_mpi_amd._build
exec python -m rocm_mpi_amd.launch -n "$N" -m "rocm_mpi_amd.apps.diffusion_2D_${VARIANT}" -- "$@"
