#!/bin/bash
# One-time environment bootstrap (counterpart of the reference's startup.sh,
# which creates a Julia project, binds MPI.jl to the system MPI and builds
# ImplicitGlobalGrid/AMDGPU). Here: check the toolchain, build the native core
# for gfx950 in-tree and verify that the package and its extension import.
#   ./scripts/startup.sh            # srun -n 1 ./startup.sh analogue
set -eo pipefail
cd "$(dirname "$0")/.."
source scripts/setenv.sh
command -v hipcc >/dev/null || { echo "hipcc not found under $ROCM_PATH/bin" >&2; exit 1; }
python - <<'EOF'
import torch
print(f"torch {torch.__version__} (HIP {torch.version.hip}), "
      f"{torch.cuda.device_count()} visible device(s)")
assert torch.version.hip, "a ROCm build of PyTorch is required"
EOF
python -m rocm_mpi_amd._build
python - <<'EOF'
import rocm_mpi_amd
from rocm_mpi_amd._native import native, native_path
n = native()
print(f"rocm_mpi_amd native core {native_path()} (RCCL {n.rccl_version()}): OK")
EOF
