#!/bin/bash
# Environment for rocm_mpi_amd on MI355X (counterpart of the reference's
# scripts/setenv.sh, which loads ROCm/MPI modules and toggles ROCm-aware MPI).
# There is no MPI and no module system here: one process per GPU, RCCL over
# xGMI for halos, torch.distributed for bootstrap.
export ROCM_PATH=${ROCM_PATH:-/opt/rocm}
export PATH=$ROCM_PATH/bin:$PATH
# dmabuf IPC (required by RCCL / cross-process tensor sharing on this driver)
export HSA_ENABLE_IPC_MODE_LEGACY=0
# halo transport: auto | rccl (GPU-direct, default with GPUs) | staged (host-staged,
# the reference's IGG_ROCMAWARE_MPI=0 mode) | gloo (CPU tensors)
export RMA_TRANSPORT=${RMA_TRANSPORT:-auto}
# legacy switch honoured for parity: IGG_ROCMAWARE_MPI=1 -> rccl, 0 -> staged
# export IGG_ROCMAWARE_MPI=1
export RMA_COMM_TIMEOUT=${RMA_COMM_TIMEOUT:-300}   # seconds before a stalled peer aborts the job
export PYTHONPATH=$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd):$PYTHONPATH
echo "ENV setup done"
