set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/y
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_guard_bands_gpu.py -x -q > gpurun_out/y/pytest.log 2>&1; rc=$?
tail -1 gpurun_out/y/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/y/$name.log 2>&1; rc=$?; echo "== $name rc=$rc $(grep -E 'Executed' gpurun_out/y/$name.log | tail -1)"; [ $rc -eq 0 ]; }
run perf128_k1 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nx 128 --ny 128 && \
run perf128_k8 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nx 128 --ny 128 --temporal 8 && \
run perf1024_k1 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nx 1024 --ny 1024 && \
run perf1024_k8 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nx 1024 --ny 1024 --temporal 8 && \
run perf4096_k8 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nx 4096 --ny 4096 --temporal 8 && \
run perf4096_k1 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nx 4096 --ny 4096 && \
run ap128 python -m rocm_mpi_amd.apps.diffusion_2D_ap --no-vis && \
run ap128_graph python -m rocm_mpi_amd.apps.diffusion_2D_ap --no-vis --graph && \
run ap256_gpu_graph python -m rocm_mpi_amd.apps.diffusion_2D_ap --no-vis --graph --nx 256 --ny 256
