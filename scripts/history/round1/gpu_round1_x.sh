set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/x
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/x/pytest.log 2>&1; rc=$?
tail -1 gpurun_out/x/pytest.log; [ $rc -eq 0 ] || exit $rc
run() { name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/x/$name.log 2>&1; rc=$?; echo "== $name rc=$rc $(grep -E 'Executed' gpurun_out/x/$name.log | tail -1)"; [ $rc -eq 0 ]; }
run cpp_k1 ./build/examples/diffusion_2D_perf_hide 16384 1000 1 1 && \
run cpp_k8 ./build/examples/diffusion_2D_perf_hide 16384 1000 1 8 && \
run perf_k8 python -m rocm_mpi_amd.apps.diffusion_2D_perf --temporal 8 && \
run perf_hide_k8 python -m rocm_mpi_amd.apps.diffusion_2D_perf_hide --temporal 8 --vis --outdir gpurun_out/x && \
run perf_hide_k1 python -m rocm_mpi_amd.apps.diffusion_2D_perf_hide --vis --outdir gpurun_out/x/k1 && \
run perf_hide_prof_k6 python -m rocm_mpi_amd.apps.diffusion_2D_perf_hide_prof --temporal 6
