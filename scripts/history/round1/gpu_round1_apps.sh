set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/apps
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/apps/$name.log 2>&1; rc=$?; echo "== $name rc=$rc"; grep -E "Executed|maximum|recv_mesg|Global grid|Warning|Error" gpurun_out/apps/$name.log | head -6; case $rc in 0|1|2) ;; *) exit $rc;; esac; }
run ap      python -m rocm_mpi_amd.apps.diffusion_2D_ap --outdir gpurun_out/apps
run ap_cpu  python -m rocm_mpi_amd.apps.diffusion_2D_ap --device cpu --preset ap256_cpu --outdir gpurun_out/apps
run kp      python -m rocm_mpi_amd.apps.diffusion_2D_kp --outdir gpurun_out/apps
run kp_graph python -m rocm_mpi_amd.apps.diffusion_2D_kp --graph --no-vis
run perf_128 python -m rocm_mpi_amd.apps.diffusion_2D_perf --nx 128 --ny 128 --no-vis
run perf_128_graph python -m rocm_mpi_amd.apps.diffusion_2D_perf --nx 128 --ny 128 --no-vis --graph
run perf    python -m rocm_mpi_amd.apps.diffusion_2D_perf
run perf_hide python -m rocm_mpi_amd.apps.diffusion_2D_perf_hide --vis --outdir gpurun_out/apps
run perf_hide_prof python -m rocm_mpi_amd.apps.diffusion_2D_perf_hide_prof
run kp16k   python -m rocm_mpi_amd.apps.diffusion_2D_kp --preset kp16k --no-vis
run smoke_ring python -m rocm_mpi_amd.apps.rocmaware_test_selectdevice
run cpp_example ./build/examples/diffusion_2D_perf_hide 12288 1000 1
ls gpurun_out/apps
cp prof.txt gpurun_out/apps/prof.txt 2>/dev/null || true
echo done
