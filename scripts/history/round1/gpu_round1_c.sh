set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== bench 16k perf_hide / perf / kp (defaults)"
for v in perf_hide perf kp; do
  timeout -k 10 300 python bench.py --nx 16384 --steps 1000 --warmup 10 --variant $v > gpurun_out/bench16k_$v.log 2>&1 || { echo BENCH_FAIL $v; tail -20 gpurun_out/bench16k_$v.log; exit 1; }
  tail -1 gpurun_out/bench16k_$v.log | cut -c1-400
done
echo "== bench default (auto-size, 1000 steps)"
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL default; tail -20 gpurun_out/bench_default.log; exit 1; }
cat gpurun_out/bench_default.log | cut -c1-600
echo "== trace perf_hide 16k"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hide16k -o run -- python3 bench.py --nx 16384 --steps 50 --warmup 5 > gpurun_out/prof_hide16k.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/prof_hide16k.log; exit 1; }
echo "== trace perf_hide 16k with marker trace"
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/prof_hide_markers -o run -- python3 -m rocm_mpi_amd.apps.diffusion_2D_perf_hide_prof --nx 16384 --ny 16384 --nt 40 > gpurun_out/prof_markers.log 2>&1 || { echo MARKER_FAIL; tail -20 gpurun_out/prof_markers.log; }
ls gpurun_out/prof_hide_markers
echo done
