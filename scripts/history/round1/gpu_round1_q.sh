set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q
export HSA_ENABLE_IPC_MODE_LEGACY=0
b() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/q/$name.log 2>&1; rc=$?; echo "$name: $(grep -o '"value": [0-9.]*' gpurun_out/q/$name.log) single=$(grep -o '"teff_single_step_kernel_GBps": [0-9.a-z]*' gpurun_out/q/$name.log)"; return $rc; }
b t1_ol2 --temporal 1 --steps 200 && b t1_ol12 --temporal 1 --overlap 12 --steps 200 && b t6 --temporal 6 --steps 300 && b t1_ol2_again --temporal 1 --steps 200 && b t6_perf --temporal 6 --variant perf --steps 300
