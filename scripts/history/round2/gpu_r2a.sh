set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r2a
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2a/bench_20_5.log 2>&1 && echo bench ok &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/r2a/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/r2a/trace.log" 2>&1) && echo trace ok
