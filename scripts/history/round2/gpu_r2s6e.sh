#!/bin/bash
# r2: perf_hide frames only on sides with a neighbour (vs RMA_FRAME_SIDES=all, the previous
# layout): GPU suite, then RCCL-self halo overhead with one dimension periodic (the two
# x-neighbours of a middle rank of a 4x1 row / the y pair), 288 GB tile and 16384^2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s6e
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"overhead": [-0-9.e]*' "$OUT/$name.log" | tr '\n' ' '; tail -2 "$OUT/$name.log" | cut -c1-200
  return $rc
}
step pytest_mr 300 python -u -m pytest tests/test_multirank_gpu.py -m gpu -q --timeout 120 --timeout-method thread ; step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ;
RMA_FRAME_SIDES=all step x101k_all_1 300 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --out $OUT/x101k_all_1.json &&
step x101k_nb_1 300 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --out $OUT/x101k_nb_1.json &&
RMA_FRAME_SIDES=all step x101k_all_2 300 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --out $OUT/x101k_all_2.json &&
step x101k_nb_2 300 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic x --out $OUT/x101k_nb_2.json &&
RMA_FRAME_SIDES=all step y101k_all 300 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic y --out $OUT/y101k_all.json &&
step y101k_nb 300 python -u bench/rccl_self_overhead.py --K 24 --steps 240 --periodic y --out $OUT/y101k_nb.json &&
RMA_FRAME_SIDES=all step x16k_all 300 python -u bench/rccl_self_overhead.py --n 16384 --K 24 --steps 960 --periodic x --out $OUT/x16k_all.json &&
step x16k_nb 300 python -u bench/rccl_self_overhead.py --n 16384 --K 24 --steps 960 --periodic x --out $OUT/x16k_nb.json &&
RMA_FRAME_SIDES=all step x16k1_all 300 python -u bench/rccl_self_overhead.py --n 16384 --K 1 --steps 400 --periodic x --out $OUT/x16k1_all.json &&
step x16k1_nb 300 python -u bench/rccl_self_overhead.py --n 16384 --K 1 --steps 400 --periodic x --out $OUT/x16k1_nb.json
