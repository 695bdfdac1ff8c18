#!/bin/bash
# r2: rocprofv3 evidence after the mirrored ring: kernel stats of the driver
# command and PMC (2 counter passes) of the K=16/20/24 passes at 101376^2
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/r2o; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --json-out $OUT/bench_20_5.json > $OUT/trace.log 2>&1 && echo "== trace ok" &&
SW="$R/bench/pass_sweep.py --pipe 16,20,24 --pipec 16 --ldsdpp 8 --old= --alt= --rounds 1" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/a -o run -- python3 $SW > $OUT/a.log 2>&1 && echo "== a ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INSTS_BRANCH GRBM_COUNT \
    --output-format csv -d $OUT/b -o run -- python3 $SW > $OUT/b.log 2>&1 && echo "== b ok"
