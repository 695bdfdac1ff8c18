#!/bin/bash
# r2: PMC of the pipelined fast5 passes K=16 / 20 / 24 at 101376^2 (two counter
# passes, each within the per-block limits: <= 8 SQ + GRBM)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=$R/gpurun_out/r2e; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SW="$R/bench/pass_sweep.py --pipe 16,20,24 --pipec 16 --ldsdpp 8 --old fast5p4:16 --alt 24:8 --rounds 1"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/a -o run -- python3 $SW > $OUT/a.log 2>&1 && echo "== a ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INSTS_BRANCH GRBM_COUNT \
    --output-format csv -d $OUT/b -o run -- python3 $SW > $OUT/b.log 2>&1 && echo "== b ok"
