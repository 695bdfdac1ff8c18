#!/bin/bash
# VALU busy / waits of fast5p4 (K=16) at 101376^2 after the per-stage row loops.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
OUT=$R/gpurun_out/pmc_valu2; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export RMA_PROBE_SET=fast RMA_PROBE_N=101376 RMA_PROBE_REPS=2 RMA_PROBE_K=16 RMA_PROBE_KERNELS=fast5p4
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/a -o run -- python3 $R/bench/pmc_probe.py > $OUT/a.log 2>&1 && echo "== a ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS GRBM_COUNT \
    --output-format csv -d $OUT/b -o run -- python3 $R/bench/pmc_probe.py > $OUT/b.log 2>&1 && echo "== b ok"
