#!/bin/bash
# PMC of fast5 (V=2) vs fast5p4 (V=4) at K=16, 101376^2: stall breakdown.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
OUT=$R/gpurun_out/pmc_p4; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export RMA_PROBE_SET=fast RMA_PROBE_N=101376 RMA_PROBE_REPS=2 RMA_PROBE_K=16 RMA_PROBE_KERNELS=fast5,fast5p4
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS \
    --output-format csv -d $OUT/sq -o run -- python3 $R/bench/pmc_probe.py > $OUT/sq.log 2>&1 && echo "== sq ok" &&
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/sq2 -o run -- python3 $R/bench/pmc_probe.py > $OUT/sq2.log 2>&1 && echo "== sq2 ok"
