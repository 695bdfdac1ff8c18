#!/bin/bash
# PMC passes over the fast-math K=8 kernels (kernel 4 vs 5) on the 288 GB tile.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../../.." && pwd)}"
OUT=$R/gpurun_out/pmc_fast5; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export RMA_PROBE_SET=fast RMA_PROBE_N=${N:-101376} RMA_PROBE_REPS=2
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- \
      python3 $R/bench/pmc_probe.py > $OUT/$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"; return $rc
}
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE &&
pass tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
