#!/bin/bash
# PMC counters of the piper kernel for alternative builds of the native core
# (librma_core_<tag>.so.alt, see scripts/ab_corelib.sh): one rocprofv3 --pmc
# run per build (counters only with --kernel-trace), original restored at exit.
set -eo pipefail
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=${OUT:-gpurun_out/pmc_corelib}
mkdir -p "$OUT"
export RMA_AUTOBUILD=0 RMA_PROBE_SET=piper RMA_PROBE_N=${N:-65536} RMA_PROBE_K=${K:-20} RMA_PROBE_REPS=2
PKG=rocm_mpi_amd
cp $PKG/librma_core.so "$OUT/librma_core.orig"
trap 'cp "$ROOT/$OUT/librma_core.orig" "$ROOT/$PKG/librma_core.so"' EXIT
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
for v in ${VARIANTS:-base r20}; do
  cp "$PKG/librma_core_$v.so.alt" $PKG/librma_core.so
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
      SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
      -d "$OUT/$v" -o run -- python3 bench/pmc_probe.py > "$OUT/$v.log" 2>&1
  echo "variant $v done"
done
