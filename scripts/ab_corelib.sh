#!/bin/bash
# A/B of alternative builds of the native core (librma_core_<tag>.so.alt next to
# the package): each variant in turn replaces librma_core.so for one process of
# bench/pass_sweep.py (the executor's K=20 and K=24 kernels on the 288 GB tile), ROUNDS times in
# alternation; the original library is restored at the end.
set -eo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/ab_corelib}
mkdir -p "$OUT"
export RMA_AUTOBUILD=0
PKG=rocm_mpi_amd
cp $PKG/librma_core.so "$OUT/librma_core.orig"
trap 'cp "$OUT/librma_core.orig" $PKG/librma_core.so' EXIT
for r in $(seq 1 "${ROUNDS:-2}"); do
  for v in ${VARIANTS:-base ilp iter}; do
    cp "$PKG/librma_core_$v.so.alt" $PKG/librma_core.so
    timeout -k 10 240 python3 bench/pass_sweep.py --pipe "" --exec "${EXEC:-20,24}" --pipec "${PIPEC:-}" --ldsdpp "" \
        --old "" --alt "" --rounds 3 --out "$OUT/sweep_${v}_$r.json" > "$OUT/sweep_${v}_$r.log" 2>&1
    echo "round $r variant $v done"
  done
done
