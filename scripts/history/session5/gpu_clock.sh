#!/bin/bash
# SCLK / power while the default K=16 bench runs (explains box-to-box spread)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
OUT=${OUT:-gpurun_out/clock}
mkdir -p "$OUT"
timeout -k 10 200 python bench.py --steps 6000 --single-step-steps 0 --json-out "$OUT/bench.json" > "$OUT/bench.log" 2>&1 &
BP=$!
rocm-smi --showclocks --showpower > "$OUT/smi_idle.txt" 2>&1
for i in 1 2 3 4 5 6; do
  sleep 5
  rocm-smi --showclocks --showpower --showtemp > "$OUT/smi_$i.txt" 2>&1
done
wait $BP; rc=$?
echo "bench rc=$rc"; tail -1 "$OUT/bench.log" | cut -c1-220
grep -h -i "sclk\|power\|junction" "$OUT"/smi_*.txt | sort | uniq -c | head -20
exit $rc
