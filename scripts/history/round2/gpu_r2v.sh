#!/bin/bash
# (experiment record: the pipem kernel variant was removed after this run, profiles/SUMMARY_r2.md)
# r2 experiment: EXEC-masking lanes with no valid cell per level (pipem) vs pipe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2v
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u - > $OUT/bitwise.log 2>&1 <<'PY' || { cat $OUT/bitwise.log; exit 1; }
import torch
from rocm_mpi_amd import ops
c = ops.StencilCoef(-1.3, 1 / 0.037, 1 / 0.041, 0.00031)
ok = True
for K in (16, 20, 24):
    for nx, vec in ((516, 4), (1030, 2), (777, 4)):
        ny = 151
        g = torch.Generator().manual_seed(nx + K)
        T = torch.rand((ny, nx), generator=g, dtype=torch.float64)
        iCp = 0.5 + 0.5 * torch.rand((ny, nx), generator=g, dtype=torch.float64)
        for r in ([ops.interior_rect(nx, ny)], [(K + 3, nx - K - 5, 2, ny - 9), (1, K + 3, 1, ny - 1)]):
            ref = torch.full_like(T, -5.0)
            ops.stencilk_step(K, ref, T, iCp, c, r, ops.StencilTuning(kernel="pipe"))
            out = torch.full((ny, nx), -5.0, dtype=torch.float64, device="cuda")
            ops.stencilk_step(K, out, T.cuda(), iCp.cuda(), c, r, ops.StencilTuning(kernel="pipem", vec=vec, chunk_rows=37, xcd_remap=1))
            e = torch.equal(out.cpu(), ref)
            ok &= e
            print(K, nx, vec, e)
print("ALL", ok)
PY
tail -1 $OUT/bitwise.log
timeout -k 10 600 python -u bench/pass_sweep.py --rounds 5 --pipe 16,20,24 --old pipem:16,pipem:20,pipem:24 --pipec "" --ldsdpp "" --alt= --out $OUT/sweep_101k.json > $OUT/sweep_101k.log 2>&1 || exit $?
timeout -k 10 600 python -u bench/pass_sweep.py --n 16384 --rounds 7 --pipe 16,20,24 --old pipem:16,pipem:20,pipem:24 --pipec "" --ldsdpp "" --alt= --out $OUT/sweep_16k.json > $OUT/sweep_16k.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/r2v/sweep_101k.json", "gpurun_out/r2v/sweep_16k.json"):
    d = json.load(open(f))
    print(f)
    for r in d["rows"]:
        print(" ", r["kernel"], r["K"], r["ms_per_pass"], r["ms_min"])
PY
timeout -k 10 300 python -u bench/power_probe.py --configs pipe:24,pipem:24,pipe:20,pipem:20 --seconds 6 --out $OUT/power.json > $OUT/power.log 2>&1 || exit $?
grep '^{"kernel' $OUT/power.log
