#!/bin/bash
# r2 experiments: non-temporal T/1/Cp loads (pipentl), no sched_barrier (pipensb); both removed after this run (slower)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2zv
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u - > $OUT/bitwise.log 2>&1 <<'PY' || { cat $OUT/bitwise.log; exit 1; }
import torch
from rocm_mpi_amd import ops
c = ops.StencilCoef(-1.3, 1 / 0.037, 1 / 0.041, 0.00031)
ok = True
for kern in ("pipentl", "pipensb"):
    for K in (20, 24):
        for nx, vec in ((516, 4), (1030, 2)):
            ny = 151
            g = torch.Generator().manual_seed(nx + K)
            T = torch.rand((ny, nx), generator=g, dtype=torch.float64)
            iCp = 0.5 + 0.5 * torch.rand((ny, nx), generator=g, dtype=torch.float64)
            r = [ops.interior_rect(nx, ny)]
            ref = torch.full_like(T, -5.0)
            ops.stencilk_step(K, ref, T, iCp, c, r, ops.StencilTuning(kernel="pipe"))
            out = torch.full((ny, nx), -5.0, dtype=torch.float64, device="cuda")
            ops.stencilk_step(K, out, T.cuda(), iCp.cuda(), c, r, ops.StencilTuning(kernel=kern, vec=vec, chunk_rows=37, xcd_remap=1))
            ok &= torch.equal(out.cpu(), ref)
print("ALL", ok)
PY
tail -1 $OUT/bitwise.log
for rep in 1 2; do
timeout -k 10 600 python -u bench/pass_sweep.py --rounds 5 --pipe 20,24 --old pipentl:20,pipentl:24,pipensb:20,pipensb:24 --pipec "" --ldsdpp "" --alt= --out $OUT/s101_$rep.json > $OUT/s101_$rep.log 2>&1 || exit $?
timeout -k 10 600 python -u bench/pass_sweep.py --n 16384 --rounds 9 --pipe 20,24 --old pipentl:20,pipentl:24,pipensb:20,pipensb:24 --pipec "" --ldsdpp "" --alt= --out $OUT/s16_$rep.json > $OUT/s16_$rep.log 2>&1 || exit $?
done
python - <<'PY'
import json
for rep in (1, 2):
    for t in ("s101", "s16"):
        d = json.load(open(f"gpurun_out/r2zv/{t}_{rep}.json"))
        print(rep, t, [(r["kernel"], r["K"], r["ms_per_pass"]) for r in d["rows"] if r["kernel"] not in ("march", "two_step")])
PY
