#!/bin/bash
# r2 experiment: K=28 passes (4 stages of 7 levels, 228 VGPRs, 2 blocks/CU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2s
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u - > $OUT/bitwise.log 2>&1 <<'PY' || { cat $OUT/bitwise.log; exit 1; }
import torch
from rocm_mpi_amd import ops
c = ops.StencilCoef(-1.3, 1 / 0.037, 1 / 0.041, 0.00031)
for nx in (516, 1030):
    ny = 151
    g = torch.Generator().manual_seed(nx)
    T = torch.rand((ny, nx), generator=g, dtype=torch.float64)
    iCp = 0.5 + 0.5 * torch.rand((ny, nx), generator=g, dtype=torch.float64)
    r = [ops.interior_rect(nx, ny)]
    ref = torch.full_like(T, -5.0)
    ops.stencilk_step(28, ref, T, iCp, c, r, ops.StencilTuning(kernel="pipe"))
    out = torch.full((ny, nx), -5.0, dtype=torch.float64, device="cuda")
    ops.stencilk_step(28, out, T.cuda(), iCp.cuda(), c, r, ops.StencilTuning(kernel="pipe", vec=4, chunk_rows=37, xcd_remap=1))
    print(nx, torch.equal(out.cpu(), ref))
PY
cat $OUT/bitwise.log
timeout -k 10 600 python -u bench/pass_sweep.py --rounds 3 --pipe 16,20,24,28 --chunks 28:1536/6144 --pipec "" --ldsdpp "" --old= --alt= --out $OUT/sweep.json > $OUT/sweep.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.load(open("gpurun_out/r2s/sweep.json"))
for r in d["rows"]:
    print(r["kernel"], r["K"], r["chunk_rows"], r["ms_per_pass"], r["ms_per_step"])
PY
