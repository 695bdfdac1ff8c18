"""Time the x-halo pack / unpack of a width-K fp64 plane at the 288 GB tile
(101376 rows, K = 16 columns, row stride 811 KB) and the same copy as a flat
contiguous memcpy of equal bytes, for the multi-rank overhead budget."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch  # noqa: E402

from rocm_mpi_amd import ops  # noqa: E402

n, K = int(os.environ.get("N", "101376")), int(os.environ.get("K", "16"))
T = torch.empty((n, n), dtype=torch.float64, device="cuda")
ops.fill_(T, 1.0)
buf = torch.empty((n, K), dtype=torch.float64, device="cuda")
flat = torch.empty(n * K, dtype=torch.float64, device="cuda")
flat2 = torch.empty_like(flat)


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


res = {"rows": n, "K": K, "bytes": n * K * 8,
       "pack_us": t(lambda: ops.copy_plane(buf, T[:, K:2 * K])),
       "unpack_us": t(lambda: ops.copy_plane(T[:, n - K:], buf)),
       "flat_copy_us": t(lambda: flat2.copy_(flat))}
print(json.dumps(res))
