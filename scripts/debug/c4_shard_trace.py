"""C4 at one rank's shard (B pairs) for a kernel trace: python scripts/debug/c4_shard_trace.py B ITERS"""
import sys

import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import ops, transforms  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 30
n, dt, dj = 8192, 1 / 12, 1 / 8
sj, _ = transforms.scales_for(n, dt, dj, 2 * dt, -1, transforms.Morlet(6))
K = transforms.boxcar_rows(transforms.Morlet(6), dj)
x1 = torch.randn(B, n, device="cuda").cumsum(1)
x2 = torch.randn(B, n, device="cuda").cumsum(1)
ws = torch.empty(ops.wct_workspace_bytes(B, n, len(sj)), dtype=torch.uint8, device="cuda")
for _ in range(iters):
    transforms.wct_batch(x1, x2, dt, dj, 2 * dt, -1, workspace=ws, want_uv=False, want_power=True,
                         want_phase=True)
torch.cuda.synchronize()
