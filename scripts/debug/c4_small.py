"""C4 at one 8-GPU shard (64 pairs) for a rocprofv3 kernel trace (diagnostic)."""
import sys

import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import ops, transforms  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
n, dt, dj = 8192, 1 / 12, 1 / 8
sj, _ = transforms.scales_for(n, dt, dj, 2 * dt, -1, transforms.Morlet(6))
K = transforms.boxcar_rows(transforms.Morlet(6), dj)
x1 = torch.randn(B, n, device="cuda").cumsum(1)
x2 = torch.randn(B, n, device="cuda").cumsum(1)
ws = torch.empty(ops.wct_workspace_bytes(B, n, len(sj)), dtype=torch.uint8, device="cuda")
for _ in range(30):
    ops.wct_morlet(x1, x2, sj, dt, 6.0, boxcar=K, want_uv=False, workspace=ws, want_power=True, want_phase=True)
torch.cuda.synchronize()
print("ok")
