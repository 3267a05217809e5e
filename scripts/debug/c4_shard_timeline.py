"""C4 step at a strong-scaling shard's batch (default 64 pairs) repeated for a kernel trace:
    rocprofv3 --kernel-trace -d DIR -- python scripts/debug/c4_shard_timeline.py [PAIRS]
then scripts/debug/trace_timeline.py DIR wct_spectra_plan."""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import ops, transforms  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
n, dt, dj = 8192, 1 / 12, 1 / 8
sj, _ = transforms.scales_for(n, dt, dj, 2 * dt, -1, transforms.Morlet(6))
K = transforms.boxcar_rows(transforms.Morlet(6), dj)
g = torch.Generator(device="cuda").manual_seed(5)
y1 = torch.randn(B, n, device="cuda", generator=g)
y2 = 0.6 * torch.roll(y1, 3, 1) + 0.8 * torch.randn(B, n, device="cuda", generator=g)
sjd = torch.tensor(sj, device="cuda")
ws = torch.empty(ops.wct_workspace_bytes(B, n, sj.size), dtype=torch.uint8, device="cuda")
for _ in range(40):
    ops.wct_morlet(y1, y2, sjd, dt, 6.0, boxcar=K, want_uv=False, want_power=True, want_phase=True,
                   workspace=ws, normalize=True)
torch.cuda.synchronize()
print("done", B)
