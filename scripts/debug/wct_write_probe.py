"""C4 shapes with different output sets, for a WRITE_SIZE pass (which kernel writes what):
python scripts/debug/wct_write_probe.py MODE   (MODE: both | power | none)"""
import sys

import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import transforms  # noqa: E402

mode = sys.argv[1]
B, n, dt, dj = 512, 8192, 1 / 12, 1 / 8
g = torch.Generator(device="cuda").manual_seed(3)
x1 = torch.randn(B, n, device="cuda", generator=g).cumsum(1)
x2 = torch.randn(B, n, device="cuda", generator=g).cumsum(1)
for _ in range(3):
    transforms.wct_batch(x1, x2, dt, dj, 2 * dt, -1, want_uv=False, want_power=mode != "none",
                         want_phase=mode == "both")
torch.cuda.synchronize()
