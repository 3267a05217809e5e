"""Five MODWT analysis + synthesis launches at the C3 shape (for rocprofv3 PMC passes)."""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import ops  # noqa: E402

lo = np.array([-0.010597401784997278, 0.032883011666982945, 0.030841381835986965,
               -0.18703481171888114, -0.02798376941698385, 0.6308807679295904,
               0.7148465705525415, 0.23037781330885523])
hi = np.array([(-1) ** (k + 1) * lo[7 - k] for k in range(8)])
x = torch.randn(8192, 16384, device="cuda")
w = ops.modwt(x, lo, hi, 10)
out = torch.empty_like(x)
for _ in range(5):
    ops.modwt(x, lo, hi, 10, out=w)
    ops.imodwt(w, lo, hi, out=out)
torch.cuda.synchronize()
print("ok")
