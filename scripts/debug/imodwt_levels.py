"""MODWT synthesis / analysis time against the level count J (C3 shape, diagnostic).

T(J) - T(J-1) is the cost of one more cascade level plus one more row; small batches show
the same with the rows (mostly) resident in the 256 MB MALL.
"""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import ops  # noqa: E402

lo = np.array([-0.010597401784997278, 0.032883011666982945, 0.030841381835986965,
               -0.18703481171888114, -0.02798376941698385, 0.6308807679295904,
               0.7148465705525415, 0.23037781330885523])
hi = np.array([(-1) ** (k + 1) * lo[7 - k] for k in range(8)])
n = 16384


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for B in [int(a) for a in (sys.argv[1:] or ["8192", "512", "256"])]:
    x = torch.randn(B, n, device="cuda")
    prev_s = prev_a = 0.0
    for J in range(1, 11):
        w = ops.modwt(x, lo, hi, J)
        out = torch.empty_like(x)
        ta = timed(lambda: ops.modwt(x, lo, hi, J, out=w))
        ts = timed(lambda: ops.imodwt(w, lo, hi, out=out))
        gb = B * n * 4 * (J + 2) / 1e9
        print(f"B={B} J={J:2d} analysis {ta:.4f} ms (+{ta - prev_a:.4f})  synthesis {ts:.4f} ms "
              f"(+{ts - prev_s:.4f})  syn {gb / ts:.2f} TB/s", flush=True)
        prev_s, prev_a = ts, ta
        del w, out
    del x
    torch.cuda.empty_cache()
