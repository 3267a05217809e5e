"""A/B of the MODWT synthesis kernels (option modwt_syn) at the C3 shape (diagnostic)."""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import _lib, ops  # noqa: E402

lo = np.array([-0.010597401784997278, 0.032883011666982945, 0.030841381835986965,
               -0.18703481171888114, -0.02798376941698385, 0.6308807679295904,
               0.7148465705525415, 0.23037781330885523])
hi = np.array([(-1) ** (k + 1) * lo[7 - k] for k in range(8)])
import os
n = int(os.environ.get("N", 16384))
B = 8192 * 16384 // n
variants = [int(a) for a in (sys.argv[1:] or ["0", "1"])]


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


x = torch.randn(B, n, device="cuda")
for J in (10, 3, 1):
    w = ops.modwt(x, lo, hi, J)
    outs = {}
    for v in variants:
        out = torch.empty_like(x)
        with _lib.option("modwt_syn", v):
            t = timed(lambda: ops.imodwt(w, lo, hi, out=out))
            tm = timed(lambda: ops.imodwt(w, lo, hi, keep_mask=0b101, out=out), reps=5)
            outs[v] = (out.clone(), ops.imodwt(w, lo, hi, keep_mask=0b101))
        d = (outs[v][0] - outs[variants[0]][0]).abs().max().item()
        dm = (outs[v][1] - outs[variants[0]][1]).abs().max().item()
        rt = (outs[v][0] - x).abs().max().item()
        gb = B * n * 4 * (J + 2) / 1e9
        print(f"J={J:2d} syn={v} {t:.4f} ms {gb / t:.2f} TB/s  masked {tm:.4f} ms  "
              f"|d| {d:.2e} masked |d| {dm:.2e} round-trip {rt:.2e}", flush=True)
    del w, outs
