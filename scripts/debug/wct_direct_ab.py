"""WCT with and without the direct smoothing of narrow time-path rows (option wct_direct),
alternating, at several (batch, n, dj): python scripts/debug/wct_direct_ab.py"""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import _lib, transforms  # noqa: E402


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for B, n, dj in [(1, 1333, 1 / 8), (64, 1333, 1 / 8), (512, 2048, 1 / 8), (512, 4096, 1 / 12),
                 (512, 4096, 1 / 8), (512, 8192, 1 / 8)]:
    g = torch.Generator(device="cuda").manual_seed(n)
    x1 = torch.randn(B, n, device="cuda", generator=g).cumsum(1)
    x2 = torch.randn(B, n, device="cuda", generator=g).cumsum(1)

    def run():
        transforms.wct_batch(x1, x2, 1 / 12, dj, 2 / 12, -1, want_uv=False, want_power=True,
                             want_phase=True)
    for rep in range(2):
        r = []
        for d in (0, 1):
            with _lib.option("wct_direct", d):
                r.append(timed(run))
        print(f"B={B:4d} n={n:5d} dj=1/{round(1 / dj)}  direct 0: {r[0]:.4f} ms  1: {r[1]:.4f} ms", flush=True)
