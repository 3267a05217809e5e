"""C3 and C4 at the per-rank batch of a 1/2/4/8-GPU strong-scaling run (diagnostic): time per
step on one GPU for the global batch divided by 1, 2, 4, 8, with a few launch options."""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import _lib, ops, transforms  # noqa: E402
from wtmi.wavelets import Wavelet  # noqa: E402


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


which = sys.argv[1] if len(sys.argv) > 1 else "c4"
if which == "c4":
    n, dt, dj = 8192, 1 / 12, 1 / 8
    sj, _ = transforms.scales_for(n, dt, dj, 2 * dt, -1, transforms.Morlet(6))
    K = transforms.boxcar_rows(transforms.Morlet(6), dj)
    for B in [int(a) for a in sys.argv[2:]] or (512, 256, 128, 64):
        x1 = torch.randn(B, n, device="cuda").cumsum(1)
        x2 = torch.randn(B, n, device="cuda").cumsum(1)
        ws = torch.empty(ops.wct_workspace_bytes(B, n, len(sj)), dtype=torch.uint8, device="cuda")
        for opts in ({}, {"wct_min_rows": 4, "wct_dec_rows": 4}, {"wct_min_rows": 2, "wct_dec_rows": 2},
                     {"wct_min_rows": 1, "wct_dec_rows": 2}):
            ctx = [_lib.option(k, v) for k, v in opts.items()]
            for c in ctx:
                c.__enter__()
            ms = timed(lambda: ops.wct_morlet(x1, x2, sj, dt, 6.0, boxcar=K, want_uv=False, workspace=ws,
                                              want_power=True, want_phase=True))
            for c in reversed(ctx):
                c.__exit__(None, None, None)
            print(f"C4 B={B:4d} {opts} {ms:.4f} ms  (x{512 // B} = {ms * 512 / B:.3f})", flush=True)
        del x1, x2, ws
else:
    w = Wavelet("db4")
    for B in (8192, 4096, 2048, 1024):
        x = torch.randn(B, 16384, device="cuda")
        out = torch.empty_like(x)

        def step():
            c = ops.modwt(x, w.dec_lo, w.dec_hi, 10)
            ops.imodwt(c, w.dec_lo, w.dec_hi, out=out)
        ms = timed(step)
        print(f"C3 B={B:5d} {ms:.4f} ms  (x{8192 // B} = {ms * 8192 / B:.3f})", flush=True)
        del x, out
