"""C2's CWT at the per-rank batch of a 1/2/4/8-GPU strong-scaling run (diagnostic): the time
per step and the HBM rate for B = 1024 / 512 / 256 / 128 series on one GPU."""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import _lib, ops  # noqa: E402

n, dt, dj = 4096, 1 / 12, 1 / 12
sj = 2 * dt * 2 ** (np.arange(128) * dj)


def timed(x, out):
    for _ in range(100):
        ops.cwt_morlet(x, sj, dt, out_w=out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        ops.cwt_morlet(x, sj, dt, out_w=out)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 50


for B in [int(a) for a in sys.argv[1:]] or (1024, 512, 256, 128):
    x = torch.randn(B, n, device="cuda")
    out = torch.empty((B, 128, n), dtype=torch.complex64, device="cuda")
    gb = B * 128 * n * 8 / 1e9 + B * n * 4 / 1e9
    for wg in (0, 256, 384, 512, 768, 1024, 1536):
        with _lib.option("cwt_target_wg", wg):
            ms = timed(x, out)
        print(f"B={B:5d} target_wg={wg:5d} {ms:.4f} ms  {gb / ms:.2f} TB/s", flush=True)
    del x, out
