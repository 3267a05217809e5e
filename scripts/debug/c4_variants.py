"""C4-shaped WCT (512 pairs x 8192, dj 1/8) under launch-option / output variants, one
process: python scripts/debug/c4_variants.py [B].  Prints ms per call for each variant."""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import _lib, ops, transforms  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
n, dt, dj = 8192, 1 / 12, 1 / 8
rng = np.random.default_rng(0)
x1 = torch.tensor(rng.standard_normal((B, n)).cumsum(1), device="cuda", dtype=torch.float32)
x2 = torch.tensor(rng.standard_normal((B, n)).cumsum(1), device="cuda", dtype=torch.float32)
sj, _ = transforms.scales_for(n, dt, dj, 2 * dt, -1, transforms.Morlet(6))
K = transforms.boxcar_rows(transforms.Morlet(6), dj)
ws = torch.empty(ops.wct_workspace_bytes(B, n, len(sj)), dtype=torch.uint8, device="cuda")


def run(**kw):
    return ops.wct_morlet(x1, x2, sj, dt, 6.0, boxcar=K, want_uv=False, workspace=ws, **kw)


PP = dict(want_power=True, want_phase=True)
variants = [("pow+phase", PP, {}),
            ("coh only", dict(), {})]
variants += [(f"pow+phase dec_rows {r}", PP, {"wct_dec_rows": r}) for r in (2, 8, 16)]
variants += [(f"pow+phase min_rows {r}", PP, {"wct_min_rows": r}) for r in (2, 8)]
for rep in range(2):
    for name, kw, opts in variants:
        ctx = [_lib.option(k, v) for k, v in opts.items()]
        for c in ctx:
            c.__enter__()
        for _ in range(20):
            run(**kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run(**kw)
        e1.record()
        torch.cuda.synchronize()
        for c in reversed(ctx):
            c.__exit__(None, None, None)
        print(f"{name:24s} {e0.elapsed_time(e1) / 20:.3f} ms", flush=True)
