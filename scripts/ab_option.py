"""A/B of a launch option on one config's step, alternating in one process (rounds x values),
results checked bitwise equal across values:

    python scripts/ab_option.py c2|c3a|c3s|c4 OPTION V0 V1 [V2 ...] [--reps R]
c2: the C2 step (1024 series, or --batch); c3a: C3's analysis (8192 x 16384, J = 10); c3s: its
synthesis; c4: the C4 step (512 pairs)."""
import argparse
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import _lib, ops, transforms  # noqa: E402
from wtmi.wavelets import Wavelet  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("what")
ap.add_argument("option")
ap.add_argument("values", type=int, nargs="+")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--batch", type=int, default=512, help="c4: pairs")
a = ap.parse_args()
if a.what == "c2":
    DT = 1 / 12
    sj = torch.tensor(2 * DT * 2 ** (np.arange(128) / 12), device="cuda")
    x = torch.randn(a.batch if a.batch != 512 else 1024, 4096, device="cuda")
    out = torch.empty((x.shape[0], 128, 4096), dtype=torch.complex64, device="cuda")

    def step():
        ops.cwt_morlet(x, sj, DT, 6.0, out_w=out)
        return out
elif a.what in ("c3a", "c3s"):
    w = Wavelet("db4")
    B, n, J = 8192, 16384, 10
    x = torch.randn(B, n, device="cuda")
    W = torch.empty((B, J + 1, n), device="cuda")
    ops.modwt(x, w.dec_lo, w.dec_hi, J, out=W)
    if a.what == "c3a":
        def step():
            ops.modwt(x, w.dec_lo, w.dec_hi, J, out=W)
            return W
    else:
        def step():
            return ops.imodwt(W, w.dec_lo, w.dec_hi)
else:
    DT, n, dj = 1 / 12, 8192, 1 / 8
    sj, _ = transforms.scales_for(n, DT, dj, 2 * DT, -1, transforms.Morlet(6))
    K = transforms.boxcar_rows(transforms.Morlet(6), dj)
    rng = np.random.default_rng(1)
    y1 = torch.tensor(rng.standard_normal((a.batch, n)).cumsum(1).astype(np.float32), device="cuda")
    y2 = torch.tensor(rng.standard_normal((a.batch, n)).cumsum(1).astype(np.float32), device="cuda")
    sjd = torch.tensor(sj, device="cuda")
    ws = torch.empty(ops.wct_workspace_bytes(a.batch, n, sj.size), dtype=torch.uint8, device="cuda")

    def step():
        return ops.wct_morlet(y1, y2, sjd, DT, 6.0, boxcar=K, want_uv=False, want_power=True,
                              want_phase=True, workspace=ws, normalize=True)["coh"]
res = {v: [] for v in a.values}
ref = None
for _ in range(a.rounds):
    for v in a.values:
        with _lib.option(a.option, v):
            for _ in range(5):
                out = step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                out = step()
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.reps)
            if ref is None:
                ref = out.clone()
            elif not torch.equal(out, ref):
                print(f"{a.option}={v}: result differs from {a.values[0]}", flush=True)
for v in a.values:
    print(f"{a.what} B={a.batch if a.what == 'c4' else ''} {a.option}={v}: " + " ".join(f"{t:.4f}" for t in res[v]) + f"  min {min(res[v]):.4f} ms",
          flush=True)
