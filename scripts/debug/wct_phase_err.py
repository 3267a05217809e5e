"""Phase-output error of the WCT engine against the fp64 oracle, per row-relative amplitude
band, for each wct_prune level (diagnostic: python scripts/debug/wct_phase_err.py [n] [dj])."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
sys.path.insert(0, "wavelet-transformer_amd")
from gpu_helpers import red_series  # noqa: E402
from oracle import pycwt_spec as pc  # noqa: E402
from wtmi import _lib, transforms  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
dj = float(sys.argv[2]) if len(sys.argv) > 2 else 1 / 8
rng = np.random.default_rng(n + 11)
y1 = red_series(rng, n).astype(np.float64)
y2 = 0.6 * np.roll(y1, 3) + 0.8 * red_series(rng, n)
W12 = (pc.cwt((y1 - y1.mean()) / y1.std(), 1 / 12, dj, 2 / 12, -1)[0]
       * pc.cwt((y2 - y2.mean()) / y2.std(), 1 / 12, dj, 2 / 12, -1)[0].conj())
a = np.abs(W12)
rel = a / a.max(axis=-1, keepdims=True)
ref_ph = np.angle(W12)
t1 = torch.tensor(np.stack([y1, y1]), device="cuda", dtype=torch.float32)
t2 = torch.tensor(np.stack([y2, y2]), device="cuda", dtype=torch.float32)
for prune in (0, 1, 2):
    with _lib.option("wct_prune", prune):
        res, _, _ = transforms.wct_batch(t1, t2, 1 / 12, dj, 2 / 12, -1, want_uv=False,
                                         want_power=True, want_phase=True)
    ph = res["phase"][0].cpu().numpy().astype(np.float64)
    d = np.abs(np.angle(np.exp(1j * (ph - ref_ph))))
    dw = np.abs(np.sqrt(res["power"][0].cpu().numpy().astype(np.float64)) - a) / a.max(axis=-1, keepdims=True)
    line = [f"prune {prune}:"]
    for lo, hi in ((1e-1, 1.01), (1e-2, 1e-1), (1e-3, 1e-2), (1e-4, 1e-3)):
        m = (rel > lo) & (rel <= hi)
        line.append(f"[{lo:g},{hi:g}] max {d[m].max():.2e}")
    line.append(f"| |W12| err / rowmax max {dw.max():.2e}")
    gm = a > 1e-3 * a.max()
    line.append(f"| global-mask max {d[gm].max():.2e}")
    print(" ".join(line), flush=True)
