"""Row errors of an N = 8192 CWT against the oracle for each cwt_prune level (diagnostic)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "wavelet-transformer_amd")
from oracle import pycwt_spec as pc  # noqa: E402
from wtmi import _lib, ops  # noqa: E402

n, dt, dj = 8192, 1 / 12, 1 / 8
sj = 2 * dt * 2 ** (np.arange(97) * dj)
rng = np.random.default_rng(1)
x = rng.standard_normal(n).cumsum()
ref = pc.cwt(x, dt, dj, 2 * dt, 96)[0]
xt = torch.tensor(np.stack([x, x]), device="cuda", dtype=torch.float32)
for prune in (0, 1, 2):
    with _lib.option("cwt_prune", prune):
        W = ops.cwt_morlet(xt, sj, dt)["w"][0].cpu().numpy().astype(np.complex128)
    err = np.linalg.norm(W - ref, axis=1) / np.linalg.norm(ref, axis=1)
    print(prune, np.round(err[::8], 4), flush=True)
