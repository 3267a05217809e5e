"""MODWT / iMODWT kernel A/B timing on the C3 workload (one GPU).

Times wtmi_modwt and wtmi_imodwt separately (HIP events, median of --n launches)
for each kernel variant selected through WTMI_MODWT_VARIANT / WTMI_IMODWT_VARIANT
(read by the launcher on every call).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "wavelet-transformer_amd")]
from bench import C3  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=10)
ap.add_argument("--variants", default="0,1")
a = ap.parse_args()
dev = torch.device("cuda", 0)
wl = C3(0, dev)
ops, wv = wl.ops, wl.w
w = ops.modwt(wl.x, wv.dec_lo, wv.dec_hi, wl.J)
xr = ops.imodwt(w, wv.dec_lo, wv.dec_hi)
torch.cuda.synchronize()


def timed(fn):
    ev = []
    for _ in range(a.n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        ev.append((s, e))
    torch.cuda.synchronize()
    return float(np.median([s.elapsed_time(e) for s, e in ev]))


for v in a.variants.split(","):
    os.environ["WTMI_MODWT_VARIANT"] = v
    os.environ["WTMI_IMODWT_VARIANT"] = v
    t_a = timed(lambda: ops.modwt(wl.x, wv.dec_lo, wv.dec_hi, wl.J, out=w))
    t_s = timed(lambda: ops.imodwt(w, wv.dec_lo, wv.dec_hi, out=xr))
    err = float((xr - wl.x).abs().max() / wl.x.abs().max())
    nb = wl.B * wl.n * 4
    print(json.dumps({"variant": v, "modwt_ms": t_a, "imodwt_ms": t_s,
                      "modwt_GBps": nb * (1 + wl.J + 1) / t_a / 1e6,
                      "imodwt_GBps": nb * (wl.J + 1 + 1) / t_s / 1e6, "roundtrip_err": err}))
