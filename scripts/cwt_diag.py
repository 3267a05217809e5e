"""CWT kernel diagnostics on the C2 workload (one GPU).

--mode seq    per-launch HIP-event times for back-to-back launches, then for launches
              separated by idle gaps, plus a torch fill_ of the same output buffer as a
              write-bandwidth reference measured on the same device.
--mode short  3 launches only (for rocprofv3 --pmc passes).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "wavelet-transformer_amd")]
from bench import C2  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", default="seq")
ap.add_argument("--n", type=int, default=30)
a = ap.parse_args()
dev = torch.device("cuda", 0)
wl = C2(0, dev)
torch.cuda.synchronize()


def timed(fn, n, gap_ms=0.0):
    out = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        if gap_ms:
            torch.cuda.synchronize()
            time.sleep(gap_ms / 1e3)
        out.append((s, e))
    torch.cuda.synchronize()
    return [s.elapsed_time(e) for s, e in out]


if a.mode == "short":
    for _ in range(3):
        wl.step()
    torch.cuda.synchronize()
    sys.exit(0)

res = {}
res["b2b"] = timed(wl.step, a.n)
res["gap5ms"] = timed(wl.step, 10, gap_ms=5)
res["b2b_again"] = timed(wl.step, a.n)
fill = lambda: wl.out.view(torch.float32).fill_(1.0)  # noqa: E731
res["fill_b2b"] = timed(fill, 10)
copy_src = torch.empty_like(wl.out)
res["copy_b2b"] = timed(lambda: wl.out.copy_(copy_src), 5)
for k, v in res.items():
    print(json.dumps({"series": k, "ms": [round(x, 4) for x in v], "median": float(np.median(v))}))
nbytes = wl.out.numel() * 8
print(json.dumps({"fill_GBps": nbytes / np.median(res["fill_b2b"]) / 1e6,
                  "copy_GBps(r+w)": 2 * nbytes / np.median(res["copy_b2b"]) / 1e6,
                  "cwt_b2b_GBps": wl.bytes / np.median(res["b2b"]) / 1e6,
                  "cwt_gap_GBps": wl.bytes / np.median(res["gap5ms"]) / 1e6}))
