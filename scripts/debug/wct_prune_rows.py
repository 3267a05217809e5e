"""Per-row coherence difference, pruned vs unpruned WCT (debug)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "wavelet-transformer_amd"), os.path.join(ROOT, "tests")]
from gpu_helpers import red_series
from wtmi import transforms
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
rng = np.random.default_rng(n)
y1 = red_series(rng, n).astype(np.float64)
y2 = 0.6 * np.roll(y1, 3) + 0.8 * red_series(rng, n)
res = {}
for p in ("0", "1"):
    os.environ["WTMI_WCT_PRUNE"] = p
    res[p] = transforms.wct(y1, y2, 1 / 12, dj=1 / 8, s0=2 / 12, J=-1, sig=False)[0]
d = np.abs(res["0"] - res["1"]).max(axis=1)
for i, v in enumerate(d):
    print(i, "%.3e" % v)
