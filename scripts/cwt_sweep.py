"""In-process A/B sweep of launch variants on one bench workload (one GPU).
Variants are selected through the launchers' env knobs; rounds are interleaved
(rule: compare variants in one process).  SWEEP_CONFIG picks the workload (c2)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "wavelet-transformer_amd")]
from bench import CONFIGS  # noqa: E402

variants = json.loads(os.environ.get("SWEEP", '[{"WTMI_CWT_NBUF":"1"},{"WTMI_CWT_NBUF":"2"}]'))
dev = torch.device("cuda", 0)
wl = CONFIGS[os.environ.get("SWEEP_CONFIG", "c2")](0, dev)
res = {i: [] for i in range(len(variants))}
for rnd in range(5):
    for i, v in enumerate(variants):
        os.environ.update(v)
        for _ in range(2):
            wl.step()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            wl.step()
        e.record()
        torch.cuda.synchronize()
        res[i].append(s.elapsed_time(e) / 5)
for i, v in enumerate(variants):
    ms = np.median(res[i])
    print(json.dumps({"variant": v, "median_ms": ms, "min_ms": min(res[i]),
                      "GBps": wl.bytes / ms / 1e6, "check": wl.check()}))
