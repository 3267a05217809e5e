"""Run each BASELINE GPU workload a few steps (for rocprofv3 --kernel-trace --stats)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "wavelet-transformer_amd")]
import bench  # noqa: E402

which = sys.argv[1:] or ["c2", "c3", "c4"]
dev = torch.device("cuda", 0)
for name in which:
    wl = bench.CONFIGS[name](0, dev)
    for _ in range(4):
        wl.step()
    torch.cuda.synchronize()
    del wl
    torch.cuda.empty_cache()
