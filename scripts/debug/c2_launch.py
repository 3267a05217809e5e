"""C2 step: per-step host cost and GPU time, eager vs hipGraph replay (one process).
python scripts/debug/c2_launch.py"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import ops  # noqa: E402

DT = 1 / 12
B, n0 = 1024, 4096
sj = 2 * DT * 2 ** (np.arange(128) / 12)
x = torch.randn(B, n0, device="cuda")
sjd = torch.tensor(sj, device="cuda")
out = torch.empty((B, sj.size, n0), dtype=torch.complex64, device="cuda")


def step():
    ops.cwt_morlet(x, sjd, DT, 6.0, out_w=out)


for _ in range(300):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(200):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"eager: host enqueue {1e3 * (t1 - t0) / 200:.3f} ms/step, wall {1e3 * (t2 - t0) / 200:.3f} ms/step", flush=True)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        step()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    step()
for _ in range(300):
    g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(200):
    g.replay()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"graph: host enqueue {1e3 * (t1 - t0) / 200:.3f} ms/step, wall {1e3 * (t2 - t0) / 200:.3f} ms/step", flush=True)
for _ in range(3):
    t0 = time.perf_counter()
    for _ in range(200):
        step()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"eager again: wall {1e3 * (t2 - t0) / 200:.3f} ms/step", flush=True)
