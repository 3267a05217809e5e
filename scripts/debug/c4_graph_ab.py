"""C4 shard: direct launches vs a hipGraph replay of the step, alternating in one process, plus
the host time to enqueue one direct step (no sync).  python scripts/debug/c4_graph_ab.py B [rounds]"""
import sys
import time

import torch

sys.path.insert(0, "scripts")
sys.path.insert(0, "wavelet-transformer_amd")
from shard_graph import c4_step, graphed, timed  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
step = c4_step(B)
rep = graphed(step)
d, g = [], []
for _ in range(rounds):
    d.append(timed(step, 40))
    g.append(timed(rep, 40))
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"c4 B={B}: direct {' '.join(f'{v:.4f}' for v in d)} min {min(d):.4f} | graph "
      f"{' '.join(f'{v:.4f}' for v in g)} min {min(g):.4f} ms | host enqueue {(t1 - t0) / 20 * 1e3:.4f} ms/step",
      flush=True)
