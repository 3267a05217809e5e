"""Strong-scaling shards on one GPU, direct launches vs a hipGraph replay of the step
(diagnostic for DESIGN 6): ms per step of C4 (pairs x 8192, dj 1/8) and C2 (series x 4096 x
128 scales) at the per-rank batch of a 1/2/4/8-GPU split, alternating the two modes.

    python scripts/shard_graph.py [c4|c2] [reps]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
sys.path.insert(0, ".")
from wtmi import ops, transforms  # noqa: E402

DT = 1 / 12


def timed(fn, reps):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def graphed(step):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        step()
    return g.replay


def c4_step(B):
    n, dj = 8192, 1 / 8
    sj, _ = transforms.scales_for(n, DT, dj, 2 * DT, -1, transforms.Morlet(6))
    K = transforms.boxcar_rows(transforms.Morlet(6), dj)
    rng = np.random.default_rng(B)
    y1 = torch.tensor(rng.standard_normal((B, n)).cumsum(1).astype(np.float32), device="cuda")
    y2 = torch.tensor(rng.standard_normal((B, n)).cumsum(1).astype(np.float32), device="cuda")
    sjd = torch.tensor(sj, device="cuda")
    ws = torch.empty(ops.wct_workspace_bytes(B, n, sj.size), dtype=torch.uint8, device="cuda")
    return lambda: ops.wct_morlet(y1, y2, sjd, DT, 6.0, boxcar=K, want_uv=False, want_power=True,
                                  want_phase=True, workspace=ws, normalize=True)


def c2_step(B):
    n, S = 4096, 128
    sj = torch.tensor(2 * DT * 2 ** (np.arange(S) / 12), device="cuda")
    x = torch.randn(B, n, device="cuda")
    out = torch.empty((B, S, n), dtype=torch.complex64, device="cuda")
    return lambda: ops.cwt_morlet(x, sj, DT, 6.0, out_w=out)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "c4"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    full = 512 if which == "c4" else 1024
    make = c4_step if which == "c4" else c2_step
    res = {}
    for world in (1, 2, 4, 8):
        B = full // world
        step = make(B)
        rep = graphed(step)
        d, g = [], []
        for _ in range(3):
            d.append(timed(step, reps))
            g.append(timed(rep, reps))
        res[world] = (B, min(d), min(g))
        print(f"{which} B={B:5d} (1/{world}): direct {min(d):.4f} ms  graph {min(g):.4f} ms  "
              f"[direct {' '.join(f'{v:.4f}' for v in d)} | graph {' '.join(f'{v:.4f}' for v in g)}]",
              flush=True)
        del step, rep
        torch.cuda.empty_cache()
    t1 = min(res[1][1:])
    for world in (2, 4, 8):
        B, d, g = res[world]
        print(f"{which} 1/{world}: efficiency vs 1/{world} of the full step: direct {t1 / world / d:.3f}, "
              f"graph {t1 / world / g:.3f}")


if __name__ == "__main__":
    main()
