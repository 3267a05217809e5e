"""C4 shard experiment: B pairs as one WCT call vs K sub-batches on K streams (each its own
workspace and the engine's side stream), interleaving their dependent kernel chains.

    python scripts/debug/c4_split_streams.py [B] [reps]
"""
import sys

import numpy as np
import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import ops, transforms  # noqa: E402

DT = 1 / 12
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 40
n, dj = 8192, 1 / 8
sj, _ = transforms.scales_for(n, DT, dj, 2 * DT, -1, transforms.Morlet(6))
K = transforms.boxcar_rows(transforms.Morlet(6), dj)
sjd = torch.tensor(sj, device="cuda")
rng = np.random.default_rng(1)
y1 = torch.tensor(rng.standard_normal((B, n)).cumsum(1).astype(np.float32), device="cuda")
y2 = torch.tensor(rng.standard_normal((B, n)).cumsum(1).astype(np.float32), device="cuda")


def make(parts):
    cuts = [B * i // parts for i in range(parts + 1)]
    streams = [torch.cuda.Stream() for _ in range(parts)]
    wss = [torch.empty(ops.wct_workspace_bytes(cuts[i + 1] - cuts[i], n, sj.size), dtype=torch.uint8,
                       device="cuda") for i in range(parts)]

    def step():
        cur = torch.cuda.current_stream()
        outs = []
        for i, s in enumerate(streams):
            s.wait_stream(cur)
            with torch.cuda.stream(s):
                outs.append(ops.wct_morlet(y1[cuts[i]:cuts[i + 1]], y2[cuts[i]:cuts[i + 1]], sjd, DT, 6.0,
                                           boxcar=K, want_uv=False, want_power=True, want_phase=True,
                                           workspace=wss[i], normalize=True))
        for s in streams:
            cur.wait_stream(s)
        return outs
    return step


def timed(fn):
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


from wtmi import _lib  # noqa: E402


def lib_split(parts):
    one = make(1)

    def step():
        with _lib.option("wct_split", parts):
            return one()
    return step


steps = {p: make(p) for p in (1, 2, 4)}
steps["lib2"] = lib_split(2)
steps["lib4"] = lib_split(4)
ref = torch.cat([o["coh"] for o in steps[1]()])
for p in (2, 4, "lib2", "lib4"):
    got = torch.cat([o["coh"] for o in steps[p]()])
    torch.cuda.synchronize()
    assert torch.equal(got, ref), p
res = {p: [] for p in steps}
for _ in range(3):
    for p, f in steps.items():
        res[p].append(timed(f))
for p, v in res.items():
    print(f"B={B} parts={p}: " + " ".join(f"{t:.4f}" for t in v) + f"  min {min(v):.4f} ms", flush=True)
