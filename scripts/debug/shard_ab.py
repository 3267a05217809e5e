"""C4 at several shard sizes under several launch-option sets, alternating (diagnostic):
python scripts/debug/shard_ab.py "opt=v,opt=v" "opt=v" ... -- B1 B2 ..."""
import sys

import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import _lib, ops, transforms  # noqa: E402

args = sys.argv[1:]
cut = args.index("--")
sets = [dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in a.split(",") if kv) for a in args[:cut]]
Bs = [int(b) for b in args[cut + 1:]]
n, dt, dj = 8192, 1 / 12, 1 / 8
sj, _ = transforms.scales_for(n, dt, dj, 2 * dt, -1, transforms.Morlet(6))


def timed(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for B in Bs:
    x1 = torch.randn(B, n, device="cuda").cumsum(1)
    x2 = torch.randn(B, n, device="cuda").cumsum(1)
    ws = torch.empty(ops.wct_workspace_bytes(B, n, len(sj)), dtype=torch.uint8, device="cuda")
    step = lambda: transforms.wct_batch(x1, x2, dt, dj, 2 * dt, -1, workspace=ws, want_uv=False,  # noqa: E731
                                        want_power=True, want_phase=True)
    timed(step)
    for rnd in range(2):
        for opts in sets:
            ctx = [_lib.option(k, v) for k, v in opts.items()]
            for c in ctx:
                c.__enter__()
            ms = timed(step)
            for c in reversed(ctx):
                c.__exit__(None, None, None)
            print(f"C4 B={B:4d} {opts} {ms:.4f} ms  (x{512 / B:g} = {ms * 512 / B:.3f})", flush=True)
    del x1, x2, ws
