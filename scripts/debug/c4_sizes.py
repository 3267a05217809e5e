"""C4 step time at several batch sizes with the library WTMI_LIB_PATH names (diagnostic, one
process per library so that A/B runs alternate builds):
    WTMI_LIB_PATH=... python scripts/debug/c4_sizes.py TAG B1 B2 ..."""
import os
import sys

import torch

sys.path.insert(0, "wavelet-transformer_amd")
from wtmi import ops, transforms  # noqa: E402

tag, Bs = sys.argv[1], [int(b) for b in sys.argv[2:]]
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


out = []
for B in Bs:
    x1 = torch.randn(B, n, device="cuda").cumsum(1)
    x2 = torch.randn(B, n, device="cuda").cumsum(1)
    ws = torch.empty(ops.wct_workspace_bytes(B, n, len(sj)), dtype=torch.uint8, device="cuda")
    step = lambda: transforms.wct_batch(x1, x2, dt, dj, 2 * dt, -1, workspace=ws, want_uv=False,  # noqa: E731
                                        want_power=True, want_phase=True)
    timed(step, 10)
    out.append(f"B={B} {min(timed(step) for _ in range(3)):.4f} ms")
print(tag, os.path.basename(os.path.dirname(os.environ.get("WTMI_LIB_PATH", "base/x"))), " ".join(out), flush=True)
