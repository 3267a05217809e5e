"""torch fill_ of a C2-sized buffer (4.3 GB) -- write-bandwidth reference (diagnostic)."""
import torch
x = torch.empty(131072 * 4096 * 2, device="cuda")
for _ in range(3):
    x.fill_(1.0)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    x.fill_(1.0)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 10
print("torch fill", ms, x.numel() * 4 / ms / 1e6)
