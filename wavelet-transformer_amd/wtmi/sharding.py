"""Series-level sharding across GPUs (one process per GPU).

Every series (CWT, MODWT, DWT) and every pair (XWT / WCT) is independent
(SURVEY 8(e)), so a batch is split into contiguous blocks, one per rank, and each
rank runs the kernels on its own device with no collective on the data path.  The
only cross-rank traffic is optional: a host-side gather of results to rank 0 for a
consumer that wants them in one place, and the max-over-ranks of a timing.
"""

from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def shard_range(batch: int, rank: int, world: int):
    """Contiguous [start, stop) block of ceil(batch / world) items for `rank`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    per = -(-batch // world)
    start = min(batch, rank * per)
    return start, min(batch, start + per)


def run_sharded(x: torch.Tensor, fn: Callable[[torch.Tensor], torch.Tensor], rank: int,
                world: int) -> torch.Tensor:
    """Apply `fn` to this rank's block of the rows of the (global) batch x."""
    s, e = shard_range(x.shape[0], rank, world)
    return fn(x[s:e])


def gather_to_rank0(local: torch.Tensor, batch: int, group=None) -> Optional[torch.Tensor]:
    """Host-side gather of per-rank result blocks into the global batch order on rank 0.

    Blocks are moved to host memory first, so the gather never touches the GPUs'
    data path (works over gloo; with RCCL only the small host copies travel)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    host = local.detach().to("cpu").contiguous()
    per = -(-batch // world)
    pad_shape = (per,) + tuple(host.shape[1:])
    buf = torch.zeros(pad_shape, dtype=host.dtype)
    buf[: host.shape[0]] = host
    out = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, out, dst=0, group=group)
    if rank != 0:
        return None
    return torch.cat(out, dim=0)[:batch]


def max_over_ranks(seconds: float, device: Optional[torch.device] = None) -> float:
    """Max of a wall time over all ranks (the bench's timed region)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device or "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
