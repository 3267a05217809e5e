"""Series-level sharding across GPUs (one process per GPU).

Every series (CWT, MODWT, DWT) and every pair (XWT / WCT) is independent
(SURVEY 8(e)), so a batch is split into contiguous blocks, one per rank, and each
rank runs the kernels on its own device with no collective on the data path.  The
only cross-rank traffic is optional: a host-side gather of results to rank 0 for a
consumer that wants them in one place, and the max-over-ranks of a timing.

Process groups: an RCCL group (backend "nccl" on ROCm) has no CPU transport, so the
host-side gather runs over a gloo side group created once from the same ranks
(``host_group``), and scalar reductions use the group's own device.  Under a gloo (or
"cpu:gloo,cuda:nccl") group everything stays on the host.
"""

from __future__ import annotations

import threading
from typing import Callable, Optional

import torch
import torch.distributed as dist

_HOST_GROUPS: dict = {}
_HOST_LOCK = threading.Lock()


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


def _has_cpu_transport(group) -> bool:
    return "gloo" in str(dist.get_backend(group)).lower()


def host_group(group=None):
    """A process group that can carry CPU tensors among the ranks of the default group: the
    group itself under gloo, else a gloo side group made once (collective: every rank of
    the default group reaches the first call together, as they do inside
    ``gather_to_rank0``).  Only the default group (None, or the WORLD group) is supported
    under RCCL: torch requires EVERY process of the default group to call ``new_group``, even
    for a subgroup, so building a side group lazily from a subgroup's ranks alone would hang.
    The cache is keyed on the ranks, not on the group object's id (ids are reused after GC)."""
    if _has_cpu_transport(group):
        return group
    if group is not None and group is not dist.group.WORLD:
        raise ValueError("host_group: an RCCL subgroup is not supported (create a gloo group on "
                         "every rank and pass that instead)")
    key = tuple(range(dist.get_world_size()))
    with _HOST_LOCK:
        g = _HOST_GROUPS.get(key)
        if g is None:
            g = dist.new_group(ranks=list(key), backend="gloo")
            _HOST_GROUPS[key] = g
    return g


def gather_to_rank0(local: torch.Tensor, batch: int, group=None) -> Optional[torch.Tensor]:
    """Host-side gather of per-rank result blocks into the global batch order on rank 0.

    Each rank copies its block to host memory (D2H) and the blocks travel over a gloo
    group (``host_group``): nothing of the data path goes through RCCL, under either
    backend.  Returns the [batch, ...] host tensor on rank 0, None elsewhere."""
    hg = host_group(group)
    world = dist.get_world_size(hg)
    rank = dist.get_rank(hg)
    host = local.detach().to("cpu").contiguous()
    per = -(-batch // world)
    s, e = shard_range(batch, rank, world)
    if host.shape[0] != e - s:
        raise ValueError(f"rank {rank} holds {host.shape[0]} rows, its shard is {e - s}")
    pad_shape = (per,) + tuple(host.shape[1:])
    buf = torch.zeros(pad_shape, dtype=host.dtype)
    buf[: host.shape[0]] = host
    out = [torch.zeros_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, out, dst=dist.get_global_rank(hg, 0) if hg is not None else 0, group=hg)
    if rank != 0:
        return None
    return torch.cat(out, dim=0)[:batch]


def _reduce_device(group=None) -> torch.device:
    if _has_cpu_transport(group) or not torch.cuda.is_available():
        return torch.device("cpu")
    return torch.device("cuda", torch.cuda.current_device())


def max_over_ranks(seconds: float, group=None) -> float:
    """Max of a wall time over all ranks (the bench's timed region); a host tensor under
    gloo, a tensor on this rank's GPU under RCCL.  An initialised group of one rank still
    runs the all-reduce (the RCCL path exercised on one GPU: bench.py --force-dist)."""
    if not dist.is_initialized():
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=_reduce_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def sum_over_ranks(value: float, group=None) -> float:
    """Sum of a scalar over all ranks (units processed), on the same device rule."""
    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=_reduce_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(t.item())
