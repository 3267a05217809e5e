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

Device-to-host copies ("D2H into pinned buffers, timed separately") go
through page-locked host buffers (``d2h``): a pageable ``.to("cpu")`` stages every byte
through a driver bounce buffer, a pinned destination is written by the DMA engine directly.
The buffers are kept in a small per-process pool keyed by size, so a consumer that gathers
every batch (the reference's per-series loop, src/utils/transform_helpers.py:116-135) pays
the page-locking once.
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


_PINNED: dict = {}
_PINNED_LOCK = threading.Lock()
PINNED_POOL_BYTES = 32 << 30  # buffers kept for reuse, at most this many bytes in total


def pinned_buffer(shape, dtype, reuse: bool = True) -> torch.Tensor:
    """A page-locked host tensor of `shape` / `dtype`.  With `reuse`, taken from (and later
    returned to, by ``release_pinned``) a per-process pool keyed by byte size."""
    shape = tuple(int(v) for v in shape)
    nbytes = torch.Size(shape).numel() * torch.empty((), dtype=dtype).element_size()
    if reuse:
        with _PINNED_LOCK:
            lst = _PINNED.get(nbytes)
            if lst:
                raw = lst.pop()
                return raw.view(dtype).view(shape) if nbytes else torch.empty(shape, dtype=dtype)
    if nbytes == 0:
        return torch.empty(shape, dtype=dtype)
    raw = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    return raw.view(dtype).view(shape)


def release_pinned(t: torch.Tensor) -> None:
    """Return a buffer from ``pinned_buffer`` (or ``d2h`` without ``out``) to the pool (dropped
    if the pool is full).  Only such buffers may be released: the pool hands them out again."""
    if not t.is_pinned() or t.numel() == 0:
        return
    raw = t.reshape(-1).view(torch.uint8)
    with _PINNED_LOCK:
        held = sum(k * len(v) for k, v in _PINNED.items())
        if held + raw.numel() <= PINNED_POOL_BYTES:
            _PINNED.setdefault(raw.numel(), []).append(raw)


def d2h(t: torch.Tensor, pinned: bool = True, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Copy a device tensor to host memory and wait for it: into `out` (any host tensor of the
    same shape and dtype), else into a pinned pool buffer (`pinned`), else a pageable one.
    The copy runs on the current stream after the work already queued there.  A host tensor
    is returned as is (contiguous)."""
    if t.device.type != "cuda":
        return t.contiguous()
    if out is None:
        out = pinned_buffer(t.shape, t.dtype) if pinned else torch.empty(t.shape, dtype=t.dtype)
    if tuple(out.shape) != tuple(t.shape) or out.dtype != t.dtype:
        raise ValueError(f"d2h: out {tuple(out.shape)} {out.dtype} for {tuple(t.shape)} {t.dtype}")
    out.copy_(t, non_blocking=out.is_pinned())
    if out.is_pinned():
        torch.cuda.current_stream(t.device).synchronize()
    return out


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


def gather_to_rank0(local: torch.Tensor, batch: int, group=None,
                    pinned: bool = True) -> Optional[torch.Tensor]:
    """Host-side gather of per-rank result blocks into the global batch order on rank 0.

    Each rank copies its block to host memory (D2H into a pinned buffer, ``d2h``; pageable
    with ``pinned=False``) and the blocks travel over a gloo group (``host_group``): nothing
    of the data path goes through RCCL, under either backend.  Rank 0 receives every block
    straight into its slot of one [world * ceil(batch / world), ...] host tensor (no
    concatenation copy).  Returns the [batch, ...] host tensor on rank 0, None elsewhere."""
    hg = host_group(group)
    world = dist.get_world_size(hg)
    rank = dist.get_rank(hg)
    per = -(-batch // world)
    s, e = shard_range(batch, rank, world)
    if local.shape[0] != e - s:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, its shard is {e - s}")
    pad_shape = (per,) + tuple(local.shape[1:])
    src = local.detach()
    # pool buffers only come from device blocks (a host block is used as it is, never pooled)
    pooled = pinned and src.device.type == "cuda"
    if src.shape[0] == per:
        buf = d2h(src, pinned=pinned)
    else:  # the last (short) block travels padded to the common block size
        buf = torch.zeros(pad_shape, dtype=src.dtype)
        if src.shape[0]:
            tmp = d2h(src, pinned=pinned)
            buf[: src.shape[0]] = tmp
            if pooled:
                release_pinned(tmp)
        pooled = False
    out = None
    if rank == 0:
        full = torch.empty((per * world,) + tuple(local.shape[1:]), dtype=local.dtype)
        out = [full[r * per:(r + 1) * per] for r in range(world)]
    dist.gather(buf.contiguous(), out, dst=dist.get_global_rank(hg, 0) if hg is not None else 0,
                group=hg)
    if pooled:
        release_pinned(buf)
    if rank != 0:
        return None
    return full[:batch]


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
