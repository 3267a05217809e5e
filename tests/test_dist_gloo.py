"""World-size-2 gloo test of the multi-GPU path's host logic (sharding, host-side
gather in series order, max-over-ranks timing).  The per-shard transform here is the
CPU oracle standing in for the GPU kernels (no GPU in this test)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, batch, n, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "wavelet-transformer_amd")]
    from oracle import modwt_spec as ms
    from wtmi import sharding
    from wtmi.wavelets import Wavelet
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(0)
    x = torch.tensor(rng.standard_normal((batch, n)))
    w = Wavelet("db4")

    def fn(block):
        if block.shape[0] == 0:  # an empty shard (batch smaller than the world)
            return torch.empty((0, 4, n), dtype=torch.float64)
        return torch.tensor(np.stack([ms.modwt(r.numpy(), w.dec_lo, w.dec_hi, 3) for r in block]))

    local = sharding.run_sharded(x, fn, rank, world)
    full = sharding.gather_to_rank0(local, batch)
    t = sharding.max_over_ranks(1.0 + rank)
    if rank == 0:
        ref = np.stack([ms.modwt(r, w.dec_lo, w.dec_hi, 3) for r in x.numpy()])
        q.put((np.abs(full.numpy() - ref).max(), tuple(full.shape), t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("batch", [1, 7, 8])
def test_sharded_gather_matches_unsharded(batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, batch, 64, q)) for r in range(2)]
    for p in procs:
        p.start()
    err, shape, t = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert err == 0.0 and shape == (batch, 4, 64) and t == 2.0


def test_shard_range_covers_batch_once():
    from wtmi.sharding import shard_range
    for batch in (0, 1, 7, 1024, 1025):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, e = shard_range(batch, r, world)
                seen.extend(range(s, e))
            assert seen == list(range(batch))


def test_pinned_pool_reuse_and_host_passthrough():
    """sharding.pinned_buffer reuses released buffers by size; d2h of a host tensor returns it
    as is (never a pool buffer), so gather_to_rank0 of host blocks cannot pool the caller's
    memory."""
    import torch
    from wtmi import sharding
    x = torch.arange(12, dtype=torch.float32).reshape(3, 4)
    assert sharding.d2h(x) is x
    if not torch.cuda.is_available():
        return
    a = sharding.pinned_buffer((3, 4), torch.float32)
    ptr = a.data_ptr()
    sharding.release_pinned(a)
    b = sharding.pinned_buffer((4, 3), torch.float32)
    assert b.data_ptr() == ptr and b.is_pinned()
