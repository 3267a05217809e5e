"""Empty batches through the HIP path (include/wtmi.h: an empty batch is a no-op returning 0,
its arrays may be NULL).  A rank's ``shard_range`` block of a batch smaller than the world is
empty (wtmi/sharding.py), and an empty torch tensor hands the C ABI a NULL pointer: every
entry point must return empty outputs of the right shape instead of raising, and the
non-empty shards around it must still be exact."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_empty_batch_every_op(db4):
    from wtmi import ops
    dev = "cuda"
    n0, S = 64, 5
    sj = 2 / 12 * 2 ** (np.arange(S) / 4)
    x = torch.empty((0, n0), dtype=torch.float32, device=dev)
    r = ops.cwt_morlet(x, sj, 1 / 12, want_power=True)
    assert r["w"].shape == (0, S, n0) and r["power"].shape == (0, S, n0)
    r = ops.xwt_morlet(x, x, sj, 1 / 12, want_w12=True, want_uv=True)
    assert r["w12"].shape == (0, S, n0) and r["u"].shape == (0, S, n0)
    r = ops.wct_morlet(x, x, sj, 1 / 12, boxcar=3, want_power=True, want_phase=True)
    assert r["coh"].shape == (0, S, n0) and r["phase"].shape == (0, S, n0)
    r = ops.wct_morlet(x, x, sj, 1 / 12, boxcar=3, normalize=True)
    assert r["coh"].shape == (0, S, n0)
    w = ops.modwt(x, db4["dec_lo"], db4["dec_hi"], 3)
    assert w.shape == (0, 4, n0)
    assert ops.imodwt(w, db4["dec_lo"], db4["dec_hi"]).shape == (0, n0)
    c, lens = ops.wavedec(x, db4["dec_lo"], db4["dec_hi"], 2)
    assert c.shape == (0, sum(lens))
    assert ops.waverec(c, n0, db4["rec_lo"], db4["rec_hi"], 2, [1, 3]).shape[:2] == (0, 2)
    assert ops.series_moments(x).shape[0] == 0
    assert ops.rednoise(0, n0, 0.7, 5, device=dev).shape == (0, n0)
    torch.cuda.synchronize()


def test_shards_of_a_small_batch_cover_it_exactly(db4):
    """Batch 3 over a world of 8: ranks 3..7 hold empty blocks.  Transforming every rank's
    block in turn and concatenating reproduces the whole-batch result bit for bit."""
    from gpu_helpers import red_batch
    from wtmi import ops, sharding
    B, n0, S, world = 3, 700, 12, 8
    sj = 2 / 12 * 2 ** (np.arange(S) / 6)
    x = torch.tensor(red_batch(7, B, n0), dtype=torch.float32, device="cuda")
    whole_w = ops.cwt_morlet(x, sj, 1 / 12)["w"]
    whole_m = ops.modwt(x, db4["dec_lo"], db4["dec_hi"], 4)
    parts_w, parts_m, sizes = [], [], []
    for rank in range(world):
        lo, hi = sharding.shard_range(B, rank, world)
        blk = x[lo:hi]
        sizes.append(hi - lo)
        parts_w.append(ops.cwt_morlet(blk, sj, 1 / 12)["w"])
        parts_m.append(ops.modwt(blk, db4["dec_lo"], db4["dec_hi"], 4))
    assert sizes.count(0) >= 1 and sum(sizes) == B
    assert torch.equal(torch.cat(parts_w), whole_w)
    assert torch.equal(torch.cat(parts_m), whole_m)
