"""Multi-rank path with the REAL engine, on the one-GPU box.

Two ranks over gloo, both on cuda:0, each run the HIP CWT and MODWT on their
``shard_range`` block and gather host-side to rank 0 (wtmi.sharding); the gathered
batch must be bit-identical to one process transforming the whole batch (the kernels
compute every series independently).  The bench's multi-rank mode runs the same way in
``--dist-backend gloo`` smoke mode: two ranks cover the global C2 batch.
"""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, N0, S, J = 13, 1500, 40, 6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch():
    from gpu_helpers import red_batch
    return red_batch(99, B, N0)


def _transform(x):
    """CWT W (complex64) and MODWT rows of a [b, n0] host batch on cuda:0."""
    import torch
    from wtmi import ops
    from wtmi.wavelets import Wavelet
    sj = 2 / 12 * 2 ** (np.arange(S) / 12)
    xd = torch.tensor(x, device="cuda:0")
    W = ops.cwt_morlet(xd, sj, 1 / 12)["w"]
    w = Wavelet("db4")
    M = ops.modwt(xd, w.dec_lo, w.dec_hi, J)
    return W, M


def _rank_main(rank, world, port, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "wavelet-transformer_amd"), os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist
    from wtmi import sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    x = _batch()
    s, e = sharding.shard_range(B, rank, world)
    W, M = _transform(x[s:e])
    gW = sharding.gather_to_rank0(torch.view_as_real(W), B)
    gM = sharding.gather_to_rank0(M, B)
    # the pageable path gathers the same bits
    pW = sharding.gather_to_rank0(torch.view_as_real(W), B, pinned=False)
    pM = sharding.gather_to_rank0(M, B, pinned=False)
    t = sharding.max_over_ranks(1.0 + rank)
    if rank == 0:
        assert torch.equal(gW, pW) and torch.equal(gM, pM)
        np.save(os.path.join(out_dir, "W.npy"), torch.view_as_complex(gW).numpy())
        np.save(os.path.join(out_dir, "M.npy"), gM.numpy())
        np.save(os.path.join(out_dir, "t.npy"), np.array([t]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_on_one_gpu_gather_bitwise(tmp_path):
    import torch
    port = _free_port()
    code = ("import sys; sys.path[:0] = [%r, %r]; import test_gpu_dist as t; "
            "t._rank_main(int(sys.argv[1]), 2, %d, %r)"
            % (os.path.join(ROOT, "tests"), ROOT, port, str(tmp_path)))
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r)], cwd=ROOT) for r in range(2)]
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0]
    W, M = _transform(_batch())
    np.testing.assert_array_equal(np.load(tmp_path / "W.npy"), W.cpu().numpy())
    np.testing.assert_array_equal(np.load(tmp_path / "M.npy"), M.cpu().numpy())
    assert float(np.load(tmp_path / "t.npy")[0]) == 2.0
    torch.cuda.synchronize()


@pytest.mark.parametrize("scaling,glob,per", [("strong", 1024, 512), ("weak", 2048, 1024)])
def test_bench_two_ranks_gloo_smoke(scaling, glob, per):
    """bench.py --gpus 2 --dist-backend gloo: both ranks on the one GPU; strong: the C2 batch
    covered (512 series each); weak (the default): each rank its own 1024-series block; one
    JSON line with n_gpus 2."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "c2",
           "--dist-backend", "gloo", "--steps", "3", "--warmup", "1", "--prewarm-s", "0",
           "--rank-timeout", "240", "--no-cpu-baseline", "--scaling", scaling]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == scaling
    cfg = line["config"]
    assert cfg["global_batch"] == glob and cfg["per_rank_batch"] == per
    assert cfg["dist_backend"] == "gloo"
    assert line["value"] > 0
    assert line["check"]["rank0_first_last_series_max_row_rel_err_vs_oracle"] < 1e-5


def _rccl_main(port, out_dir):
    """One rank of an RCCL group of one on cuda:0: the barrier with device_ids, the max / sum
    over ranks on device tensors, and the host-side gather through the gloo side group that
    sharding.host_group creates under RCCL (bench.py's and sharding's RCCL branch)."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "wavelet-transformer_amd"), os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist
    from wtmi import sharding
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    dist.barrier(device_ids=[0])
    W, M = _transform(_batch())
    gW = sharding.gather_to_rank0(torch.view_as_real(W), B)
    gM = sharding.gather_to_rank0(M, B)
    assert str(dist.get_backend(sharding.host_group())) == "gloo"
    t = sharding.max_over_ranks(2.5)
    u = sharding.sum_over_ranks(7.0)
    np.save(os.path.join(out_dir, "W.npy"), torch.view_as_complex(gW).numpy())
    np.save(os.path.join(out_dir, "M.npy"), gM.numpy())
    np.save(os.path.join(out_dir, "tu.npy"), np.array([t, u]))
    dist.barrier(device_ids=[0])
    dist.destroy_process_group()


def test_rccl_branch_one_rank(tmp_path):
    """the RCCL code path on the one-GPU box (a fresh child process): init with
    device_id, barrier(device_ids=[0]), all-reduces on device tensors, the gloo side group of
    the gather; the gathered batch is bit-identical to a direct transform."""
    port = _free_port()
    code = ("import sys; sys.path[:0] = [%r, %r]; import test_gpu_dist as t; t._rccl_main(%d, %r)"
            % (os.path.join(ROOT, "tests"), ROOT, port, str(tmp_path)))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    W, M = _transform(_batch())
    np.testing.assert_array_equal(np.load(tmp_path / "W.npy"), W.cpu().numpy())
    np.testing.assert_array_equal(np.load(tmp_path / "M.npy"), M.cpu().numpy())
    np.testing.assert_array_equal(np.load(tmp_path / "tu.npy"), [2.5, 7.0])


def test_bench_force_dist_rccl():
    """bench.py --force-dist at --gpus 1: the measured path's RCCL group (one rank), its timing
    barrier and reductions, and the host gather; the JSON line says dist_backend "rccl"."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--config", "c2",
           "--force-dist", "--steps", "3", "--warmup", "1", "--prewarm-s", "0",
           "--no-cpu-baseline"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["config"]["dist_backend"] == "rccl"
    assert line["config"]["dist_gather"] == [[0.0, 1024 * 128 * 4096.0]]
    assert line["value"] > 0
    assert line["check"]["rank0_first_last_series_max_row_rel_err_vs_oracle"] < 1e-5
    g = line["gather"]  # the host gather of rank 0's whole W, timed outside the region
    assert g["bytes"] == 1024 * 128 * 4096 * 8
    assert g["pinned_ms"] > 0 and g["pinned_ms_max_over_ranks"] == g["pinned_ms"]
    print("gather", {k: g[k] for k in ("pinned_ms", "pinned_GBps", "pageable_ms", "pageable_GBps")})


def test_pinned_d2h_bitwise_equal_to_pageable():
    """sharding.d2h: the page-locked copy (pool buffer, reused) and the pageable copy of the
    same device tensors hold the same bits, for a CWT output and for odd sizes / dtypes."""
    import torch
    from wtmi import sharding
    W, M = _transform(_batch())
    for t in (torch.view_as_real(W), M, M[3:7], torch.arange(12345, device="cuda", dtype=torch.int64)):
        a = sharding.d2h(t)
        assert a.is_pinned()
        b = sharding.d2h(t, pinned=False)
        assert not b.is_pinned()
        assert torch.equal(a, b) and torch.equal(a, t.cpu())
        sharding.release_pinned(a)
    again = sharding.d2h(M)  # taken from the pool
    assert torch.equal(again, M.cpu())
