"""Row stores stay inside their rows, launch chains replay from a hipGraph, and the WCT's
side streams do not leak across short-lived threads.

* Padded rows (n0 < N = 2^ceil(log2 n0)): each thread of a row's workgroup holds 16
  positions t + m NT, of which those >= n0 must not be written.  The buffer stores put the
  out-of-range positions' offset past the descriptor's extent in voffset (wct.hip put_row,
  cwt.hip store_row), so they are dropped whatever the hardware's range check does with the
  SGPR offset.  Each output here is written into the head of a larger buffer filled with a
  sentinel: the sentinel tail must survive bit for bit and the head must equal the ops
  result (same kernels, deterministic).
* hipGraph: the C ABI promises capture safety (no allocation, no sync inside a call).  One CWT
  step and one full-row WCT step (fork / join of the side stream included) are captured
  with torch.cuda.graph and replayed; the replay equals direct launches bit for bit, also
  after the inputs change in place.
* Side streams: a pool, not one per thread (include/wtmi.h wtmi_wct_side_streams).
* Launch policies (r04): the scheduling options of the WCT give bitwise-identical outputs.
"""

import threading

import numpy as np
import pytest
import torch

from gpu_helpers import red_batch

pytestmark = pytest.mark.gpu

SENT = np.float32(-12345.678)
TAIL = 1 << 16  # floats after the outputs


def _sentinel(nfloat):
    return torch.full((nfloat + TAIL,), float(SENT), dtype=torch.float32, device="cuda")


def _tail_ok(buf, nfloat):
    t = buf[nfloat:].cpu().numpy()
    return bool((t.view(np.uint32) == np.array([SENT], np.float32).view(np.uint32)[0]).all())


def _scales(n0, dj, S):
    sj = 2 / 12 * 2 ** (np.arange(S) * dj)
    return torch.tensor(sj, device="cuda", dtype=torch.float64)


@pytest.mark.parametrize("n0", [100, 700, 1333, 5000, 12000, 20000])
def test_cwt_xwt_padded_rows_write_only_their_samples(n0):
    from wtmi import _lib, ops
    from wtmi.ops import _ptr, _stream
    B, S = 3, 40
    x1 = torch.tensor(red_batch(n0, B, n0), device="cuda")
    x2 = torch.tensor(red_batch(n0 + 1, B, n0), device="cuda")
    sj = _scales(n0, 1 / 8, S)
    sig = torch.rand(S, dtype=torch.float64, device="cuda") + 0.5
    ref = ops.cwt_morlet(x1, sj, 1 / 12, 6.0, sig_scale=sig, want_w=True, want_power=True, want_sig=True)
    nf = B * S * n0
    bw, bp, bs = _sentinel(2 * nf), _sentinel(nf), _sentinel(nf)
    dev = x1.device

    def ws(pair):  # rows above 16384 samples run the four-step path through a workspace
        need = ops.cwt_workspace_bytes(B, n0, S, pair)
        return torch.empty(need, dtype=torch.uint8, device="cuda") if need else None

    _lib.call("wtmi_cwt_mother", _ptr(x1), x1.stride(0), B, n0, None, _ptr(sj), S, 1 / 12, 0, 6.0,
              _ptr(sig), 0, _ptr(bw), _ptr(bp), _ptr(bs), _ptr(ws(False)), _stream(dev))
    torch.cuda.synchronize()
    assert _tail_ok(bw, 2 * nf) and _tail_ok(bp, nf) and _tail_ok(bs, nf)
    assert torch.equal(bw[:2 * nf].view(torch.complex64).view(B, S, n0), ref["w"])
    assert torch.equal(bp[:nf].view(B, S, n0), ref["power"])
    assert torch.equal(bs[:nf].view(B, S, n0), ref["sig"])

    rx = ops.xwt_morlet(x1, x2, sj, 1 / 12, sig_scale=sig, want_w12=True, want_power=True,
                        want_sig=True, want_uv=True)
    bufs = [_sentinel(2 * nf)] + [_sentinel(nf) for _ in range(4)]
    _lib.call("wtmi_xwt_mother", _ptr(x1), _ptr(x2), x1.stride(0), B, n0, None, None, _ptr(sj), S,
              1 / 12, 0, 6.0, _ptr(sig), 0, *[_ptr(b) for b in bufs], _ptr(ws(True)), _stream(dev))
    torch.cuda.synchronize()
    assert _tail_ok(bufs[0], 2 * nf) and all(_tail_ok(b, nf) for b in bufs[1:])
    assert torch.equal(bufs[0][:2 * nf].view(torch.complex64).view(B, S, n0), rx["w12"])
    for b, k in zip(bufs[1:], ("power", "sig", "u", "v")):
        assert torch.equal(b[:nf].view(B, S, n0), rx[k]), k


@pytest.mark.parametrize("n0,dj", [(100, 1 / 8), (1333, 1 / 8), (5000, 1 / 8), (12000, 1 / 12),
                                  (20000, 1 / 4)])
def test_wct_padded_rows_write_only_their_samples(n0, dj):
    from wtmi import _lib, ops, transforms
    from wtmi.ops import _ptr, _stream
    B = 3
    y1 = torch.tensor(red_batch(2 * n0, B, n0), device="cuda")
    y2 = torch.tensor(red_batch(2 * n0 + 1, B, n0), device="cuda")
    sj_h, _ = transforms.scales_for(n0, 1 / 12, dj, 2 / 12, -1, transforms.as_morlet(None))
    S = sj_h.size
    sj = torch.tensor(sj_h, device="cuda")
    K = transforms.boxcar_rows(transforms.as_morlet(None), dj)
    norm = n0 <= 16384  # pycwt's normalisation in the first kernel (FFT rows); raw above
    ref = ops.wct_morlet(y1, y2, sj, 1 / 12, boxcar=K, want_uv=True, want_power=True,
                         want_phase=True, normalize=norm)
    nf = B * S * n0
    bufs = [_sentinel(nf) for _ in range(5)]
    ws = torch.empty(ops.wct_workspace_bytes(B, n0, S), dtype=torch.uint8, device="cuda")
    if norm:
        _lib.call("wtmi_wct_morlet_norm", _ptr(y1), _ptr(y2), y1.stride(0), B, n0, _ptr(sj), S, 1 / 12, 6.0,
                  K, _ptr(ws), *[_ptr(b) for b in bufs], _stream(y1.device))
    else:
        _lib.call("wtmi_wct_morlet", _ptr(y1), _ptr(y2), y1.stride(0), B, n0, None, None, _ptr(sj), S,
                  1 / 12, 6.0, K, _ptr(ws), *[_ptr(b) for b in bufs], _stream(y1.device))
    torch.cuda.synchronize()
    for b, k in zip(bufs, ("coh", "power", "phase", "u", "v")):
        assert _tail_ok(b, nf), k
        assert torch.equal(b[:nf].view(B, S, n0), ref[k]), k


def _capture(fn):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # warm (pool side streams, caches) outside the capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    out = {}
    with torch.cuda.graph(g):
        out.update(fn())
    return g, out


def test_cwt_step_replays_from_a_graph_bitwise():
    from wtmi import ops
    B, n0, S = 64, 4096, 64
    x = torch.tensor(red_batch(11, B, n0), device="cuda")
    sj = _scales(n0, 1 / 12, S)
    outw = torch.empty((B, S, n0), dtype=torch.complex64, device="cuda")
    g, out = _capture(lambda: {"w": ops.cwt_morlet(x, sj, 1 / 12, 6.0, out_w=outw)["w"]})
    outw.zero_()
    g.replay()
    torch.cuda.synchronize()
    direct = ops.cwt_morlet(x, sj, 1 / 12, 6.0)["w"]
    assert torch.equal(outw, direct)
    x.copy_(torch.tensor(red_batch(12, B, n0), device="cuda"))  # new input, same graph
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(outw, ops.cwt_morlet(x, sj, 1 / 12, 6.0)["w"])


@pytest.mark.parametrize("n0,B", [(4096, 16), (8192, 8)])
def test_full_row_wct_step_replays_from_a_graph_bitwise(n0, B):
    """Full rows (n0 = 2^k >= 1024): the side-stream fork / join is part of the graph."""
    from wtmi import ops, transforms
    y1 = torch.tensor(red_batch(21, B, n0), device="cuda")
    y2 = torch.tensor(red_batch(22, B, n0), device="cuda")
    sj_h, _ = transforms.scales_for(n0, 1 / 12, 1 / 8, 2 / 12, -1, transforms.as_morlet(None))
    sj = torch.tensor(sj_h, device="cuda")
    K = transforms.boxcar_rows(transforms.as_morlet(None), 1 / 8)
    ws = torch.empty(ops.wct_workspace_bytes(B, n0, sj_h.size), dtype=torch.uint8, device="cuda")

    def step():
        return ops.wct_morlet(y1, y2, sj, 1 / 12, boxcar=K, want_uv=False, want_power=True,
                              want_phase=True, workspace=ws, normalize=True)

    g, out = _capture(step)
    for rnd in range(2):
        g.replay()
        torch.cuda.synchronize()
        direct = step()
        torch.cuda.synchronize()
        for k in ("coh", "power", "phase"):
            assert torch.equal(out[k], direct[k]), (rnd, k)
        y1.copy_(torch.tensor(red_batch(23 + rnd, B, n0), device="cuda"))


def test_side_streams_pooled_across_short_lived_threads():
    """64 short-lived threads each run one 1024-sample full-row run_wct (the side-stream
    path): results equal the sequential run bit for bit, and the side-stream pool grows by
    at most the number of calls that overlapped -- with one thread at a time, not at all."""
    import src.wct as wct
    from wtmi import ops
    from wtmi.wavelets import Morlet
    rng = np.random.default_rng(5)
    pairs = [(red_batch(100 + i, 1, 1024)[0].astype(np.float64),
              red_batch(200 + i, 1, 1024)[0].astype(np.float64)) for i in range(8)]

    def run(i):
        y1, y2 = pairs[i % len(pairs)]
        d = wct.DataForWCT(y1, y2, Morlet(6), 1 / 12, 1 / 8, 2 / 12, wct.WCT_LEVELS)
        r = wct.run_wct(d, calculate_signficance=False)
        return r.coherence

    seq = [run(i) for i in range(len(pairs))]
    base = ops.wct_side_streams()
    assert base >= 1
    got = [None] * 64
    errs = []

    def worker(i):
        try:
            got[i] = run(i)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    for wave in range(8):  # 8 waves of 8 concurrent short-lived threads
        ts = [threading.Thread(target=worker, args=(8 * wave + k,)) for k in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert not errs, errs
    for i in range(64):
        np.testing.assert_array_equal(got[i], seq[i % len(pairs)])
    after = ops.wct_side_streams()
    assert after <= base + 8, (base, after)
    for i in range(64):  # one thread at a time: the pool has an idle stream for each
        t = threading.Thread(target=worker, args=(i,))
        t.start()
        t.join()
    assert not errs, errs
    assert ops.wct_side_streams() == after


@pytest.mark.parametrize("n0,B", [(1024, 6), (8192, 8), (16384, 3)])
def test_wct_launch_policies_bitwise_equal(n0, B):
    """The launch-policy options change only how the work is scheduled (r04): the decimation
    classes in one launch or one per class (wct_dec_merge), the side stream and phase C's third
    stream on or off, rows per workgroup -- every combination writes the same bits."""
    from wtmi import _lib, ops, transforms
    y1 = torch.tensor(red_batch(31, B, n0), device="cuda")
    y2 = torch.tensor(red_batch(32, B, n0), device="cuda")
    sj_h, _ = transforms.scales_for(n0, 1 / 12, 1 / 8, 2 / 12, -1, transforms.as_morlet(None))
    sj = torch.tensor(sj_h, device="cuda")
    K = transforms.boxcar_rows(transforms.as_morlet(None), 1 / 8)
    ws = torch.empty(ops.wct_workspace_bytes(B, n0, sj_h.size), dtype=torch.uint8, device="cuda")

    def run():
        r = ops.wct_morlet(y1, y2, sj, 1 / 12, boxcar=K, want_uv=False, want_power=True,
                           want_phase=True, workspace=ws, normalize=True)
        torch.cuda.synchronize()
        return {k: r[k].clone() for k in ("coh", "power", "phase")}

    ref = run()
    for opts in ({"wct_dec_merge": 0}, {"wct_dec_merge": 1}, {"wct_side_stream": 0},
                 {"wct_pc_early": 0}, {"wct_pc_early": 1}, {"wct_min_rows": 1},
                 {"wct_dec_merge": 1, "wct_min_rows": 2, "wct_dec_rows": 2},
                 {"wct_depth": 0}, {"wct_depth": 0, "wct_pc_early": 1}):
        ctx = [_lib.option(k, v) for k, v in opts.items()]
        for c in ctx:
            c.__enter__()
        try:
            out = run()
        finally:
            for c in reversed(ctx):
                c.__exit__(None, None, None)
        for k in ref:
            assert torch.equal(out[k], ref[k]), (opts, k)
