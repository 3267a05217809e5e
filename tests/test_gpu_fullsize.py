"""Parity at the exact BASELINE sizes (C2-C5), against the oracle on sampled rows.

The per-shape tests elsewhere use small batches; here the whole configured batch runs,
so the grid- and offset-dependent paths are exercised: chunk counts, the XCD remap of
the WCT over 512 pairs, C2's 4.3 GB W and C3's 5.9 GB decomposition (the last series sits
at the highest addresses), and a full C5 streaming chunk.  Rows are sampled at the start,
middle and END of each batch.  Tolerances as SURVEY 8(d): CWT row-normwise <= 1e-5, MODWT
per-row normwise <= 1e-5 and round trip <= 1e-5 max|x|, WCT coherence abs <= 1e-4,
power row-normwise <= 1e-5, phase <= 1e-4 rad where |W12| > 1e-3 max.
"""

import numpy as np
import pytest
import torch

from gpu_helpers import gate, red_batch, row_relerr
from oracle import modwt_spec as ms
from oracle import pycwt_spec as pc

pytestmark = pytest.mark.gpu
DT = 1 / 12


def _cwt_rows_ok(W, x, rows, dj, J):
    for r in rows:
        ref = pc.cwt(x[r].astype(np.float64), DT, dj, 2 * DT, J)[0]
        got = W[r].cpu().numpy().astype(np.complex128)
        gate(f"W[{r}]", row_relerr(got, ref))


def test_c2_full_batch():
    """C2: 1024 x 4096 x 128 scales, complex64 W (4.3 GB); series 0, 511, 1023."""
    from wtmi import ops
    B, n, dj, J = 1024, 4096, 1 / 12, 127
    x = red_batch(1002, B, n)
    sj = 2 * DT * 2 ** (np.arange(J + 1) * dj)
    W = ops.cwt_morlet(torch.tensor(x, device="cuda"), sj, DT)["w"]
    assert W.shape == (B, 128, n)
    _cwt_rows_ok(W, x, (0, 511, 1023), dj, J)
    del W
    torch.cuda.empty_cache()


@pytest.mark.parametrize("B,n,dj,J", [(1024, 4096, 1 / 12, 127), (512, 8192, 1 / 24, 255)],
                         ids=["c2_batch", "c5_chunk"])
def test_cwt_full_size_linearity_every_series(B, n, dj, J):
    """C2's batch and a C5 chunk at full size through a size-independent property, on EVERY
    (series, scale) row: the transform is linear, W(x + 2y) = W(x) + 2 W(y), to fp32 rounding
    (row-normwise <= 1e-5 of ||W(x)|| + 2 ||W(y)||).  Catches a wrong row offset, a skipped
    chunk or a grid-dependent path anywhere in the 4.3 / 8.6 GB output, which the sampled rows
    above cannot."""
    from wtmi import ops
    x = torch.tensor(red_batch(1012 + n, B, n), device="cuda")
    y = torch.tensor(red_batch(2012 + n, B, n), device="cuda")
    sj = 2 * DT * 2 ** (np.arange(J + 1) * dj)
    wx = ops.cwt_morlet(x, sj, DT)["w"]
    wy = ops.cwt_morlet(y, sj, DT)["w"]
    wz = ops.cwt_morlet(x + 2 * y, sj, DT)["w"]
    worst = 0.0
    for c in range(0, B, 128):
        d = torch.linalg.vector_norm(wz[c:c + 128] - wx[c:c + 128] - 2 * wy[c:c + 128], dim=-1)
        s = (torch.linalg.vector_norm(wx[c:c + 128], dim=-1)
             + 2 * torch.linalg.vector_norm(wy[c:c + 128], dim=-1))
        assert bool((s > 0).all())
        worst = max(worst, (d / s).max().item())
    gate("linearity every row", worst)
    del wx, wy, wz
    torch.cuda.empty_cache()


def test_c5_full_chunk():
    """C5: one full 512-series streaming chunk, 8192 samples x 256 scales (dj = 1/24)."""
    from wtmi import ops
    B, n, dj, J = 512, 8192, 1 / 24, 255
    x = red_batch(1005, B, n)
    sj = 2 * DT * 2 ** (np.arange(J + 1) * dj)
    W = ops.cwt_morlet(torch.tensor(x, device="cuda"), sj, DT)["w"]
    _cwt_rows_ok(W, x, (0, 257, 511), dj, J)
    del W
    torch.cuda.empty_cache()


def test_c3_full_batch():
    """C3: 8192 x 16384, db4 J = 10; decomposition rows [W_1..W_10, V_10] of series 0, 4095
    and 8191 vs src/modwt.py's algorithm, and their reconstruction."""
    from wtmi import ops
    from wtmi.wavelets import Wavelet
    B, n, J = 8192, 16384, 10
    w = Wavelet("db4")
    x = np.empty((B, n), np.float32)
    for c in range(0, B, 1024):
        x[c:c + 1024] = red_batch(1003 + c, 1024, n)
    xd = torch.tensor(x, device="cuda")
    C = ops.modwt(xd, w.dec_lo, w.dec_hi, J)
    assert C.shape == (B, J + 1, n)
    xr = ops.imodwt(C, w.dec_lo, w.dec_hi)
    for r in (0, 4095, 8191):
        ref = ms.modwt_direct(x[r].astype(np.float64), w.dec_lo, w.dec_hi, J)
        got = C[r].cpu().numpy().astype(np.float64)
        assert row_relerr(got, ref).max() <= 1e-5, r
        scale = np.abs(ref).max(axis=1, keepdims=True)
        assert (np.abs(got - ref) <= 1e-5 * scale).all(), r
        back = xr[r].cpu().numpy()
        assert np.abs(back - x[r]).max() <= 1e-5 * np.abs(x[r]).max(), r
    err = ((xr - xd).abs().amax(dim=1) / xd.abs().amax(dim=1)).max().item()
    assert err <= 1e-5, err  # every series' round trip
    # energy (MODWT with an orthonormal filter: sum_j ||W_j||^2 + ||V_J||^2 = ||x||^2), every series
    worst = 0.0
    for c in range(0, B, 512):
        e_c = C[c:c + 512].double().square().sum(dim=(1, 2))
        e_x = xd[c:c + 512].double().square().sum(dim=1)
        worst = max(worst, ((e_c - e_x).abs() / e_x).max().item())
    assert worst <= 1e-5, worst
    del C, xr
    torch.cuda.empty_cache()


def test_c4_full_batch():
    """C4: 512 pairs x 8192, dj = 1/8 (97 scales); pairs 0, 255, 511."""
    from wtmi import transforms
    P, n, dj = 512, 8192, 1 / 8
    y1 = red_batch(1004, P, n)
    y2 = (0.6 * np.roll(y1, 3, axis=1) + 0.8 * red_batch(2004, P, n)).astype(np.float32)
    res, sj, _ = transforms.wct_batch(torch.tensor(y1, device="cuda"), torch.tensor(y2, device="cuda"),
                                      DT, dj, 2 * DT, -1, want_uv=False, want_power=True,
                                      want_phase=True)
    assert res["coh"].shape == (P, 97, n)
    for p in (0, 255, 511):
        a1, a2 = y1[p].astype(np.float64), y2[p].astype(np.float64)
        rc = pc.wct(a1, a2, DT, dj=dj, s0=2 * DT, J=-1, sig=False)[0]
        gate(f"coherence abs[{p}]", np.abs(res["coh"][p].cpu().numpy() - rc), 1e-4)
        W12 = (pc.cwt((a1 - a1.mean()) / a1.std(), DT, dj, 2 * DT, -1)[0]
               * pc.cwt((a2 - a2.mean()) / a2.std(), DT, dj, 2 * DT, -1)[0].conj())
        pw = res["power"][p].cpu().numpy().astype(np.float64)
        gate(f"wct power[{p}]", row_relerr(pw, np.abs(W12) ** 2))
        mask = np.abs(W12) > 1e-3 * np.abs(W12).max()
        dphi = np.angle(np.exp(1j * (res["phase"][p].cpu().numpy() - np.angle(W12))))
        gate(f"phase rad[{p}]", np.abs(dphi[mask]), 1e-4)
    del res
    torch.cuda.empty_cache()


def test_c4_full_batch_properties_every_pair():
    """C4 at full size through size-independent properties, on EVERY pair, scale and sample:
    a series is fully coherent with itself (WCT(x, x) = 1) and coherence is symmetric
    (WCT(x, y) = WCT(y, x)), both to fp32 rounding (abs <= 1e-4, the coherence tolerance)."""
    from wtmi import transforms
    P, n, dj = 512, 8192, 1 / 8
    y1 = torch.tensor(red_batch(1014, P, n), device="cuda")
    y2 = torch.tensor((0.6 * np.roll(red_batch(1014, P, n), 3, axis=1)
                       + 0.8 * red_batch(2014, P, n)).astype(np.float32), device="cuda")

    def coh(a, b):
        return transforms.wct_batch(a, b, DT, dj, 2 * DT, -1, want_uv=False)[0]["coh"]

    c = coh(y1, y1)
    assert c.shape == (P, 97, n)
    assert (c - 1).abs().max().item() <= 1e-4
    del c
    cxy = coh(y1, y2)
    cyx = coh(y2, y1)
    assert bool(torch.isfinite(cxy).all())
    assert (cxy - cyx).abs().max().item() <= 1e-4
    del cxy, cyx
    torch.cuda.empty_cache()
