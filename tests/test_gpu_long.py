"""Series longer than one workgroup's row (n0 > 16384 -> the four-step long-row path,
csrc/fft_long.hpp) and boxcar windows wider than the register ring (K > 24), vs the
oracle (pycwt restatement).  Tolerances as SURVEY 8(d): CWT / XWT rows <= 1e-5
row-normwise (power, W12 too), coherence abs <= 1e-4, phase <= 1e-4 rad where
|W12| > 1e-3 max.  The reference (pycwt over scipy.fftpack) has no length limit; the
engine transforms up to 2^20 samples per row.
"""

import numpy as np
import pytest
import torch

from gpu_helpers import gate, red_batch, row_relerr
from oracle import pycwt_spec as pc

pytestmark = pytest.mark.gpu
DT = 1 / 12


def _scales(n0, dj, J):
    return 2 * DT * 2 ** (np.arange(J + 1) * dj)


@pytest.mark.parametrize("n0,dj,J", [(20000, 1 / 4, 40), (32768, 1 / 2, 24), (65536, 1 / 2, 26),
                                     (100000, 1, 14), (300000, 1, 16)])
def test_long_cwt_matches_oracle(n0, dj, J):
    from wtmi import ops
    x = red_batch(n0, 2, n0)
    x[1] += 40.0  # an offset: the removed-mean spectrum path
    sj = _scales(n0, dj, J)
    r = ops.cwt_morlet(torch.tensor(x, device="cuda"), sj, DT, want_w=True, want_power=True)
    W, P = r["w"].cpu().numpy(), r["power"].cpu().numpy()
    for b in range(2):
        ref = pc.cwt(x[b].astype(np.float64), DT, dj, 2 * DT, J)[0]
        assert W.shape[1:] == ref.shape
        gate(f"W[{b}]", row_relerr(W[b].astype(np.complex128), ref))
        gate(f"power[{b}]", row_relerr(P[b].astype(np.float64), np.abs(ref) ** 2))


def test_long_cwt_per_series_significance_and_chunking():
    """Many scales x series so that several scale chunks and series sub-batches run; the
    [B, S] significance multiplier indexes the right series."""
    from wtmi import ops
    n0, dj, J, B = 17000, 1 / 8, 60, 3
    x = red_batch(7, B, n0)
    sj = _scales(n0, dj, J)
    ss = np.stack([np.full(J + 1, 1.0 + b) for b in range(B)])
    r = ops.cwt_morlet(torch.tensor(x, device="cuda"), sj, DT, sig_scale=ss, want_w=False,
                       want_power=True, want_sig=True)
    p, s = r["power"].cpu().numpy(), r["sig"].cpu().numpy()
    for b in range(B):
        np.testing.assert_allclose(s[b], p[b] * (1.0 + b), rtol=1e-6)
    ref = np.abs(pc.cwt(x[2].astype(np.float64), DT, dj, 2 * DT, J)[0]) ** 2
    gate("power[2]", row_relerr(p[2].astype(np.float64), ref))


def test_long_xwt_pair_outputs():
    from wtmi import ops
    n0, dj, J = 40000, 1 / 4, 36
    y1 = red_batch(11, 2, n0)
    y2 = (0.6 * np.roll(y1, 3, axis=1) + 0.8 * red_batch(12, 2, n0)).astype(np.float32)
    sj = _scales(n0, dj, J)
    r = ops.xwt_morlet(torch.tensor(y1, device="cuda"), torch.tensor(y2, device="cuda"), sj, DT,
                       want_w12=True, want_power=True, want_uv=True)
    for b in range(2):
        W12 = (pc.cwt(y1[b].astype(np.float64), DT, dj, 2 * DT, J)[0]
               * pc.cwt(y2[b].astype(np.float64), DT, dj, 2 * DT, J)[0].conj())
        got = r["w12"][b].cpu().numpy().astype(np.complex128)
        gate(f"W12[{b}]", row_relerr(got, W12))
        gate(f"xwt power[{b}]", row_relerr(r["power"][b].cpu().numpy().astype(np.float64), np.abs(W12) ** 2))
        mask = np.abs(W12) > 1e-3 * np.abs(W12).max()
        ang = np.angle(W12)
        np.testing.assert_allclose(r["u"][b].cpu().numpy()[mask], np.sin(ang[mask]), atol=1e-4)
        np.testing.assert_allclose(r["v"][b].cpu().numpy()[mask], np.cos(ang[mask]), atol=1e-4)


@pytest.mark.parametrize("n0,dj", [(20000, 1 / 8), (65536, 1 / 4)])
def test_long_wct_matches_oracle(n0, dj):
    from wtmi import transforms
    y1 = red_batch(n0 + 1, 1, n0)[0].astype(np.float64)
    y2 = 0.6 * np.roll(y1, 3) + 0.8 * red_batch(n0 + 2, 1, n0)[0]
    coh, aw, coi, freq, _ = transforms.wct(y1, y2, DT, dj=dj, s0=2 * DT, J=-1, sig=False)
    rc, ra, rcoi, rfreq, _ = pc.wct(y1, y2, DT, dj=dj, s0=2 * DT, J=-1, sig=False)
    assert coh.shape == rc.shape
    assert np.abs(coh - rc).max() <= 1e-4, np.abs(coh - rc).max()
    W12 = (pc.cwt((y1 - y1.mean()) / y1.std(), DT, dj, 2 * DT, -1)[0]
           * pc.cwt((y2 - y2.mean()) / y2.std(), DT, dj, 2 * DT, -1)[0].conj())
    mask = np.abs(W12) > 1e-3 * np.abs(W12).max()
    assert np.abs(np.angle(np.exp(1j * (aw - ra)))[mask]).max() <= 1e-4


@pytest.mark.parametrize("n0,dj", [(1000, 1 / 32), (700, 1 / 24), (20000, 1 / 24)])
def test_wide_boxcar_wct(n0, dj):
    """dj < 1/20 gives a scale window of K = round(1.2 / dj) > 24 rows (29, 38): the generic
    phase B (short and long rows)."""
    from wtmi import transforms
    y1 = red_batch(n0 + 5, 1, n0)[0].astype(np.float64)
    y2 = 0.6 * np.roll(y1, 3) + 0.8 * red_batch(n0 + 6, 1, n0)[0]
    assert transforms.boxcar_rows(transforms.as_morlet(None), dj) > 24
    coh = transforms.wct(y1, y2, DT, dj=dj, s0=2 * DT, J=-1, sig=False)[0]
    rc = pc.wct(y1, y2, DT, dj=dj, s0=2 * DT, J=-1, sig=False)[0]
    assert np.abs(coh - rc).max() <= 1e-4


def test_wct_significance_long_noise():
    """n = 4096 at the app's settings needs ~6 n = 24576 noise samples per Monte-Carlo
    series (the long-row path); the levels are finite in (0, 1] below maxscale and NaN
    above it (statistical parity with the oracle is tests/test_gpu_wct_sig.py)."""
    from wtmi import transforms
    n0, dj = 4096, 1 / 8
    s0 = 2 * DT
    J = int(np.round(np.log2(n0 * DT / s0) / dj))
    N, sj, _, _, anyout, maxscale = transforms.wct_sig_geometry(DT, dj, s0, J)
    assert N > 16384
    sig = transforms.wct_significance(0.6, 0.4, DT, dj, s0, J, mc_count=60, cache=False, seed=3)
    assert sig.shape == (J + 1,)
    ok = sig[:maxscale]
    assert np.isfinite(ok).all() and (ok > 0).all() and (ok <= 1).all()
    assert np.isnan(sig[maxscale:][anyout[maxscale:]]).all()


def test_too_long_rows_raise_clearly():
    from wtmi import ops
    with pytest.raises(ValueError, match="at most"):
        ops.cwt_morlet(torch.zeros(1, (1 << 20) + 1, device="cuda"), [1.0], DT)


@pytest.mark.parametrize("n,J", [(20000, 10), (65536, 12), (40001, 5)])
def test_long_modwt_matches_oracle(n, J, db4):
    """n > 16384: one launch per level through HBM (csrc/modwt.hip modwt_long)."""
    from oracle import modwt_spec as ms
    from wtmi import ops
    x = red_batch(n + 3, 3, n)
    xd = torch.tensor(x, device="cuda")
    W = ops.modwt(xd, db4["dec_lo"], db4["dec_hi"], J)
    for b in (0, 2):
        ref = ms.modwt_direct(x[b].astype(np.float64), db4["dec_lo"], db4["dec_hi"], J)
        got = W[b].cpu().numpy().astype(np.float64)
        assert np.abs(got - ref).max() <= 1e-5 * np.abs(ref).max(axis=1).max()
        assert row_relerr(got, ref).max() <= 1e-5
    back = ops.imodwt(W, db4["dec_lo"], db4["dec_hi"]).cpu().numpy()
    assert np.abs(back - x).max() <= 1e-5 * np.abs(x).max()
    # synthesis of a non-range input and of a masked row (MRA component) vs the oracle
    rng = np.random.default_rng(n)
    wr = rng.standard_normal((1, J + 1, n)).astype(np.float32)
    got = ops.imodwt(torch.tensor(wr, device="cuda"), db4["dec_lo"], db4["dec_hi"]).cpu().numpy()[0]
    ref = ms.imodwt_direct(wr[0].astype(np.float64), db4["dec_lo"], db4["dec_hi"])
    assert np.abs(got - ref).max() <= 3e-5 * np.abs(ref).max()
    iso = W[:1].clone()
    comp = ops.imodwt(iso, db4["dec_lo"], db4["dec_hi"], keep_mask=1 << 2).cpu().numpy()[0]
    only = np.zeros((J + 1, n))
    only[2] = W[0, 2].cpu().numpy()
    ref = ms.imodwt_direct(only, db4["dec_lo"], db4["dec_hi"])
    assert np.abs(comp - ref).max() <= 1e-5 * max(np.abs(ref).max(), 1e-12)


@pytest.mark.parametrize("n,level", [(20000, None), (65537, 6), (30000, 0)])
def test_long_dwt_matches_oracle(n, level, db4):
    from oracle import dwt_spec as ds
    from wtmi import ops, transforms
    x = red_batch(n + 9, 2, n).astype(np.float64)
    lev = transforms.dwt_max_level(n, 8) if level is None else level
    C, lens = ops.wavedec(torch.tensor(x, device="cuda"), db4["dec_lo"], db4["dec_hi"], lev)
    for b in range(2):
        ref = ds.wavedec(x[b], db4["dec_lo"], db4["dec_hi"], lev)
        assert [r.size for r in ref] == lens
        flat = np.concatenate(ref)
        assert np.abs(C[b].cpu().numpy() - flat).max() <= 1e-5 * np.abs(flat).max()
    full = (1 << (lev + 1)) - 1
    masks = [full, 1, 1 << lev] if lev > 0 else [full, 0]
    R = ops.waverec(C, n, db4["rec_lo"], db4["rec_hi"], lev, masks).cpu().numpy()
    coeffs = ds.wavedec(x[1], db4["dec_lo"], db4["dec_hi"], lev)
    for v, m in enumerate(masks):
        kept = [c if (m >> k) & 1 else np.zeros_like(c) for k, c in enumerate(coeffs)]
        ref = ds.waverec(kept, db4["rec_lo"], db4["rec_hi"])
        got = R[1, v, :ref.size]
        assert np.abs(got - ref).max() <= 1e-5 * max(np.abs(x[1]).max(), 1e-12), (v, m)


@pytest.mark.parametrize("n0,dj", [(2, 1 / 8), (3, 1 / 8), (5, 1 / 12), (8, 1 / 8), (7, 1 / 32)])
def test_tiny_wct_matches_oracle(n0, dj):
    """n0 <= 8 (N <= 8, below the FFT engine's 16-point row): the direct fp64 WCT kernel."""
    from wtmi import transforms
    rng = np.random.default_rng(n0)
    y1 = rng.standard_normal(n0).cumsum()
    y2 = 0.5 * y1 + rng.standard_normal(n0)
    coh, aw, coi, freq, _ = transforms.wct(y1, y2, DT, dj=dj, s0=2 * DT, J=-1, sig=False)
    rc, ra, rcoi, rfreq, _ = pc.wct(y1, y2, DT, dj=dj, s0=2 * DT, J=-1, sig=False)
    assert coh.shape == rc.shape
    # n0 = 2: pycwt's normalisation sqrt(s * 2 pi fftfreq(2)[1] / dt * N) is the root of a
    # negative number, every coefficient NaN; the engine returns the same NaNs
    np.testing.assert_allclose(coh, rc, rtol=0, atol=1e-4, equal_nan=True)
    assert np.isnan(coh).all() == (n0 == 2)
    np.testing.assert_allclose(freq, rfreq, rtol=1e-12)


@pytest.mark.parametrize("n0", [2, 3, 5, 8])
def test_tiny_cwt_matches_oracle(n0):
    """n0 <= 8: the direct CWT kernel; n0 = 2 is all-NaN in pycwt (and here)."""
    from wtmi import ops
    rng = np.random.default_rng(100 + n0)
    x = rng.standard_normal((2, n0)).astype(np.float32)
    sj = _scales(n0, 1 / 8, 12)
    W = ops.cwt_morlet(torch.tensor(x, device="cuda"), sj, DT)["w"].cpu().numpy()
    for b in range(2):
        ref = pc.cwt(x[b].astype(np.float64), DT, 1 / 8, 2 * DT, 12)[0]
        np.testing.assert_allclose(W[b], ref, rtol=0, atol=1e-5 * np.nanmax(np.abs(ref), initial=1.0),
                                   equal_nan=True)
