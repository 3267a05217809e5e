"""MODWT / DWT kernel parity vs vectors produced by the reference's own code.

MODWT golden vectors: src/modwt.py functions run in the build container
(tests/golden/make_golden.py).  DWT golden vectors: PyWavelets 1.1.1.
Tolerance: row order/shape identical; per row normwise <= 1e-5 and
elementwise abs <= 1e-5 * max|row|; round trip ||x^ - x||_inf <= 1e-5 ||x||_inf.
"""

import numpy as np
import pytest
import torch

from gpu_helpers import red_series, row_relerr
from oracle import dwt_spec as ds
from oracle import glue_spec as gs
from oracle import modwt_spec as ms

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _ops():
    from wtmi import ops
    return ops


def _check_rows(got, ref):
    """Per row: normwise <= TOL and elementwise <= TOL * max|row|.  Rows that vanish
    analytically (e.g. dilation = 0 mod N, where the taps sum to 0) hold only fp
    round-off in either implementation, so every row also gets an absolute floor of
    TOL * 1e-1 * the largest row max (documented in DESIGN.md)."""
    assert got.shape == ref.shape
    floor = 0.1 * TOL * np.abs(ref).max()
    num = np.linalg.norm((got - ref).reshape(-1, ref.shape[-1]).astype(np.float64), axis=-1)
    den = np.linalg.norm(ref.reshape(-1, ref.shape[-1]).astype(np.float64), axis=-1)
    assert (num <= TOL * den + floor * np.sqrt(ref.shape[-1])).all(), (num / np.maximum(den, 1e-300)).max()
    scale = np.abs(ref).max(axis=-1, keepdims=True)
    assert (np.abs(got - ref) <= TOL * scale + floor).all()


def test_modwt_matches_reference_golden(modwt_golden, db4):
    g = modwt_golden
    ops = _ops()
    for i in range(int(g["ncases"])):
        x, w, J = g[f"c{i}_x"], g[f"c{i}_w"], int(g[f"c{i}_J"])
        got = ops.modwt(torch.tensor(x.astype(np.float32), device="cuda"), db4["dec_lo"],
                        db4["dec_hi"], J)[0].cpu().numpy()
        assert got.shape == (J + 1, x.size)  # [W_1 .. W_J, V_J]
        _check_rows(got, w)
        inv = ops.imodwt(torch.tensor(w.astype(np.float32), device="cuda"), db4["dec_lo"],
                         db4["dec_hi"])[0].cpu().numpy()
        ref = g[f"c{i}_inv"]
        assert np.abs(inv - ref).max() <= TOL * np.abs(ref).max()
        if f"c{i}_wrand" in g:  # adjoint on non-range input
            inv = ops.imodwt(torch.tensor(g[f"c{i}_wrand"].astype(np.float32), device="cuda"),
                             db4["dec_lo"], db4["dec_hi"])[0].cpu().numpy()
            ref = g[f"c{i}_invrand"]
            assert np.abs(inv - ref).max() <= 3 * TOL * np.abs(ref).max()


def test_modwt_masks_give_mra_and_smoothing(modwt_golden, db4):
    g = modwt_golden
    ops = _ops()
    for i in range(int(g["ncases"])):
        if f"c{i}_mra" not in g:
            continue
        w = g[f"c{i}_w"]
        J = int(g[f"c{i}_J"])
        wd = torch.tensor(w.astype(np.float32), device="cuda")
        mra = np.stack([ops.imodwt(wd, db4["dec_lo"], db4["dec_hi"], 1 << j)[0].cpu().numpy()
                        for j in range(J + 1)])
        ref = g[f"c{i}_mra"]
        assert np.abs(mra - ref).max() <= TOL * np.abs(ref).max()
        for lvl in range(1, J + 1):
            keep = ((1 << (J + 1)) - 1) & ~((1 << lvl) - 1)
            s = ops.imodwt(wd, db4["dec_lo"], db4["dec_hi"], keep)[0].cpu().numpy()
            r = g[f"c{i}_smooth{lvl}"]
            assert np.abs(s - r).max() <= TOL * max(1.0, np.abs(r).max())


@pytest.mark.parametrize("n", [1000, 4096, 16384])
def test_modwt_batched_round_trip_and_energy(n, db4):
    rng = np.random.default_rng(n)
    B, J = 16, 10
    x = np.stack([red_series(rng, n) for _ in range(B)])
    ops = _ops()
    xd = torch.tensor(x, device="cuda")
    w = ops.modwt(xd, db4["dec_lo"], db4["dec_hi"], J)
    xr = ops.imodwt(w, db4["dec_lo"], db4["dec_hi"]).cpu().numpy()
    assert np.abs(xr - x).max() <= TOL * np.abs(x).max()
    wn = w.cpu().numpy().astype(np.float64)
    np.testing.assert_allclose((wn ** 2).sum(axis=(1, 2)), (x.astype(np.float64) ** 2).sum(axis=1),
                               rtol=1e-5)
    # spot-check two series against the textbook oracle
    for b in (0, B - 1):
        ref = ms.modwt_direct(x[b].astype(np.float64), db4["dec_lo"], db4["dec_hi"], J)
        _check_rows(wn[b], ref)


@pytest.mark.parametrize("n,J", [(64, 9), (200, 10), (1000, 12), (4096, 13)])
def test_modwt_dilations_past_n(n, J, db4):
    """Levels whose dilation 2^(j-1) reaches or passes n (taken mod n, possibly 0):
    the vectorised kernels' dilation/tap-offset arithmetic vs the textbook oracle."""
    rng = np.random.default_rng(n + J)
    x = np.stack([red_series(rng, n) for _ in range(3)])
    ops = _ops()
    w = ops.modwt(torch.tensor(x, device="cuda"), db4["dec_lo"], db4["dec_hi"], J)
    wn = w.cpu().numpy()
    for b in range(3):
        _check_rows(wn[b], ms.modwt_direct(x[b].astype(np.float64), db4["dec_lo"], db4["dec_hi"], J))
    xr = ops.imodwt(w, db4["dec_lo"], db4["dec_hi"]).cpu().numpy()
    assert np.abs(xr - x).max() <= TOL * np.abs(x).max()


def test_modwt_other_filter_lengths(pywt_filters):
    rng = np.random.default_rng(3)
    ops = _ops()
    for name in ("haar", "db2", "sym8", "coif3", "db20"):
        f = pywt_filters[name]
        for n in (128, 333):
            x = red_series(rng, n)
            w = ops.modwt(torch.tensor(x, device="cuda"), f["dec_lo"], f["dec_hi"], 4)[0].cpu().numpy()
            ref = ms.modwt(x.astype(np.float64), f["dec_lo"], f["dec_hi"], 4)
            _check_rows(w, ref)


def _dwt_case(g, i):
    nlev = int(g[f"c{i}_nlev"])
    lvl = int(g[f"c{i}_level"])
    return (g[f"c{i}_x"], str(g[f"c{i}_wavelet"]), None if lvl < 0 else lvl,
            [g[f"c{i}_coef{k}"] for k in range(nlev)])


def test_wavedec_waverec_match_pywt_golden(dwt_golden, pywt_filters):
    g = dwt_golden
    ops = _ops()
    for i in range(int(g["ncases"])):
        x, wname, level, coeffs = _dwt_case(g, i)
        f = pywt_filters[wname]
        lev = len(coeffs) - 1
        ct, lens = ops.wavedec(torch.tensor(x.astype(np.float32), device="cuda"), f["dec_lo"],
                               f["dec_hi"], lev)
        assert lens == [c.size for c in coeffs], (i, lens)
        flat = ct[0].cpu().numpy()
        off = 0
        for c in coeffs:
            got = flat[off:off + c.size]
            off += c.size
            assert np.abs(got - c).max() <= TOL * max(np.abs(c).max(), 1e-30), (i, wname)
        full = (1 << len(coeffs)) - 1
        cin = torch.tensor(np.concatenate(coeffs).astype(np.float32), device="cuda")
        rec = ops.waverec(cin, x.size, f["rec_lo"], f["rec_hi"], lev, [full])[0, 0].cpu().numpy()
        ref = g[f"c{i}_rec"]
        assert rec.size == ref.size
        assert np.abs(rec - ref).max() <= TOL * np.abs(ref).max()


def test_dwt_smooth_and_components_batched(dwt_golden, pywt_filters):
    g = dwt_golden
    f = pywt_filters["db4"]
    ops = _ops()
    for i in range(int(g["ncases"])):
        if f"c{i}_comp0" not in g:
            continue
        x, _, _, coeffs = _dwt_case(g, i)
        lev = len(coeffs) - 1
        nl = len(coeffs)
        full = (1 << nl) - 1
        smooth_masks = []
        for lvl in range(lev, 0, -1):
            m = full
            for k in range(1, lvl + 1):
                m &= ~(1 << (nl - k))
            smooth_masks.append(m)
        comp_masks = [1 << k for k in range(nl)]
        cin = torch.tensor(np.concatenate(coeffs).astype(np.float32), device="cuda")
        out = ops.waverec(cin, x.size, f["rec_lo"], f["rec_hi"], lev,
                          smooth_masks + comp_masks)[0].cpu().numpy()
        for vi, lvl in enumerate(range(lev, 0, -1)):
            got = gs.trim_signal(x, out[vi])
            ref = g[f"c{i}_smooth{lvl}"]
            assert np.abs(got - ref).max() <= TOL * np.abs(ref).max()
        for k in range(nl):
            ref = g[f"c{i}_comp{k}"]
            got = out[len(smooth_masks) + k]
            assert np.abs(got - ref).max() <= TOL * max(np.abs(ref).max(), 1e-12)


def test_wavedec_batched_vs_oracle():
    rng = np.random.default_rng(8)
    from wtmi.wavelets import Wavelet
    w = Wavelet("db4")
    B, n = 32, 4097
    x = np.stack([red_series(rng, n) for _ in range(B)])
    lev = ds.dwt_max_level(n, 8)
    ct, lens = _ops().wavedec(torch.tensor(x, device="cuda"), w.dec_lo, w.dec_hi, lev)
    ct = ct.cpu().numpy()
    for b in (0, 17, 31):
        ref = np.concatenate(ds.wavedec(x[b].astype(np.float64), w.dec_lo, w.dec_hi, lev))
        assert np.abs(ct[b] - ref).max() <= TOL * np.abs(ref).max()


@pytest.mark.parametrize("syn", [1, 2, 0])
@pytest.mark.parametrize("n,J", [(16384, 10), (16384, 15), (8192, 12), (4096, 3)])
def test_imodwt_adjoint_and_masks_at_bench_shape(n, J, syn, db4):
    """Synthesis on NON-range input (adjoint, every tap exercised) and with row masks at
    the C3 shape vs the textbook oracle, for the n = 16384 / 8192 kernels (option modwt_syn: 1
    the hybrid with every level staged through LDS, 2 the hybrid with chain levels from L2,
    0 dilation chains only).  J = 15 reaches dilations
    past the chain range (2^12 samples) and 2^14 = 0 mod n."""
    from wtmi import _lib
    rng = np.random.default_rng(n + J)
    w = rng.standard_normal((2, J + 1, n)).astype(np.float32)
    ops = _ops()
    wd = torch.tensor(w, device="cuda")
    for keep in ((1 << (J + 1)) - 1, 0b101 << (J - 2), 1 << J, 0b1011):
        with _lib.option("modwt_syn", syn):
            got = ops.imodwt(wd, db4["dec_lo"], db4["dec_hi"], keep).cpu().numpy()
        for b in range(2):
            wm = w[b].astype(np.float64) * np.array([(keep >> r) & 1 for r in range(J + 1)])[:, None]
            ref = ms.imodwt_direct(wm, db4["dec_lo"], db4["dec_hi"])
            assert np.abs(got[b] - ref).max() <= 3 * TOL * np.abs(ref).max(), (keep, b)
