"""WCT kernels, per-series moments and the drop-in src.* modules vs the oracle.

WCT tolerance: coherence elementwise abs <= 1e-4; phase arrows compared
where |W12| > 1e-3 max.  The drop-in modules are compared with the oracle's
restatement of the reference wrapper glue (oracle/glue_spec.py).
"""

import os

import numpy as np
import pandas as pd
import pytest
import torch

from gpu_helpers import gate, red_series, row_relerr
from oracle import glue_spec as gs
from oracle import pycwt_spec as pc

pytestmark = pytest.mark.gpu
SAMPLE = os.path.join(os.path.dirname(__file__), "golden", "sample_data")


def load_sample(name):
    df = pd.read_csv(os.path.join(SAMPLE, name), sep=None, parse_dates=[0], index_col=0,
                     engine="python")
    return df.iloc[:, 0].to_numpy(dtype=float), df.index.to_numpy()


def _pair(rng, n):
    y1 = red_series(rng, n).astype(np.float64)
    y2 = 0.6 * np.roll(y1, 3) + 0.8 * red_series(rng, n)
    return y1, y2


@pytest.mark.parametrize("n,dj", [(64, 1 / 8), (256, 1 / 8), (1000, 1 / 8), (1333, 1 / 12),
                                  (2048, 1 / 8), (5000, 1 / 8), (8192, 1 / 8), (16384, 1 / 4)])
def test_wct_matches_oracle(n, dj):
    from wtmi import transforms
    rng = np.random.default_rng(n)
    y1, y2 = _pair(rng, n)
    coh, aw, coi, freq, sig = transforms.wct(y1, y2, 1 / 12, dj=dj, s0=2 / 12, J=-1, sig=False)
    rc, ra, rcoi, rfreq, rsig = pc.wct(y1, y2, 1 / 12, dj=dj, s0=2 / 12, J=-1, sig=False)
    assert coh.shape == rc.shape
    gate("coherence abs", np.abs(coh - rc), 1e-4)
    W12 = (pc.cwt((y1 - y1.mean()) / y1.std(), 1 / 12, dj, 2 / 12, -1)[0]
           * pc.cwt((y2 - y2.mean()) / y2.std(), 1 / 12, dj, 2 / 12, -1)[0].conj())
    mask = np.abs(W12) > 1e-3 * np.abs(W12).max()
    dphi = np.angle(np.exp(1j * (aw - ra)))
    gate("phase rad", np.abs(dphi[mask]), 1e-4)
    np.testing.assert_allclose(coi, rcoi, rtol=1e-12)
    np.testing.assert_allclose(freq, rfreq, rtol=1e-12)


@pytest.mark.parametrize("n,B", [(1000, 3), (8192, 2)])
def test_wct_fused_power_and_phase_outputs(n, B):
    """n = 8192 runs the C4 shape: rows of every band regime, the narrowest through the
    spectral-correlation path of phase A."""
    from wtmi import ops, transforms  # noqa: F401
    rng = np.random.default_rng(31)
    pairs = [_pair(rng, n) for _ in range(B)]
    y1 = torch.tensor(np.stack([p[0] for p in pairs]), device="cuda", dtype=torch.float32)
    y2 = torch.tensor(np.stack([p[1] for p in pairs]), device="cuda", dtype=torch.float32)
    res, sj, _ = transforms.wct_batch(y1, y2, 1 / 12, 1 / 8, 2 / 12, -1, want_uv=True,
                                      want_power=True, want_phase=True)
    for b in range(B):
        a1 = y1[b].cpu().numpy().astype(np.float64)
        a2 = y2[b].cpu().numpy().astype(np.float64)
        W12 = (pc.cwt((a1 - a1.mean()) / a1.std(), 1 / 12, 1 / 8, 2 / 12, -1)[0]
               * pc.cwt((a2 - a2.mean()) / a2.std(), 1 / 12, 1 / 8, 2 / 12, -1)[0].conj())
        p = res["power"][b].cpu().numpy().astype(np.float64)
        gate(f"wct power[{b}]", row_relerr(p, np.abs(W12) ** 2))
        mask = np.abs(W12) > 1e-3 * np.abs(W12).max()
        ph = res["phase"][b].cpu().numpy()
        assert np.abs(np.angle(np.exp(1j * (ph - np.angle(W12))))[mask]).max() < 1e-4
        u, v = res["u"][b].cpu().numpy(), res["v"][b].cpu().numpy()
        np.testing.assert_allclose(u[mask], np.sin(ph[mask]), atol=1e-5)
        np.testing.assert_allclose(v[mask], np.cos(ph[mask]), atol=1e-5)
        rc = pc.wct(a1, a2, 1 / 12, dj=1 / 8, s0=2 / 12, J=-1, sig=False)[0]
        gate(f"coherence abs[{b}]", np.abs(res["coh"][b].cpu().numpy() - rc), 1e-4)


@pytest.mark.parametrize("n,dj", [(1024, 1 / 8), (2048, 1 / 12), (4096, 1 / 12), (8000, 1 / 8),
                                  (8192, 1 / 8), (3000, 1 / 16), (16384, 1 / 4)])
def test_wct_band_paths_match_unpruned(n, dj):
    """Band-pruned transforms, the spectral-correlation rows of phase A, the decimated spectra
    of full rows (wct_prune 2: forward transforms on every (N/M)-th sample, band inverses of
    M bins) and phase C's band-spectrum coherence against the unpruned path (six full
    transforms per row, every output row through phase B).  Boxcar widths 14, 10, 19 and 5
    rows; padded and full rows."""
    from wtmi import transforms
    rng = np.random.default_rng(n + 11)
    B = 2
    pairs = [_pair(rng, n) for _ in range(B)]
    y1 = torch.tensor(np.stack([p[0] for p in pairs]), device="cuda", dtype=torch.float32)
    y2 = torch.tensor(np.stack([p[1] for p in pairs]), device="cuda", dtype=torch.float32)
    out = {}
    from wtmi import _lib
    for prune in (0, 1, 2):
        with _lib.option("wct_prune", prune):
            res, _, _ = transforms.wct_batch(y1, y2, 1 / 12, dj, 2 / 12, -1, want_uv=False,
                                             want_power=True, want_phase=True)
        out[prune] = {k: v.cpu().numpy().astype(np.float64) for k, v in res.items()}
    full = out[0]
    # phases where |W12| > 1e-2 of its row's max: fp32 transforms leave |dW12| ~ 1e-6 of the
    # row max in every path (the unpruned one included: 1.4e-4 rad against the fp64 oracle at
    # 1e-3..1e-2 of the row max, scripts/debug/wct_phase_err.py), i.e. <= 1e-4 rad from there on
    mask = full["power"] > 1e-4 * full["power"].max(axis=-1, keepdims=True)
    for band in (out[1], out[2]):
        gate("coherence band vs unpruned", np.abs(full["coh"] - band["coh"]), 2e-5)
        gate("power band vs unpruned", row_relerr(band["power"], full["power"]))
        dphi = np.angle(np.exp(1j * (band["phase"] - full["phase"])))
        assert np.abs(dphi[mask]).max() <= 1e-4


def test_wct_batched_self_coherence_is_one():
    from wtmi import transforms
    rng = np.random.default_rng(2)
    B, n = 8, 512
    y = torch.tensor(np.stack([red_series(rng, n) for _ in range(B)]), device="cuda")
    res, sj, _ = transforms.wct_batch(y, y, 1 / 12, 1 / 8, 2 / 12, -1)
    c = res["coh"].cpu().numpy()
    assert np.abs(c - 1).max() < 1e-4


def test_moments_and_standardize_match_numpy():
    from wtmi import ops, transforms
    rng = np.random.default_rng(4)
    for n in (2, 17, 1333, 5000):
        x = rng.standard_normal(n).cumsum() + 100
        m = ops.series_moments(torch.tensor(x, device="cuda")).cpu().numpy()[0]
        p = np.polyfit(np.arange(n), x, 1)
        xc = x - x.mean()
        np.testing.assert_allclose(m[:4], [x.mean(), x.std(), p[0], p[1]], rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(m[4], xc @ xc / n, rtol=1e-10)
        np.testing.assert_allclose(m[5], xc[:-1] @ xc[1:] / (n - 1), rtol=1e-10, atol=1e-12)
        for kw in (dict(), dict(detrend=False, remove_mean=True), dict(detrend=False),
                   dict(standardize=False)):
            np.testing.assert_allclose(transforms.standardize_series(x, **kw),
                                       gs.standardize_series(x, **kw), rtol=1e-9, atol=1e-9)
    with pytest.raises(ValueError):
        transforms.standardize_series(x, detrend=True, remove_mean=True)
    # the one-pass affine coefficients (wtmi_series_affine) == the moments-derived ones
    xs = torch.tensor(rng.standard_normal((3, 777)).cumsum(1) + 50, device="cuda")
    mom = ops.series_moments(xs)
    for det, std, rm in ((True, True, False), (False, True, True), (False, True, False), (True, False, False)):
        mode = (ops.AFF_DETREND if det else 0) | (ops.AFF_STANDARDIZE if std else 0) | \
            (ops.AFF_REMOVE_MEAN if rm else 0)
        torch.testing.assert_close(ops.series_affine(xs, mode),
                                   transforms.standardize_coefs(mom, det, std, rm), rtol=1e-14, atol=0)
    torch.testing.assert_close(ops.series_affine(xs.float()), transforms.normalize_coefs(ops.series_moments(xs.float())),
                               rtol=1e-14, atol=0)
    with pytest.raises(ValueError):
        ops.series_affine(xs, ops.AFF_DETREND | ops.AFF_REMOVE_MEAN)


def test_ar1_and_cpi_fallback_warning():
    from wtmi import transforms
    y, _ = load_sample("inflation.csv")
    ys = gs.standardize_series(y)
    g, a, mu2 = transforms.ar1(ys)
    rg, ra, rmu = pc.ar1(ys)
    np.testing.assert_allclose([g, a, mu2], [rg, ra, rmu], rtol=1e-9)
    cpi, _ = load_sample("cpi.csv")
    with pytest.raises(Warning):
        transforms.ar1(gs.standardize_series(cpi))


def test_src_cwt_run_cwt_on_inflation():
    import src.cwt as cwt
    from src.utils.wavelet_helpers import standardize_series
    y, t = load_sample("inflation.csv")
    ys = standardize_series(y)  # the app standardises before run_cwt (quirk B.2)
    data = cwt.DataForCWT(t, ys, cwt.MOTHER, cwt.DT, cwt.DJ, cwt.S0, cwt.LEVELS)
    assert data.time_range.shape == (y.size,)
    for kwargs in (dict(), dict(standardize=True), dict(calculate_significance=False)):
        res = cwt.run_cwt(data, **kwargs)
        p, period, sig, coi = gs.run_cwt(
            ys, y.size, standardize=kwargs.get("standardize", False),
            calculate_significance=kwargs.get("calculate_significance", True))
        assert res.power.shape == p.shape == (85, 1333)
        gate(f"run_cwt power {sorted(kwargs)}", row_relerr(res.power, p))
        np.testing.assert_allclose(res.period, period, rtol=1e-12)
        np.testing.assert_allclose(res.coi, coi, rtol=1e-12)
        if sig is None:
            assert res.significance_levels is None
        else:
            gate(f"run_cwt sig ratio {sorted(kwargs)}", row_relerr(res.significance_levels, sig))


def test_src_cwt_64_scales_config1():
    """BASELINE config 1: inflation.csv, 64 scales (J = 63)."""
    from wtmi import ops, transforms
    y, _ = load_sample("inflation.csv")
    ys = gs.standardize_series(y)
    sj, freqs = transforms.scales_for(y.size, 1 / 12, 1 / 12, 2 / 12, 63, transforms.as_morlet(None))
    assert sj.size == 64
    P = ops.cwt_morlet(torch.tensor(ys, device="cuda", dtype=torch.float32), sj, 1 / 12,
                       want_w=False, want_power=True)["power"][0].cpu().numpy()
    ref = np.abs(pc.cwt(ys.astype(np.float32).astype(np.float64), 1 / 12, 1 / 12, 2 / 12, 63)[0]) ** 2
    gate("C1 power", row_relerr(P.astype(np.float64), ref))


def test_src_xwt_and_wct(monkeypatch):
    import src.wct as wct
    import src.xwt as xwt
    rng = np.random.default_rng(12)
    y1, y2 = _pair(rng, 600)
    d = xwt.DataForXWT(y1, y2, xwt.MOTHER_DICT["morlet"], xwt.DT, xwt.DJ, xwt.S0, xwt.LEVELS)
    r = xwt.run_xwt(d)
    ref = gs.run_xwt(y1, y2, xwt.DT, xwt.DJ, xwt.S0, xwt.LEVELS)
    assert r.power.shape == ref[0].shape
    gate("run_xwt power", row_relerr(r.power, ref[0]))
    np.testing.assert_allclose(r.period, ref[1], rtol=1e-12)
    gate("run_xwt sig ratio", row_relerr(r.significance_levels, ref[2]))
    np.testing.assert_allclose(r.coi, ref[3], rtol=1e-12)
    assert r.phase_diff_u.shape == ref[4].shape  # phase at dj = 1/12 (quirk B.5)
    assert r.phase_diff_u.shape[0] != r.power.shape[0]
    W12 = (pc.cwt((y1 - y1.mean()) / y1.std(), 1 / 12, 1 / 12, xwt.S0, -1)[0]
           * pc.cwt((y2 - y2.mean()) / y2.std(), 1 / 12, 1 / 12, xwt.S0, -1)[0].conj())
    mask = np.abs(W12) > 1e-3 * np.abs(W12).max()
    np.testing.assert_allclose(r.phase_diff_u[mask], ref[4][mask], atol=1e-4)
    np.testing.assert_allclose(r.phase_diff_v[mask], ref[5][mask], atol=1e-4)

    dw = wct.DataForWCT(y1, y2, wct.MOTHER_DICT["morlet"], wct.DT, wct.DJ, wct.S0, wct.LEVELS)
    rw = wct.run_wct(dw, calculate_signficance=False)
    refw = gs.run_wct(y1, y2, wct.DT, wct.DJ, wct.S0)
    gate("run_wct coherence abs", np.abs(rw.coherence - refw[0]), 1e-4)
    assert np.isinf(rw.significance_levels).all() and np.isinf(refw[2]).all()  # quirk B.8
    # significance on (the reference's default): Monte-Carlo levels from pycwt's masked
    # counter ("Monte-Carlo quantile"; test_gpu_wct_sig.py pins them statistically),
    # the coherence unchanged and the ratio |coh| / sig95 per scale; the explicit
    # quantile="unmasked" reading raises
    from wtmi import transforms
    rs = wct.run_wct(dw, calculate_signficance=True)
    np.testing.assert_array_equal(rs.coherence, rw.coherence)
    fin = np.isfinite(rs.significance_levels)
    assert fin.any() and (rs.significance_levels[fin] > 0).all()
    monkeypatch.setattr(transforms, "SIG_QUANTILE", "unmasked")
    with pytest.raises(ValueError, match="object too deep for desired array"):
        wct.run_wct(dw, calculate_signficance=True)


@pytest.mark.parametrize("normalize", [True, False])
def test_xwt_significance_on_app_shaped_series(normalize):
    """sigma != 1 inputs as create_xwt_dict builds them (detrended, then divided by the
    ORIGINAL std: src/utils/transform_helpers.py:74-75, src/utils/wavelet_helpers.py:22-57).
    pycwt.xwt resets std1 = std2 = 1 when it normalises, so the significance ratio of
    run_xwt must not carry sigma1 sigma2 (parity unpinned: pycwt is absent, the oracle
    restates it)."""
    import src.xwt as xwt
    from wtmi import transforms
    rng = np.random.default_rng(77)
    n = 700
    t = np.arange(n)
    y1r = 3.0 * red_series(rng, n) + 0.05 * t + 40
    y2r = 0.5 * np.roll(y1r, 5) + 2.0 * red_series(rng, n) - 0.1 * t
    y1, y2 = gs.standardize_series(y1r), gs.standardize_series(y2r)
    assert abs(y1.std() - 1) > 0.05 and abs(y2.std() - 1) > 0.05
    # pycwt-level xwt under both normalize values
    W12, coi, freq, signif = transforms.xwt(y1, y2, xwt.DT, xwt.DJ, xwt.S0, normalize=normalize)
    rW12, rcoi, rfreq, rsignif = pc.xwt(y1, y2, xwt.DT, xwt.DJ, xwt.S0, normalize=normalize)
    np.testing.assert_allclose(signif, rsignif, rtol=1e-9)
    gate("xwt W12", row_relerr(W12, rW12))
    ratio = rsignif / pc.xwt(y1, y2, xwt.DT, xwt.DJ, xwt.S0, normalize=True)[3]
    if normalize:
        np.testing.assert_allclose(ratio, 1.0)
    else:
        np.testing.assert_allclose(ratio, y1.std() * y2.std(), rtol=1e-12)
    # drop-in run_xwt: the reference always calls pycwt.xwt with normalize=True
    d = xwt.DataForXWT(y1, y2, xwt.MOTHER_DICT["morlet"], xwt.DT, xwt.DJ, xwt.S0, xwt.LEVELS)
    if not normalize:  # the reference's run_xwt raises NameError (quirk B.7), so does this one
        with pytest.raises(NameError):
            xwt.run_xwt(d, normalize=False)
    r = xwt.run_xwt(d) if normalize else xwt.run_xwt_batch([d], normalize=False)[0]
    if normalize:
        ref = gs.run_xwt(y1, y2, xwt.DT, xwt.DJ, xwt.S0, xwt.LEVELS)
        gate("run_xwt power", row_relerr(r.power, ref[0]))
        gate("run_xwt sig ratio", row_relerr(r.significance_levels, ref[2]))
    else:  # engine extension run_xwt_batch(normalize=False): raw W12 and W12 / signif
        rW12n, _, rf, rs = pc.xwt(y1, y2, xwt.DT, xwt.DJ, xwt.S0)
        gate("run_xwt_batch raw W12", row_relerr(r.power, rW12n))
        gate("run_xwt_batch raw sig ratio", row_relerr(r.significance_levels, rW12n / rs[:, None]))


def test_src_dwt_and_modwt(dwt_golden, modwt_golden):
    import src.dwt as dwt
    import src.modwt as modwt
    g = dwt_golden
    for i in range(int(g["ncases"])):
        if f"c{i}_comp0" not in g:
            continue
        x = g[f"c{i}_x"]
        nlev = int(g[f"c{i}_nlev"])
        lvl0 = int(g[f"c{i}_level"])
        res = dwt.run_dwt(dwt.DataForDWT(x, dwt.MOTHER, None if lvl0 < 0 else lvl0))
        assert res.levels == nlev - 1
        for k, c in enumerate(res.coeffs):
            ref = g[f"c{i}_coef{k}"]
            assert c.shape == ref.shape and np.abs(c - ref).max() <= 1e-5 * np.abs(ref).max()
        res.smooth_signal(x, dwt.MOTHER)
        for lvl, dd in res.smoothed_signal_dict.items():
            ref = g[f"c{i}_smooth{lvl}"]
            assert np.abs(dd["signal"] - ref).max() <= 1e-5 * np.abs(ref).max()
        comp = dwt.reconstruct_signal_component(res.coeffs, dwt.MOTHER, 1)
        ref = g[f"c{i}_comp1"]
        assert np.abs(comp - ref).max() <= 1e-5 * max(np.abs(ref).max(), 1e-12)
        # every component (served by the batched cache) bitwise equal to its own launch
        from wtmi import transforms
        for lvl in range(len(res.coeffs)):
            got = dwt.reconstruct_signal_component(res.coeffs, dwt.MOTHER, lvl)
            one = transforms.waverec_variants(res.coeffs, dwt.MOTHER, [1 << lvl])[0]
            assert np.array_equal(got, one)
            if f"c{i}_comp{lvl}" in g:
                ref = g[f"c{i}_comp{lvl}"]
                assert np.abs(got - ref).max() <= 1e-5 * max(np.abs(ref).max(), 1e-12)
    m = modwt_golden
    for i in range(int(m["ncases"])):
        x, w, J = m[f"c{i}_x"], m[f"c{i}_w"], int(m[f"c{i}_J"])
        got = modwt.modwt(x, "db4", J)
        assert got.dtype == x.dtype and got.shape == w.shape
        assert np.abs(got - w).max() <= 1e-5 * np.abs(w).max()
        if f"c{i}_mra" in m:
            mra = modwt.modwtmra(w, "db4")
            assert np.abs(mra - m[f"c{i}_mra"]).max() <= 1e-5 * np.abs(w).max()
