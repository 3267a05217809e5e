"""Known-answer tests that pin the (otherwise unpinned) pycwt restatement.

pycwt 0.4.0b0 is absent from the container and the reference's own tests assert
lengths only, so CWT/XWT/WCT parity is "unpinned"; these are the analytic checks
of SURVEY.md Appendix A.6.
"""

import os

import numpy as np
import pandas as pd
import pytest
from scipy.signal import convolve2d

from oracle import glue_spec as gs
from oracle import pycwt_spec as pc

SAMPLE = os.path.join(os.path.dirname(__file__), "golden", "sample_data")
DT = 1 / 12


def load_sample(name):
    df = pd.read_csv(os.path.join(SAMPLE, name), sep=None, parse_dates=[0], index_col=0,
                     engine="python")
    return df.iloc[:, 0].to_numpy(dtype=float)


def test_scales_freqs_coi_closed_forms():
    m = pc.Morlet(6)
    lam = 4 * np.pi / (6 + np.sqrt(38))
    assert np.isclose(m.flambda(), lam) and np.isclose(lam, 1.0330436477492537)
    x = np.zeros(100)
    W, sj, freqs, coi, _, _ = pc.cwt(x + 1.0, DT, 1 / 12, 2 * DT, 63, m)
    assert sj.size == 64 and W.shape == (64, 100)
    assert np.isclose(sj[0], 1 / 6) and np.isclose(1 / freqs[0], lam / 6)
    np.testing.assert_allclose(sj, (1 / 6) * 2 ** (np.arange(64) / 12), rtol=1e-14)
    t = np.arange(100)
    np.testing.assert_allclose(coi, lam / np.sqrt(2) * DT * (50 - np.abs(t - 49.5)))
    # default J for the WCT configuration (probe C.7)
    sj, _ = pc.scales_for(8192, DT, 1 / 8, 2 * DT, -1, m)
    assert sj.size == 97
    sj, _ = pc.scales_for(1333, DT, 1 / 8, 2 * DT, -1, m)
    assert sj.size == 76


def test_sinusoid_peaks_at_its_period():
    n = 1024
    for P in (16.0, 40.0, 100.0):
        t = np.arange(n)
        x = np.sin(2 * np.pi * t / P)
        W, sj, freqs, coi, _, _ = pc.cwt(x, 1.0, 1 / 12, 2.0, 80, pc.Morlet(6))
        period = 1 / freqs
        power = np.abs(W[:, 300:700]) ** 2
        best = np.argmax(power.mean(axis=1))
        assert abs(np.log2(period[best] / P)) < 0.1
        row = power[best]
        assert row.std() / row.mean() < 0.05


def direct_cwt(x, sj, dt, f0=6.0):
    """O(N^2) circular convolution with h_j = IFFT(psi_bar_j) (A.6 item 3)."""
    n0 = x.size
    N = pc.next_pow2(n0)
    xp = np.zeros(N)
    xp[:n0] = x
    k = np.arange(N)
    kk = np.where(k < N // 2, k, k - N)
    w = 2 * np.pi * kk / (N * dt)
    m = pc.Morlet(f0)
    out = np.zeros((sj.size, n0), complex)
    tt = np.arange(N)
    E = np.exp(2j * np.pi * np.outer(kk, tt) / N) / N
    for j, s in enumerate(sj):
        psibar = np.sqrt(s * (2 * np.pi / (N * dt)) * N) * m.psi_ft(s * w)
        h = psibar @ E  # impulse response (IFFT of psi_bar)
        for t in range(n0):
            out[j, t] = np.sum(xp * h[(t - tt) % N])
    return out


@pytest.mark.parametrize("n0", [37, 64, 100])
def test_fft_path_equals_direct_circular_convolution(n0):
    rng = np.random.default_rng(n0)
    x = rng.standard_normal(n0)
    W, sj, _, _, _, _ = pc.cwt(x, DT, 1 / 4, 2 * DT, 12, pc.Morlet(6))
    D = direct_cwt(x, sj, DT)
    assert np.abs(W - D).max() < 1e-12 * np.abs(D).max()


def test_impulse_response_is_analytic_psi_bar():
    N = 256
    x = np.zeros(N)
    x[0] = 1.0
    W, sj, _, _, _, _ = pc.cwt(x, DT, 1 / 4, 2 * DT, 20, pc.Morlet(6))
    k = np.arange(N)
    kk = np.where(k < N // 2, k, k - N)
    w = 2 * np.pi * kk / (N * DT)
    for j, s in enumerate(sj):
        psibar = np.sqrt(s * 2 * np.pi / DT) * np.pi ** -0.25 * np.exp(-0.5 * (s * w - 6) ** 2)
        np.testing.assert_allclose(np.fft.fft(W[j]), psibar, atol=1e-12)


def test_linearity_and_shift_equivariance():
    rng = np.random.default_rng(3)
    a, b = rng.standard_normal((2, 512))
    Wa = pc.cwt(a, DT, 1 / 8, 2 * DT, 40)[0]
    Wb = pc.cwt(b, DT, 1 / 8, 2 * DT, 40)[0]
    Wab = pc.cwt(2 * a - 3 * b, DT, 1 / 8, 2 * DT, 40)[0]
    np.testing.assert_allclose(Wab, 2 * Wa - 3 * Wb, atol=1e-12)
    Ws = pc.cwt(np.roll(a, 17), DT, 1 / 8, 2 * DT, 40)[0]
    np.testing.assert_allclose(Ws, np.roll(Wa, 17, axis=1), atol=1e-12)


def test_ar1_known_answers():
    rng = np.random.default_rng(7)
    e = rng.standard_normal(100_000)
    x = np.zeros_like(e)
    for i in range(1, x.size):
        x[i] = 0.7 * x[i - 1] + e[i]
    g, a, mu2 = pc.ar1(x)
    assert abs(g - 0.7) < 0.01
    infl = gs.standardize_series(load_sample("inflation.csv"))
    g, _, _ = pc.ar1(infl)
    assert abs(g - 0.98883) < 5e-5  # probe C.9 (self-consistency value)
    with pytest.raises(Warning):
        pc.ar1(gs.standardize_series(load_sample("cpi.csv")))


def test_significance_closed_form():
    sj = (1 / 6) * 2 ** (np.arange(10) / 12)
    signif, theor = pc.significance(1.0, DT, sj, 0, 0.5, significance_level=0.95)
    freq = DT / (sj * pc.Morlet(6).flambda())
    pk = 0.75 / (1.25 - np.cos(2 * np.pi * freq))
    np.testing.assert_allclose(signif, pk * 2.995732273553991)


def test_wct_self_coherence_is_one_and_noise_is_low():
    rng = np.random.default_rng(11)
    y = rng.standard_normal(512).cumsum()
    coh, phase, coi, freq, sig = pc.wct(y, y, DT, dj=1 / 8, s0=2 * DT, J=-1, sig=False)
    np.testing.assert_allclose(coh, 1.0, atol=1e-10)
    np.testing.assert_allclose(phase, 0.0, atol=1e-12)
    a, b = rng.standard_normal((2, 512))
    coh, *_ = pc.wct(a, b, DT, dj=1 / 8, s0=2 * DT, J=-1, sig=False)
    assert coh[:8].mean() < 0.5


def test_smooth_identity_and_scale_alignment():
    m = pc.Morlet(6)
    rng = np.random.default_rng(5)
    W = rng.standard_normal((30, 64))
    # s -> 0: time filter is the identity; check with tiny scales and a 1-row window
    # dj = 1.2 -> wsize = 1 -> rect(1) = [1.0]: the scale step is the identity too
    T = m.smooth(W, 1.0, 1.2, np.full(30, 1e-9))
    np.testing.assert_allclose(T, W, atol=1e-12)
    # scale boxcar alignment (probe C.8): impulse at row 15, K=10 reaches rows 11..20
    imp = np.zeros((30, 1))
    imp[15] = 1
    win = pc.rect(10, normalize=True)
    out = convolve2d(imp, win[:, None], "same")[:, 0]
    assert set(np.nonzero(out)[0]) == set(range(11, 21))
    assert np.isclose(out[11], 0.5 / 9) and np.isclose(out[15], 1 / 9)
    win = pc.rect(14, normalize=True)
    out = convolve2d(imp, win[:, None], "same")[:, 0]
    assert set(np.nonzero(out)[0]) == set(range(9, 23))


def test_run_cwt_glue_quirks():
    y = gs.standardize_series(load_sample("inflation.csv"))
    p, period, sig, coi = gs.run_cwt(y, y.size)
    assert p.shape == (85, 1333) and sig.shape == p.shape and coi.shape == (1333,)
    p2, *_ = gs.run_cwt(y, y.size, normalize=False)
    np.testing.assert_array_equal(p, p2)  # quirk B.1
    with pytest.raises(ValueError):
        gs.standardize_series(y, detrend=True, remove_mean=True)


def test_xwt_significance_sigma_reset():
    """pycwt.xwt: std1 = std2 = 1 when the series are normalised (the transformed series
    have unit variance), the raw deviations otherwise.  Invariant to rescaling the inputs
    under normalize=True; scales with sigma1 sigma2 under normalize=False."""
    rng = np.random.default_rng(9)
    e = rng.standard_normal((2, 300))
    y1 = np.zeros(300)
    for t in range(1, 300):
        y1[t] = 0.7 * y1[t - 1] + e[0, t]
    y2 = 0.5 * np.roll(y1, 2) + e[1]
    s = pc.xwt(y1, y2, DT, 1 / 8, 2 * DT)[3]
    s_scaled = pc.xwt(7 * y1, 0.2 * y2, DT, 1 / 8, 2 * DT)[3]
    np.testing.assert_allclose(s_scaled, s, rtol=1e-12)
    raw = pc.xwt(y1, y2, DT, 1 / 8, 2 * DT, normalize=False)[3]
    np.testing.assert_allclose(raw, s * y1.std() * y2.std(), rtol=1e-12)
    freq = pc.xwt(y1, y2, DT, 1 / 8, 2 * DT)[2]
    Pk = (pc.ar1_spectrum(freq * DT, pc.ar1(y1)[0]) * pc.ar1_spectrum(freq * DT, pc.ar1(y2)[0])) ** 0.5
    np.testing.assert_allclose(s, Pk * 2.995732273553991, rtol=1e-12)


@pytest.mark.parametrize("mother", [pc.Paul(4), pc.DOG(2), pc.DOG(3), pc.MexicanHat(), pc.Paul(2)])
def test_other_mothers_known_answers(mother):
    """pycwt's Paul / DOG restated (oracle/pycwt_spec.py): unit energy of psi_hat (the
    Torrence & Compo normalisation, int |psi_hat|^2 dw = 1, which every pycwt mother meets),
    and the Fourier wavelength: the CWT of a sinusoid of period P peaks at the scale whose
    flambda * s is nearest P (A.6.2 for these mothers, within one dj = 1/24 step)."""
    w = np.linspace(-60, 60, 240001)
    e = np.sum(np.abs(mother.psi_ft(w)) ** 2) * (w[1] - w[0])
    np.testing.assert_allclose(e, 1.0, rtol=1e-6)
    n, P = 2048, 64.0
    t = np.arange(n)
    x = np.sin(2 * np.pi * t / P)
    W, sj, freqs, coi, _, _ = pc.cwt(x, 1.0, 1 / 24, 2.0, 24 * 7, mother)
    pw = (np.abs(W[:, n // 4: 3 * n // 4]) ** 2).mean(axis=1)  # T&C's (unrectified) power
    j = int(np.argmax(pw))
    period = 1 / freqs
    assert abs(np.log2(period[j] / P)) <= 1 / 24, (period[j], P)
    np.testing.assert_allclose(coi[1] / coi[0], 3.0)  # (n0/2 - |t - (n0-1)/2|) slope
