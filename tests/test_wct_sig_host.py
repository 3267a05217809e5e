"""Host-side pieces of the Monte-Carlo coherence significance vs the
oracle restatement of pycwt wct_significance (oracle/pycwt_spec.py).  CPU only: the
geometry (noise length, COI intervals, maxscale) and the counter -> quantile step.
Parity of the whole Monte Carlo is statistical and lives in test_gpu_wct_sig.py.
"""

import numpy as np
import pytest

from oracle import pycwt_spec as pc


@pytest.mark.parametrize("dt,dj,s0,J", [(1.0, 0.25, 2.0, 8), (1 / 12, 1 / 8, 2 / 12, 75),
                                        (1 / 12, 1 / 12, 2 / 12, 100), (1.0, 0.5, 1.0, 3)])
def test_geometry_matches_oracle(dt, dj, s0, J):
    from wtmi import transforms
    N, sj, t_lo, t_hi, anyout, maxscale = transforms.wct_sig_geometry(dt, dj, s0, J)
    rN, rsj, outside, rmax = pc.wct_sig_geometry(dt, dj, s0, J)
    assert N == rN and maxscale == rmax
    np.testing.assert_allclose(sj, rsj, rtol=1e-15)
    np.testing.assert_array_equal(anyout, outside.any(axis=1))
    for s in range(J + 1):
        mask = np.zeros(N, dtype=bool)
        mask[t_lo[s]:t_hi[s]] = True
        np.testing.assert_array_equal(mask, outside[s])  # the outside-COI set is one interval


def test_quantile_step_matches_oracle():
    from wtmi import transforms
    rng = np.random.default_rng(5)
    J1, nbins = 9, 1000
    wlc = np.zeros((J1, nbins))
    for s in range(J1):
        # sparse, skewed counters like a real coherence distribution, with empty bins
        idx = np.clip((rng.beta(2, 3, size=3000) * nbins).astype(int), 0, nbins - 1)
        np.add.at(wlc[s], idx, 1)
    anyout = np.array([True] * 7 + [False] * 2)
    outside = np.repeat(anyout[:, None], 4, axis=1)
    got = transforms.significance_from_histogram(wlc, anyout, 6, 0.95)
    ref = pc.significance_from_histogram(wlc, outside, 6, 0.95)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(ref))
    np.testing.assert_allclose(got[~np.isnan(got)], ref[~np.isnan(ref)], rtol=0, atol=1e-15)
    assert np.isnan(got[6]) and got[7] == 0 and got[8] == 0  # s = maxscale stays NaN


def test_oracle_counter_clamps_and_counts():
    R2 = np.array([[0.0, 0.0004, 0.9999, 1.0, 0.5]])
    outside = np.ones_like(R2, dtype=bool)
    wlc = pc.coherence_histogram(np.vstack([R2, R2]), np.vstack([outside, outside]), 1)
    assert wlc[0].sum() == 5 and wlc[0, 0] == 2 and wlc[0, 999] == 2 and wlc[0, 500] == 1
    assert wlc[1].sum() == 0  # s = maxscale is not counted


def test_oracle_rednoise_modes():
    """noise="red": AR(1) with lag-1 correlation g and variance 1/(1-g^2).  noise="pycwt"
    (the default, pycwt's published rednoise taken literally): lfilter along the length-1
    axis of randn(N + tau, 1) is the identity, so the draws are white -- exactly the normals
    after the tau burn-in of the same generator state -- and g == 0 raises AttributeError
    (pycwt's np.randn)."""
    x = pc.rednoise(200000, 0.7, 1.0, np.random.default_rng(1), noise="red")
    r1 = np.corrcoef(x[:-1], x[1:])[0, 1]
    assert abs(r1 - 0.7) < 0.01
    assert abs(x.var() - 1 / (1 - 0.49)) < 0.05
    w = pc.rednoise(200000, 0.7, 1.0, np.random.default_rng(1))
    assert abs(np.corrcoef(w[:-1], w[1:])[0, 1]) < 0.01
    assert abs(w.var() - 1.0) < 0.02
    tau = int(np.ceil(-2 / np.log(0.7)))
    e = np.random.default_rng(1).standard_normal((200000 + tau, 1)).flatten()
    np.testing.assert_array_equal(w, e[tau:])
    # the red series is the AR(1) filter of those same normals
    np.testing.assert_allclose(x[1:] - 0.7 * x[:-1], e[tau + 1:], atol=1e-9)
    with pytest.raises(AttributeError):
        pc.rednoise(100, 0.0, 1.0, np.random.default_rng(1))
    assert pc.rednoise(100, 0.0, 1.0, np.random.default_rng(1), noise="red").shape == (100,)


def test_quantile_known_answer_with_empty_bins_at_the_crossing():
    """Hand-built counter: 10 counts in bin 0, bins 1-4 EMPTY, 10 counts in bin 5 (nbins 10).
    The selection rule interpolates over non-empty bins only: P = ((10, 20) - 0.5) / 20 =
    (0.475, 0.975) on the mid-bin grid (0.05, 0.55), so the 95 % level is
    0.05 + (0.95 - 0.475) / 0.5 * 0.5 = 0.525.  (Parity unpinned: the rule restates pycwt's
    masked-array selection; no reference fixture exists for this step.)"""
    from wtmi import transforms
    wlc = np.zeros((2, 10))
    wlc[0, 0] = wlc[0, 5] = 10
    got = transforms.significance_from_histogram(wlc, np.array([True, True]), 1, 0.95)
    assert got[0] == pytest.approx(0.525, abs=1e-15)
    assert np.isnan(got[1])
    ref = pc.significance_from_histogram(wlc, np.ones((2, 4), dtype=bool), 1, 0.95)
    assert ref[0] == pytest.approx(0.525, abs=1e-15)


def test_significance_cache_persists_on_disk(tmp_path, monkeypatch):
    """wct_significance(cache=True) keeps results in memory AND on disk (pycwt's cache=True,
    src/wct.py:117): a fresh process (empty memory cache) reads the stored levels back."""
    from wtmi import transforms
    monkeypatch.setenv("WTMI_CACHE_DIR", str(tmp_path))
    key = ("wct_significance", 1, 0.7, 0.5, 1 / 12, 0.125, 2 / 12, 40, 0.95, 6.0, 300, 1000, None)
    assert transforms.sig_cache_load(key) is None
    sig = np.linspace(0.1, 0.9, 41)
    sig[-3:] = np.nan
    transforms.sig_cache_store(key, sig)
    monkeypatch.setattr(transforms, "_sig_cache", {})
    back = transforms.sig_cache_load(key)
    np.testing.assert_array_equal(back, sig)
    files = list((tmp_path / "wct_sig").iterdir())
    assert len(files) == 1 and files[0].suffix == ".npy"
    # an unreadable entry is recomputed, never trusted
    files[0].write_bytes(b"garbage")
    monkeypatch.setattr(transforms, "_sig_cache", {})
    assert transforms.sig_cache_load(key) is None
