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


def test_oracle_rednoise_is_ar1():
    x = pc.rednoise(200000, 0.7, 1.0, np.random.default_rng(1))
    r1 = np.corrcoef(x[:-1], x[1:])[0, 1]
    assert abs(r1 - 0.7) < 0.01
    assert abs(x.var() - 1 / (1 - 0.49)) < 0.05
