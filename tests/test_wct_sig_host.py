"""Host-side pieces of the Monte-Carlo coherence significance vs the
oracle restatement of pycwt wct_significance (oracle/pycwt_spec.py).  CPU only: the
geometry (noise length, COI intervals, maxscale) and the counter -> quantile step.
Parity of the whole Monte Carlo is statistical and lives in test_gpu_wct_sig.py.
"""

import os
import subprocess

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
    ref = pc.significance_from_histogram(wlc, outside, 6, 0.95, quantile="nonempty")
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
    The "nonempty" rule (pycwt's masked counter, the default) interpolates over non-empty bins only: P = ((10, 20) - 0.5) / 20 =
    (0.475, 0.975) on the mid-bin grid (0.05, 0.55), so the 95 % level is
    0.05 + (0.95 - 0.475) / 0.5 * 0.5 = 0.525 -- also what pycwt's masked counter selects
    (quantile="pycwt").  (Parity unpinned: no reference fixture exists for this step.)"""
    from wtmi import transforms
    wlc = np.zeros((2, 10))
    wlc[0, 0] = wlc[0, 5] = 10
    got = transforms.significance_from_histogram(wlc, np.array([True, True]), 1, 0.95)
    assert got[0] == pytest.approx(0.525, abs=1e-15)
    assert np.isnan(got[1])
    for q in ("nonempty", "pycwt"):
        ref = pc.significance_from_histogram(wlc, np.ones((2, 4), dtype=bool), 1, 0.95, quantile=q)
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


# pycwt 0.4.0b0 wavelet.wct_significance, the counter and the quantile step as published
# (the loop body over Monte-Carlo passes replaced by fixed counts; MASK_LINE is the line
# ``wlc.mask = (wlc.data == 0.)`` that follows the Monte-Carlo loop).  Executed as written, in
# this interpreter and under the reference's numpy pin (requirements.txt:25, numpy 1.26.4).
PYCWT_QUANTILE_LINES = """
import json
import numpy as np
J, nbins, maxscale, significance_level = 5, 1000, 4, 0.95
sig95 = np.zeros(J + 1)
wlc = np.ma.zeros([J + 1, nbins])
rng = np.random.default_rng(0)
for s in range(maxscale):
    for t in np.floor(rng.beta(2, 5, 400) * nbins):
        wlc[s, int(t)] += 1
counts = wlc.data.tolist()
MASK_LINE
R2y = (np.arange(nbins) + 0.5) / nbins
try:
    for s in range(maxscale):
        sel = ~wlc[s, :].mask
        P = wlc[s, sel].data.cumsum()
        P = (P - 0.5) / P[-1]
        sig95[s] = np.interp(significance_level, P, R2y[sel])
    print("RESULT ok", np.__version__, json.dumps({"sig95": sig95[:maxscale].tolist(), "wlc": counts}))
except Exception as e:
    print("RESULT", type(e).__name__, np.__version__, sel.shape, R2y[sel].shape, e)
"""
PY39 = "/opt/conda/bin/python3.9"


def _run_quantile_lines(cmd, masked=True):
    src = PYCWT_QUANTILE_LINES.replace("MASK_LINE", "wlc.mask = (wlc.data == 0.)" if masked else "")
    out = subprocess.run(cmd, input=src, capture_output=True, text=True,
                         timeout=120, env={**os.environ, "PYTHONWARNINGS": "ignore"})
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("RESULT")]
    assert line, out.stdout + out.stderr
    print(line[-1][:200])
    return line[-1]


def _interpreters():
    import sys
    yield sys.executable, None
    if os.path.exists(PY39):
        yield PY39, "1.26.4"


@pytest.mark.parametrize("cmd,version", list(_interpreters()))
def test_pycwt_quantile_statements_equal_the_nonempty_rule(cmd, version):
    """pycwt's quantile step as published -- the np.ma counter masked at its empty bins after the
    Monte Carlo, then np.interp over each scale's unmasked bins -- run as written, under this
    interpreter's numpy and under numpy 1.26.4 (the reference's pin, /opt/conda/bin/python3.9
    when present), returns EXACTLY what the oracle's "nonempty" rule, the engine's host rule and
    (tests/test_gpu_wct_sig.py) its device kernel K15 return on the same counters."""
    import json
    from wtmi import transforms
    line = _run_quantile_lines([cmd, "-"], masked=True)
    assert line.startswith("RESULT ok"), line
    if version is not None:
        assert line.split()[2] == version
    res = json.loads(line.split(" ", 3)[3])
    wlc = np.asarray(res["wlc"])
    literal = np.asarray(res["sig95"])
    outside = np.ones((wlc.shape[0], 4), bool)
    ref = pc.significance_from_histogram(wlc, outside, 4, 0.95, quantile="nonempty")
    np.testing.assert_array_equal(literal, ref[:4])
    np.testing.assert_array_equal(pc.significance_from_histogram(wlc, outside, 4, 0.95), ref)
    eng = transforms.significance_from_histogram(wlc, outside.any(axis=1), 4, 0.95)
    np.testing.assert_allclose(eng[:4], literal, rtol=0, atol=1e-15)


def test_unmasked_quantile_reading_raises():
    """Without the mask line the counter's mask is np.ma.nomask, ``~wlc[s, :].mask`` is the
    scalar True, a 0-d boolean index adds an axis (R2y[sel] has shape (1, nbins)) and np.interp
    raises ValueError('object too deep for desired array') under numpy 1.26.4 and 2.x.  That
    reading (r05's default) is kept only as the explicit quantile="unmasked" option."""
    for cmd, version in _interpreters():
        here = _run_quantile_lines([cmd, "-"], masked=False)
        assert here.startswith("RESULT ValueError") and "object too deep for desired array" in here
        assert "(1, 1000)" in here
        if version is not None:
            assert here.startswith(f"RESULT ValueError {version}"), here
    wlc = np.zeros((3, 1000))
    wlc[:2, 100:900] = 1
    with pytest.raises(ValueError, match="object too deep"):
        pc.significance_from_histogram(wlc, np.ones((3, 4), bool), 2, 0.95, quantile="unmasked")
    with pytest.raises(ValueError, match="object too deep"):
        pc.wct_significance(0.5, 0.3, 1.0, 0.5, 2.0, 4, mc_count=2, rng=np.random.default_rng(0),
                            quantile="unmasked")
    # the default (masked) reading returns levels on the same inputs
    got = pc.wct_significance(0.5, 0.3, 1.0, 0.5, 2.0, 4, mc_count=2, rng=np.random.default_rng(0))
    assert np.isfinite(got[:2]).all()
    # maxscale == 0: the loop never runs, pycwt returns its initial levels
    got = pc.significance_from_histogram(wlc, np.zeros((3, 4), bool), 0, 0.95, quantile="unmasked")
    np.testing.assert_array_equal(got, np.zeros(3))


def test_engine_quantile_default_is_pycwt_masked_and_unmasked_raises_before_gpu_work():
    from wtmi import transforms
    assert transforms.SIG_QUANTILE == "pycwt"
    assert transforms.QUANTILE_MODES == ("pycwt", "nonempty", "unmasked")
    with pytest.raises(ValueError, match="object too deep for desired array"):
        transforms.wct_significance(0.7, 0.5, 1 / 12, 1 / 8, 2 / 12, 56, cache=False,
                                    quantile="unmasked")
    with pytest.raises(ValueError, match="quantile must be one of"):
        transforms.wct_significance(0.7, 0.5, 1 / 12, 1 / 8, 2 / 12, 56, quantile="median")
    # g == 0 fails first (pycwt's rednoise runs in the Monte-Carlo loop, before the quantile)
    with pytest.raises(AttributeError, match="randn"):
        transforms.wct_significance(0.0, 0.5, 1 / 12, 1 / 8, 2 / 12, 56, cache=False)


def test_pycwt_cache_name_is_nan_above_a_quarter():
    """pycwt's cache file name rounds arctanh(4 al): NaN for |al| > 0.25, so every such pair of
    series shares one name per (dj, s0 / dt, J, wavelet).  The engine keys on the exact al
    and does not reproduce the sharing, which would hand one series' levels to another."""
    a = pc.pycwt_cache_name(0.98, 0.6, 1 / 12, 1 / 8, 2 / 12, 75)
    b = pc.pycwt_cache_name(0.3, 0.9, 1 / 12, 1 / 8, 2 / 12, 75)
    assert a == b == "wct_sig_nan_nan_0.12500_2.00000_75_morlet"
    assert pc.pycwt_cache_name(0.1, -0.2, 1 / 12, 1 / 8, 2 / 12, 75).startswith("wct_sig_0.00000_1.50000_")
