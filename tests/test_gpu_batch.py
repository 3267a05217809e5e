"""The batch API (run_cwt_batch / run_xwt_batch / run_dwt_batch and the batched
src.utils.transform_helpers dict builders) against the one-series functions (GPU).

A batch groups equal-length series into one launch; each series' result must be the
one run_cwt / run_xwt / run_dwt gives it alone -- same kernel per series, so equal to
fp32 rounding of the same operations (checked at 1e-6 relative).  The dict builders are
run with a stand-in ``constants`` package carrying the app's transform constants
(constants/results_configs.py:27-58, constants/ids.py DATE).
"""

import sys
import types

import numpy as np
import pandas as pd
import pytest

from gpu_helpers import red_series

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=1e-6):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape
    assert np.abs(a - b).max() <= rtol * max(np.abs(b).max(), 1e-30)


def _series(seed, n):
    return red_series(np.random.default_rng(seed), n).astype(np.float64)


def test_run_cwt_batch_matches_run_cwt():
    from src import cwt
    lens = [300, 517, 300, 1024, 517, 300]
    data = [cwt.DataForCWT(np.arange(n).astype("datetime64[M]"), _series(i, n), cwt.MOTHER,
                           cwt.DT, cwt.DJ, cwt.S0, cwt.LEVELS) for i, n in enumerate(lens)]
    for kw in ({}, {"standardize": True}, {"calculate_significance": False}):
        batch = cwt.run_cwt_batch(data, **kw)
        for d, r in zip(data, batch):
            one = cwt.run_cwt(d, **kw)
            _close(r.power, one.power)
            _close(r.period, one.period)
            _close(r.coi, one.coi)
            if one.significance_levels is None:
                assert r.significance_levels is None
            else:
                _close(r.significance_levels, one.significance_levels)
    with pytest.raises(TypeError):
        cwt.run_cwt_batch(data, standardize=True, detrendd=False)


def test_run_xwt_batch_matches_run_xwt():
    from src import xwt
    pairs = [(_series(10 + i, n), _series(20 + i, n)) for i, n in enumerate([400, 400, 640, 400])]
    data = [xwt.DataForXWT(a, b, xwt.MOTHER_DICT["morlet"], xwt.DT, xwt.DJ, xwt.S0, xwt.LEVELS)
            for a, b in pairs]
    for norm in (True, False):
        batch = xwt.run_xwt_batch(data, normalize=norm)
        for d, r in zip(data, batch):
            one = xwt.run_xwt_batch([d], normalize=norm)[0]
            if norm:
                one_dropin = xwt.run_xwt(d)
                _close(r.power, one_dropin.power)
            for f in ("power", "period", "significance_levels", "coi", "phase_diff_u", "phase_diff_v"):
                _close(getattr(r, f), getattr(one, f))


def test_run_dwt_batch_matches_run_dwt():
    from src import dwt
    lens = [101, 256, 101, 1333]
    data = [dwt.DataForDWT(_series(30 + i, n), dwt.MOTHER, None if i % 2 else 3)
            for i, n in enumerate(lens)]
    for d, r in zip(data, dwt.run_dwt_batch(data)):
        one = dwt.run_dwt(d)
        assert r.levels == one.levels and len(r.coeffs) == len(one.coeffs)
        for c, c1 in zip(r.coeffs, one.coeffs):
            _close(c, c1)


@pytest.fixture
def app_constants(monkeypatch):
    from src import cwt, dwt, xwt
    ids = types.SimpleNamespace(DATE="date")
    rc = types.SimpleNamespace(XWT_MOTHER="morlet", XWT_MOTHER_DICT=xwt.MOTHER_DICT, XWT_DT=1 / 12,
                               XWT_DJ=1 / 8, XWT_S0=2 / 12, LEVELS=cwt.LEVELS,
                               DWT_MOTHER_WAVELET=dwt.MOTHER)
    pkg = types.ModuleType("constants")
    pkg.ids, pkg.results_configs = ids, rc
    monkeypatch.setitem(sys.modules, "constants", pkg)
    monkeypatch.setitem(sys.modules, "constants.ids", ids)
    monkeypatch.setitem(sys.modules, "constants.results_configs", rc)
    return rc


def test_transform_helpers_dicts(app_constants):
    from src import cwt, dwt, xwt
    from src.utils import transform_helpers as th
    from src.utils.wavelet_helpers import standardize_series
    n = 480
    df = pd.DataFrame({"date": pd.date_range("1980-01-01", periods=n, freq="MS"),
                       "a": _series(1, n), "b": _series(2, n), "c": _series(3, n)})
    df.loc[:5, "c"] = np.nan  # a shorter series: its own length group
    measures = ["a", "b", "c"]
    cd = th.create_cwt_dict(df, measures, mother_wavelet=cwt.MOTHER, delta_t=cwt.DT,
                            delta_j=cwt.DJ, initial_scale=cwt.S0, levels=cwt.LEVELS)
    assert cd["c"].y_values.size == n - 6
    res = th.create_cwt_results_dict(cd, measures)
    for m in measures:
        one = cwt.run_cwt(cd[m])
        _close(res[m].power, one.power)
        _close(res[m].significance_levels, one.significance_levels)
    xd = th.create_xwt_dict(df, [("a", "b"), ("b", "c")], detrend=False, remove_mean=True)
    assert xd[("a", "b")].y1_values.size == n - 6  # dropna over every column, as the reference
    np.testing.assert_allclose(xd[("a", "b")].y1_values,
                               standardize_series(df.dropna()["a"].to_numpy(), detrend=False,
                                                  remove_mean=True))
    xr = th.create_xwt_results_dict(xd, [("a", "b"), ("b", "c")])
    for k in xd:
        _close(xr[k].power, xwt.run_xwt(xd[k]).power)
    dd = th.create_dwt_dict(df.dropna(), measures)
    assert all(d.levels == 6 for d in dd.values())  # dwt_max_level(474, 8)
    dr = th.create_dwt_results_dict(dd, measures)
    rr = th.create_dwt_regression_dict(dd, measures)
    for m in measures:
        one = dwt.run_dwt(dd[m])
        assert dr[m].levels == rr[m].levels == 6
        for c, c1, c2 in zip(dr[m].coeffs, rr[m].coeffs, one.coeffs):
            _close(c, c1)
            _close(c1, c2)
