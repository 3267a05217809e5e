"""Every drop-in plot function, end to end on engine results (GPU, Agg backend).

The flows follow the app (src/wavelet_plots.py:126-151 CWT, :371-393 XWT, :500-526 WCT,
:228-290 DWT smoothing; src/utils/plot_helpers.py:47-78 components): transform with the
drop-in modules on the GPU, then draw with the drop-in plot functions and render to PNG.
The drawing itself is pinned against the reference's plot functions by
tests/test_plots.py; this test shows the engine's outputs feed them unchanged.
"""

import io
import os

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import pytest  # noqa: E402

import figsig  # noqa: E402

pytestmark = pytest.mark.gpu
SAMPLE = os.path.join(os.path.dirname(__file__), "golden", "sample_data")
P = figsig.PLOT_PROPS
CWT_PROPS = {k: P[k] for k in ("cmap", "sig_colors", "sig_linewidths", "coi_color", "coi_alpha",
                               "coi_hatch")}


def _series(name):
    df = pd.read_csv(os.path.join(SAMPLE, name), parse_dates=[0], index_col=0)
    return df.index.to_numpy(), df.iloc[:, 0].to_numpy(dtype=float)


def _render(fig):
    buf = io.BytesIO()
    fig.savefig(buf, format="png")
    plt.close("all")
    assert buf.tell() > 10_000
    return buf


def test_plot_cwt_on_inflation():
    from src import cwt
    from src.utils.wavelet_helpers import standardize_series
    t, y = _series("inflation.csv")
    data = cwt.DataForCWT(t, standardize_series(y), cwt.MOTHER, cwt.DT, cwt.DJ, cwt.S0, cwt.LEVELS)
    res = cwt.run_cwt(data, standardize=True, calculate_significance=True, significance_level=0.95)
    fig, ax = plt.subplots(1, 1, figsize=(20, 10), dpi=72)
    cwt.plot_cwt(ax, data, res, include_significance=True, **CWT_PROPS)
    sig = figsig.axes_signature(ax)
    assert [c["type"] for c in sig["collections"]] == ["QuadContourSet", "QuadContourSet"]
    assert sig["collections"][0]["filled"] and sig["collections"][1]["levels"] == [-99.0, 1.0]
    assert len(sig["patches"]) == 1 and sig["ylim"][0] > sig["ylim"][1]  # inverted
    _render(fig)


def _pair():
    t1, y1 = _series("inflation.csv")
    t2, y2 = _series("cpi.csv")
    common = np.intersect1d(t1, t2)
    a = y1[np.isin(t1, common)]
    b = np.diff(np.log(y2[np.isin(t2, common)]), prepend=np.nan)[1:]
    return a[1:], b


def test_plot_xwt_and_wct_on_sample_pair(monkeypatch):
    from src import wct, xwt
    from src.utils.wavelet_helpers import standardize_series
    y1, y2 = _pair()
    y1 = standardize_series(y1, detrend=False, remove_mean=True)
    y2 = standardize_series(y2, detrend=False, remove_mean=True)
    dx = xwt.DataForXWT(y1, y2, xwt.MOTHER_DICT[xwt.MOTHER], xwt.DT, xwt.DJ, xwt.S0, xwt.LEVELS)
    rx = xwt.run_xwt(dx)
    fig, ax = plt.subplots(1, 1, figsize=(10, 8))
    xwt.plot_xwt(ax, dx, rx, include_significance=True, include_cone_of_influence=True,
                 include_phase_difference=True, **P)
    types = [c["type"] for c in figsig.axes_signature(ax)["collections"]]
    assert types == ["QuadContourSet", "QuadContourSet", "Quiver"]
    _render(fig)

    dw = wct.DataForWCT(y1, y2, wct.MOTHER_DICT[wct.MOTHER], wct.DT, wct.DJ, wct.S0, wct.LEVELS)
    rw = wct.run_wct(dw, calculate_signficance=True, significance_level=0.95)
    fig, ax = plt.subplots(1, 1, figsize=(10, 8))
    wct.plot_wct(ax, dw, rw, include_significance=True, include_cone_of_influence=True,
                 include_phase_difference=True, **P)
    sig = figsig.axes_signature(ax)
    assert [c["type"] for c in sig["collections"]] == ["QuadContourSet", "QuadContourSet", "Quiver"]
    assert sig["collections"][0]["levels"] == [float(v) for v in wct.WCT_LEVELS]
    _render(fig)


def test_plot_dwt_components_and_smoothing():
    from src import dwt, modwt
    t, y = _series("inflation.csv")
    data = dwt.DataForDWT(y, dwt.MOTHER)
    res = dwt.run_dwt(data)
    fig = dwt.plot_components(label="inflation", coeffs=res.coeffs, time=t, levels=res.levels,
                              wavelet=dwt.MOTHER, figsize=(15, 20), sharex=True)
    assert len(fig.axes) == res.levels + 1
    _render(fig)
    res.smooth_signal(y_values=data.y_values, mother_wavelet=data.mother_wavelet)
    fig = dwt.plot_smoothing(res.smoothed_signal_dict, t, data.y_values, ascending=True,
                             figsize=(15, 20), sharex=True)
    assert len(fig.axes) == res.levels
    _render(fig)
    w = modwt.modwt(y[: 1024], "db4", 5)
    sm = modwt.smooth_signal(w, "db4", 5)
    fig = modwt.plot_smoothing(sm, t[:1024], y[:1024], figsize=(15, 20))
    assert len(fig.axes) == 5
    _render(fig)
