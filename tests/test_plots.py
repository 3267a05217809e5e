"""The drop-in plot functions draw what the reference's draw (CPU, Agg).

``tests/golden/plot_signatures.json`` holds the figure signatures (contour levels and
path/vertex sums, COI polygon vertices, quiver arrows, lines, titles, ticks, legends)
of the reference's OWN plot functions run on the seeded inputs of
``figsig.plot_inputs`` (``scripts/make_plot_golden.py``, build container).  Here the
repo's functions draw the same inputs and must give the same signature.  The one
numeric call inside a plot function (``dwt.plot_components`` reconstructs each
component with an inverse DWT on the GPU) is served by the oracle's PyWavelets
restatement, as in the generator, so that only the drawing is compared on CPU; the
GPU-backed end-to-end rendering is ``tests/test_gpu_plots.py``.
"""

import json
import os

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import pytest  # noqa: E402

import figsig  # noqa: E402
from conftest import GOLDEN  # noqa: E402

with open(os.path.join(GOLDEN, "plot_signatures.json")) as _fh:
    GOLD = json.load(_fh)["cases"]

P = figsig.PLOT_PROPS
CWT_PROPS = {k: P[k] for k in ("cmap", "sig_colors", "sig_linewidths", "coi_color", "coi_alpha",
                               "coi_hatch")}


@pytest.fixture(scope="module")
def inp():
    return figsig.plot_inputs()


@pytest.fixture
def oracle_waverec(monkeypatch, db4):
    """transforms.waverec_variants on the oracle (CPU), for the drawing-only comparison."""
    from oracle import dwt_spec
    from wtmi import transforms

    def fake(coeffs, wavelet, masks):
        out = []
        for m in masks:
            kept = [c if (m >> k) & 1 else np.zeros_like(c) for k, c in enumerate(coeffs)]
            out.append(dwt_spec.waverec(kept, db4["rec_lo"], db4["rec_hi"]))
        return out
    monkeypatch.setattr(transforms, "waverec_variants", fake)


def _axes_case(fn):
    fig, ax = plt.subplots(1, 1, figsize=(10, 5), dpi=72)
    fn(ax)
    sig = figsig.figure_signature(fig)
    plt.close(fig)
    return sig


def test_plot_cwt(inp):
    from src import cwt
    d, r = inp["cwt"]
    figsig.compare(_axes_case(lambda ax: cwt.plot_cwt(ax, d, r, **CWT_PROPS)), GOLD["cwt.plot_cwt"])
    figsig.compare(_axes_case(lambda ax: cwt.plot_cwt(ax, d, r, include_significance=False,
                                                      **CWT_PROPS)), GOLD["cwt.plot_cwt[no_sig]"])


def test_plot_xwt(inp):
    from src import xwt
    d, r = inp["xwt"]
    figsig.compare(_axes_case(lambda ax: xwt.plot_xwt(ax, d, r, **P)), GOLD["xwt.plot_xwt"])
    figsig.compare(_axes_case(lambda ax: xwt.plot_phase_difference(
        ax, d.t_values, r.period, r.phase_diff_u, r.phase_diff_v, **P)),
        GOLD["xwt.plot_phase_difference"])


def test_plot_wct(inp):
    from src import wct
    d, r = inp["wct"]
    figsig.compare(_axes_case(lambda ax: wct.plot_wct(ax, d, r, **P)), GOLD["wct.plot_wct"])
    figsig.compare(_axes_case(lambda ax: wct.plot_wct(ax, d, r, include_cone_of_influence=False,
                                                      include_phase_difference=False, **P)),
                   GOLD["wct.plot_wct[no_coi_no_arrows]"])


def test_wavelet_helpers_plots(inp):
    from src.utils import wavelet_helpers as wh
    r = inp["cwt"][1]
    figsig.compare(_axes_case(lambda ax: wh.plot_cone_of_influence(
        ax, r.coi, inp["t_years"], figsig.LEVELS, r.period, 1 / 12, tranform_type="cwt", **P)),
        GOLD["wavelet_helpers.plot_cone_of_influence[cwt]"])
    figsig.compare(_axes_case(lambda ax: wh.plot_signficance_levels(
        ax, r.significance_levels, inp["t_years"], r.period, **P)),
        GOLD["wavelet_helpers.plot_signficance_levels"])


def test_dwt_plot_components(inp, oracle_waverec):
    from src import dwt
    fig = dwt.plot_components("series", inp["coeffs"], inp["t_years"], 5, "db4", figsize=(8, 12))
    figsig.compare(figsig.figure_signature(fig), GOLD["dwt.plot_components"], rtol=1e-7)
    plt.close("all")


@pytest.mark.parametrize("ascending", [False, True])
@pytest.mark.parametrize("module", ["dwt", "modwt"])
def test_plot_smoothing(inp, module, ascending):
    import importlib
    mod = importlib.import_module(f"src.{module}")
    kw = {"figsize": (8, 12), "sharex": True} if module == "dwt" else {"figsize": (8, 12)}
    fig = mod.plot_smoothing(inp["smooth"], inp["t_years"], inp["y"], ascending=ascending, **kw)
    figsig.compare(figsig.figure_signature(fig), GOLD[f"{module}.plot_smoothing[ascending={ascending}]"])
    plt.close("all")
